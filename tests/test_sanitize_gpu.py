"""The planner's host code under AddressSanitizer + UndefinedBehaviorSanitizer, on the GPU box
(VERDICT r3 item 9).  tools/asan/build.sh model builds every csrc/ file with the sanitizers on the host
side only (-Xarch_host -fsanitize=address,undefined; GPU ASan / xnack are not available on this pool)
and links tools/asan/model_fuzz.cpp: MNIST-8 and SqueezeNet-1.0 load, plan under five fusion settings
and run (f32 at batch 1 / 4 / 300, no-Winograd, f16), then 300 byte-mutated MNIST models are loaded
(parse, shape rules, planner, weight packing; never run) and destroyed.  A sanitizer report aborts it.
The driver is not part of the product build (__graft_entry__.build()) and does not travel with the
tree (.gpurunignore): this test builds it where it runs (about 45 s over 16 compile jobs) unless a
fresh one is already there."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
BIN = os.path.join(REPO, "tools", "asan", "build", "model_fuzz")


def _fresh():
    """The driver exists and is newer than every source it is built from."""
    if not os.path.exists(BIN):
        return False
    t = os.path.getmtime(BIN)
    srcs = [os.path.join(REPO, "tools", "asan", "model_fuzz.cpp"), os.path.join(REPO, "include", "ore.h")]
    csrc = os.path.join(REPO, "onnx-rusty-inference-engine_amd", "csrc")
    srcs += [os.path.join(csrc, f) for f in os.listdir(csrc)]
    return all(os.path.getmtime(s) <= t for s in srcs)


def test_planner_asan_ubsan_clean(tmp_path):
    from ore import squeezenet
    if not _fresh():
        b = subprocess.run(["bash", os.path.join(REPO, "tools", "asan", "build.sh"), "model"], capture_output=True,
                           text=True, timeout=600)
        assert b.returncode == 0, (b.stdout + b.stderr)[-4000:]
    assert os.path.exists(BIN), BIN
    sq = tmp_path / "sq.onnx"
    sq.write_bytes(squeezenet.build(224))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([BIN, os.path.join(HERE, "golden", "mnist-8.onnx"), str(sq), "300"], capture_output=True,
                       text=True, timeout=280, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "no sanitizer report" in r.stdout, r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
