"""CPU: the host code under AddressSanitizer + UndefinedBehaviorSanitizer.

tools/asan/build.sh builds the ONNX wire parser (csrc/ore_onnx.cpp, the reference's
ModelProto::parse_from_bytes + get_stored_tensor decode, main.rs:30 / utils.rs:113-185) host-only with
-fsanitize=address,undefined -fno-sanitize-recover=all into tools/asan/build/parse_fuzz; this test runs
it on mnist-8.onnx, on every wire-type mismatch case of test_abi.py (each must be rejected) and on
3000 random mutations / truncations (each parses or is rejected).  Any sanitizer finding aborts the
driver, so exit 0 is a clean run.  The planner (ore_model.cpp) needs a HIP device; its host-ASan
driver (tools/asan/model_fuzz.cpp) runs on the GPU box (tests/test_sanitize_gpu.py)."""
import os
import subprocess

import pytest

from test_abi import _mini_model

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _mismatch_cases():
    from ore import onnx_wire as w
    good = w._vi(1, 3) + w._vi(2, 1)
    return [
        _mini_model(node_fields=w._vi(1, 5) + w._ld(2, b"y") + w._ld(4, b"Relu")),
        _mini_model(node_fields=w._ld(1, b"x") + w._ld(2, b"y") + w._key(4, 5) + b"Relu"),
        _mini_model(attr=w._ld(1, b"a") + w._vi(20, 3) + w._vi(4, 7)),
        _mini_model(attr=w._vi(1, 9) + w._vi(20, 2) + w._vi(3, 1)),
        _mini_model(attr=w._ld(1, b"a") + w._vi(20, 1) + w._vi(2, 1)),
        _mini_model(attr=w._ld(1, b"a") + w._vi(20, 1) + w._key(2, 1) + b"\0" * 8),
        _mini_model(tensor_fields=good + w._ld(9, b"\0" * 12) + w._vi(8, 1)),
        _mini_model(tensor_fields=good + w._vi(4, 1) + w._ld(8, b"b")),
        _mini_model(tensor_fields=good + w._vi(9, 1) + w._ld(8, b"b")),
        _mini_model(tensor_fields=good + w._ld(4, b"\0" * 10) + w._ld(8, b"b")),
        _mini_model(tensor_fields=w._vi(1, 3) + w._ld(2, b"\1") + w._ld(8, b"b")),
        w._vi(1, 3) + w._vi(7, 1),
    ]


@pytest.fixture(scope="module")
def parse_fuzz():
    r = subprocess.run(["bash", os.path.join(REPO, "tools", "asan", "build.sh"), "parse"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout.strip().splitlines()[-1]


def test_parser_asan_ubsan_clean(parse_fuzz, tmp_path):
    cases = []
    for i, b in enumerate(_mismatch_cases()):
        p = tmp_path / f"case{i}.onnx"
        p.write_bytes(b)
        cases.append(str(p))
    mnist = os.path.join(HERE, "golden", "mnist-8.onnx")
    trunc = tmp_path / "trunc.onnx"
    trunc.write_bytes(open(mnist, "rb").read()[:13000])
    cases.append(str(trunc))
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([parse_fuzz, mnist, "3000"] + cases, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "no sanitizer report" in r.stdout and f"{len(cases)} rejected cases" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr


def test_squeezenet_parses_under_asan(parse_fuzz, tmp_path):
    from ore import squeezenet
    p = tmp_path / "sq.onnx"
    p.write_bytes(squeezenet.build(224))
    r = subprocess.run([parse_fuzz, str(p), "200"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
