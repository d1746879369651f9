"""Config 4 (BASELINE.json configs[3]: SqueezeNet-1.0 at a global batch of 2048 split over 1 / 2 / 4 / 8
GPUs) and the exact plan bench.py times, on the one GPU of the test box.

* Per-GPU batches of config 4's strong-scaling points -- 2048 (N = 1), 1024 (N = 2), 512 (N = 4) -- on
  the default f32 plan: the model loads at that max_batch (run_batch = the images one pass of the graph
  covers; past it ore_model_run runs the batch in image chunks, because fire4's concat alone is 3 MB per
  image), autotunes on the batch, and every image's output equals the same image run alone, bit for bit
  (images are independent: convolution_op.rs:480 is per image); the two fixture images placed at the
  ends of the batch match the oracle within 1e-5 (SURVEY §8(e) correctness check).
* bench.py's headline plan -- max_batch 256, autotuned on a 256-image batch, two streams -- on the eight
  images of tests/golden/squeezenet_synth8_*.npz, against the oracle AND against the float64 executor
  (tests/golden/f64_ref.py) of the same graph; the margins are printed (DESIGN.md section 5 records
  them).  The tolerance, per image i (DESIGN.md section 5 for the measurements behind it):
    |gpu - oracle| <= 1e-5 + |oracle - f64|   the north_star bound plus the reference's own f32
                                              rounding, which on these peaky synthetic outputs (top
                                              probability 0.62-0.95) reaches 8.7e-6 by itself;
    |gpu - f64| <= 1e-5 (Winograd, the default plan) / 2e-5 (winograd=False, the reference's k order
                                              on 9C-long f32 chains); same argmax.
* the same plan on bench.py's own model, the zoo-calibrated SqueezeNet, on the 16 images of
  tests/golden/squeezenet_calib16_*.npz (zoo image + 15 U(-50,50) draws): the plain north_star bound
  max |gpu - oracle| <= 1e-5 per image, same argmax (the oracle is within 1.4e-6 of float64 there, so a
  ~1e-5 regression cannot hide in rounding).
* bench.py's collective path at world size 1 (--dist): a one-rank RCCL communicator and the device-tensor
  all-gather, launched by torch.distributed.run.
* bench.py's N > 1 branch (global-batch slicing, the per-step all-gather, the max over ranks, the
  gathered max-abs sample) as two processes on this GPU, over gloo (--dist-backend gloo: the rows staged
  through host memory; the RCCL leg needs one GPU per rank).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLD = os.path.join(HERE, "golden")


def _batch(B, seed):
    import torch
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.rand((B, 3, 224, 224), generator=g, device="cuda") * 100.0 - 50.0


@pytest.mark.parametrize("B", [2048, 1024, 512])
def test_config4_per_gpu_batch(gpu_ctx, B):
    import torch
    import ore
    from ore import squeezenet
    from golden.make_golden import squeezenet_inputs
    m = ore.Model(gpu_ctx, squeezenet.build(224), max_batch=B)
    assert 1 <= m.run_batch <= B
    if B == 2048:
        assert m.run_batch < B  # the chunked path runs (fire4's concat passes 2 GiB at 2048 images)
    fx = torch.from_numpy(squeezenet_inputs()).cuda()
    x = _batch(B, 7)
    x[0] = fx[0]
    x[B - 1] = fx[1]
    out = torch.empty((B, m.output_elems), device="cuda")
    m.set_streams(2)
    out.fill_(float("nan"))
    m.autotune(x, out)
    torch.cuda.synchronize()
    y_tuned = out.cpu().numpy()  # autotune leaves every image's output, chunked batches included
    m.run_into(x, out)
    torch.cuda.synchronize()
    y = out.cpu().numpy()
    assert np.isfinite(y).all()
    np.testing.assert_array_equal(y_tuned, y)
    np.testing.assert_allclose(y.sum(axis=1), 1.0, atol=1e-4)
    ref = np.load(os.path.join(GOLD, "squeezenet_synth_oracle.npz"))["output"]
    err = float(np.abs(y[[0, B - 1]] - ref).max())
    assert err <= 1e-5, err
    assert np.array_equal(y[[0, B - 1]].argmax(1), ref.argmax(1))
    one = torch.empty((1, m.output_elems), device="cuda")
    for i in (0, 1, B // 2, B - 1):  # each image alone through the same model: the same bits
        m.run_into(x[i:i + 1].contiguous(), one)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(one.cpu().numpy()[0], y[i])
    # the rows around the first chunk boundary (or the batch's end) against a run of just that slice
    lo = max(0, min(m.run_batch, B) - 3)
    cnt = min(6, B - lo)
    part = torch.empty((cnt, m.output_elems), device="cuda")
    m.run_into(x[lo:lo + cnt].contiguous(), part)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(part.cpu().numpy(), y[lo:lo + cnt])
    print(json.dumps({"max_batch": B, "run_batch": m.run_batch, "fixture_max_abs_vs_oracle": err}))
    m.close()


def test_chunked_run_timing_and_read_value(gpu_ctx):
    """A chunked run's per-step times are summed over its chunks, and its intermediate values (which
    hold only the last chunk) are refused rather than returned stale."""
    import torch
    import ore
    from ore import squeezenet
    m = ore.Model(gpu_ctx, squeezenet.build(224), max_batch=2048)
    n = m.run_batch + 5
    x = _batch(n, 3)
    out = torch.empty((n, m.output_elems), device="cuda")
    m.enable_timing(True)
    m.run_into(x, out)
    t = np.asarray(m.step_times_ms())
    m.enable_timing(False)
    torch.cuda.synchronize()
    assert len(t) == len(m.steps()) and (t > 0).all()
    with pytest.raises(ore.OreError, match="chunks"):
        m.read_value("data_0")  # a chunked run keeps no whole-batch intermediates
    m.close()


def _margins(y, ref, ref64):
    return [{"image": i, "vs_oracle": float(np.abs(y[i] - ref[i]).max()), "vs_f64": float(np.abs(y[i] - ref64[i]).max()),
             "oracle_vs_f64": float(np.abs(ref[i] - ref64[i]).max())} for i in range(len(ref))]


@pytest.mark.parametrize("winograd", [True, False])
def test_benched_plan_parity(gpu_ctx, winograd):
    """bench.py's plan exactly: max_batch 256, autotune on a B = 256 batch, set_streams(2); the eight
    fixture images sit inside the batch (positions spread over it)."""
    import torch
    import ore
    from ore import squeezenet
    from golden.make_golden import squeezenet_inputs8
    ref = np.load(os.path.join(GOLD, "squeezenet_synth8_oracle.npz"))["output"]
    ref64 = np.load(os.path.join(GOLD, "squeezenet_synth8_f64.npz"))["output"]
    B = 256
    m = ore.Model(gpu_ctx, squeezenet.build(224), max_batch=B, winograd=winograd)
    m.set_streams(2)
    x = _batch(B, 1000)  # bench.py's seeded batch
    pos = [0, 37, 64, 101, 128, 170, 222, 255]
    x[pos] = torch.from_numpy(squeezenet_inputs8()).cuda()
    out = torch.empty((B, m.output_elems), device="cuda")
    m.autotune(x, out)
    names = {ore.Model.TILE_NAMES[t] for t in m.tiles() if t >= 0}
    if winograd:
        assert "wino lds" in names or any(n.startswith("wino") for n in names), names
    for _ in range(2):  # the timed loop runs the plan repeatedly
        m.run_into(x, out)
    torch.cuda.synchronize()
    y = out.cpu().numpy()[pos]
    rows = _margins(y, ref, ref64)
    print(json.dumps({"winograd": winograd, "tiles": sorted(names), "margins": rows}))
    for r in rows:
        assert r["vs_oracle"] <= 1e-5 + r["oracle_vs_f64"], r
        assert r["vs_f64"] <= (1e-5 if winograd else 2e-5), r
    assert np.array_equal(y.argmax(1), ref.argmax(1))
    m.close()


@pytest.mark.parametrize("winograd", [True, False])
def test_benched_plan_parity_calibrated(gpu_ctx, winograd):
    """The strict north_star bound on bench.py's exact plan and model: the zoo-calibrated SqueezeNet
    (squeezenet.build_calibrated: the zoo image's softmax peaks at 0.074, like squeezenet_output_0.pb),
    max_batch 256, autotuned on bench.py's seeded B = 256 batch with the 16 fixture images at bench.py's
    sample positions, two streams, run twice.  Every image: max |gpu - oracle| <= 1e-5 (no allowance for
    the oracle's own rounding: on this set the oracle is within 1.4e-6 of float64), same argmax."""
    import torch
    import ore
    from ore import squeezenet
    from golden.make_golden import squeezenet_inputs_calib16
    ref = np.load(os.path.join(GOLD, "squeezenet_calib16_oracle.npz"))["output"]
    ref64 = np.load(os.path.join(GOLD, "squeezenet_calib16_f64.npz"))["output"]
    assert float(np.abs(ref - ref64).max()) <= 2e-6  # the fixture sits far below the bound
    B = 256
    m = ore.Model(gpu_ctx, squeezenet.build_calibrated(224), max_batch=B, winograd=winograd)
    m.set_streams(2)
    x = _batch(B, 1000)  # bench.py's seeded batch
    pos = sorted({int(round(i * (B - 1) / 15)) for i in range(16)})  # bench.py's sample_idx at G = 256
    assert len(pos) == 16
    x[pos] = torch.from_numpy(squeezenet_inputs_calib16()).cuda()
    out = torch.empty((B, m.output_elems), device="cuda")
    m.autotune(x, out)
    for _ in range(2):
        m.run_into(x, out)
    torch.cuda.synchronize()
    y = out.cpu().numpy()[pos]
    rows = _margins(y, ref, ref64)
    print(json.dumps({"winograd": winograd, "margins": rows}))
    for r in rows:
        assert r["vs_oracle"] <= 1e-5, r
    assert np.array_equal(y.argmax(1), ref.argmax(1))
    m.close()


def test_benched_plan_conv1_band_vs_window(gpu_ctx):
    """bench.py's plan at B = 256 (one band per image: the headline launch of the band walker) with conv1 +
    pool1 + fire2/squeeze1x1 forced onto each of its two kernels: the 256 probability rows are equal bit
    for bit, and the calibrated images stay within the strict 1e-5 of the oracle fixture."""
    import torch
    import ore
    from ore import squeezenet
    from golden.make_golden import squeezenet_inputs_calib16
    ref = np.load(os.path.join(GOLD, "squeezenet_calib16_oracle.npz"))["output"]
    B = 256
    m = ore.Model(gpu_ctx, squeezenet.build_calibrated(224), max_batch=B)
    x = _batch(B, 1000)
    pos = sorted({int(round(i * (B - 1) / 15)) for i in range(16)})
    x[pos] = torch.from_numpy(squeezenet_inputs_calib16()).cuda()
    out = torch.empty((B, m.output_elems), device="cuda")
    m.autotune(x, out)
    ys = []
    for name in ("epool window f32", "epool band f32"):
        m.set_tile(0, ore.Model.TILE_NAMES.index(name))
        m.run_into(x, out)
        torch.cuda.synchronize()
        assert ore.Model.TILE_NAMES[m.tiles()[0]] == name
        ys.append(out.cpu().numpy())
    np.testing.assert_array_equal(ys[1], ys[0])
    assert float(np.abs(ys[1][pos] - ref).max()) <= 1e-5
    m.close()


def test_bench_world1_rccl():
    """bench.py's collective path at world size 1 on this GPU (--dist): torch.distributed.run with one
    process, init_process_group("nccl", device_id=...) -- a one-rank RCCL communicator -- and the
    per-step all_gather_into_tensor of the device rows (ore.parallel.gather_rows_into), the max over
    ranks, and the max-abs sample taken from the gathered rows."""
    env = dict(os.environ)
    env["MASTER_ADDR"] = "127.0.0.1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "1", "--dist", "--dist-backend", "nccl", "--steps", "3", "--warmup", "1", "--batch", "64",
           "--no-cpu-baseline", "--no-b1", "--no-f16-line", "--no-step-timing"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    print(json.dumps({k: res[k] for k in ("value", "ms_per_step", "max_abs_diff_vs_cpu")} | {"collective": res["config"]["collective"]}))
    assert res["n_gpus"] == 1 and res["config"]["global_batch"] == 64
    assert res["config"]["collective"].startswith("RCCL all_gather"), res["config"]
    assert "gathered over RCCL" in res["max_abs_sample"], res["max_abs_sample"]
    assert res["max_abs_diff_vs_cpu"] <= 1e-5 and res["top1_agrees_with_cpu"], res["max_abs_per_image"]
    assert res["value"] > 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("extra", [[], ["--global-batch", "256"]])
def test_bench_world2_gloo(extra):
    """bench.py's world > 1 branch end to end: two ranks (torch.distributed.run, 127.0.0.1) sharing this
    GPU, each running its slice of the one seeded global batch through the HIP model; rank 0 prints the
    JSON line whose max-abs sample comes out of the gathered rows."""
    env = dict(os.environ)
    env["MASTER_ADDR"] = "127.0.0.1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "64", "--dist-backend", "gloo",
           "--no-cpu-baseline", "--no-b1", "--no-f16-line", "--no-step-timing"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    G = 256 if extra else 128
    assert res["config"]["global_batch"] == G and res["config"]["per_gpu_batch"] == G // 2
    assert res["scaling"] == ("strong" if extra else "weak")
    assert "gloo" in res["config"]["collective"] and "gathered over gloo" in res["max_abs_sample"]
    assert res["max_abs_diff_vs_cpu"] <= 1e-5, res["max_abs_diff_vs_cpu"]
    assert res["value"] > 0
