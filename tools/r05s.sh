# band walker: B ring depth 3; parity + probe + bench
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread \
  tests/test_model_gpu.py tests/test_config4_gpu.py -k "band or conv_pool_squeeze_fused" > gpurun_out/r05s_tests.log 2>&1 || { tail -40 gpurun_out/r05s_tests.log; exit 1; }
tail -2 gpurun_out/r05s_tests.log
timeout -k 10 120 python -u tools/band_probe.py || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 > gpurun_out/r05s_bench.json 2> gpurun_out/r05s_bench.err || { tail -20 gpurun_out/r05s_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05s_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["conv_tiles"]["tile_per_conv"][:2], d["roofline"]["kernel"][:60], d["roofline"]["launch_us"], d["max_abs_diff_vs_cpu"])
print("f16", d.get("f16", {}).get("value") if isinstance(d.get("f16"), dict) else None)
PY
