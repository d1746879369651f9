# band walker (pooled-conv variant 8): parity tests, then bench with autotune and a kernel-trace profile
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_model_gpu.py tests/test_config4_gpu.py -k "band or conv_pool_squeeze_fused or conv1_squeeze_fused" > gpurun_out/r05l_tests.log 2>&1 || { tail -40 gpurun_out/r05l_tests.log; exit 1; }
tail -5 gpurun_out/r05l_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05l_bench.json 2> gpurun_out/r05l_bench.err || { tail -20 gpurun_out/r05l_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05l_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["conv_tiles"]["tile_per_conv"][:2], d["roofline"]["kernel"][:60], d["roofline"]["launch_us"], d["max_abs_diff_vs_cpu"])
PY
bash tools/gpu_check.sh r05l prof > gpurun_out/r05l_profcheck.log 2>&1 || { tail -20 gpurun_out/r05l_profcheck.log; exit 1; }
