# pool_conv1x1: 4 pooled columns per pooling task (16-B LDS reads); parity + probe + bench layers
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread \
  tests/test_model_gpu.py -k "pool_squeeze or pool_expand" > gpurun_out/r05x_tests.log 2>&1 || { tail -40 gpurun_out/r05x_tests.log; exit 1; }
tail -2 gpurun_out/r05x_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --no-f16-line --layers > gpurun_out/r05x_bench.json 2> gpurun_out/r05x_bench.err || { tail -20 gpurun_out/r05x_bench.err; exit 1; }
grep -E "pool|conv1" gpurun_out/r05x_bench.err | head
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05x_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["max_abs_diff_vs_cpu"])
PY
