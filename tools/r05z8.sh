# band walker: idle waves skip the last partial step; parity + probe + bench
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_model_gpu.py tests/test_config4_gpu.py -k "band or conv_pool_squeeze_fused or conv1_squeeze" > gpurun_out/r05z8_tests.log 2>&1 || { tail -40 gpurun_out/r05z8_tests.log; exit 1; }
tail -1 gpurun_out/r05z8_tests.log
timeout -k 10 120 python -u tools/band_probe.py || exit 1
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-b1 --no-f16-line --layers > gpurun_out/r05z8_bench.json 2> gpurun_out/r05z8_bench.err || { tail -20 gpurun_out/r05z8_bench.err; exit 1; }
grep -E "conv1" gpurun_out/r05z8_bench.err | head -2
python -c "import json; d=json.loads(open('gpurun_out/r05z8_bench.json').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'], d['conv_tiles']['tile_per_conv'][0])"
done
