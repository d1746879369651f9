# A/B: pool3 with e1 recomputed inside (FUSE_ALL = 14311) vs e1 as its own launch beside the Winograd e3 (6119)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_model_gpu.py -k "band_units" > gpurun_out/r05z2_tests.log 2>&1 || { tail -30 gpurun_out/r05z2_tests.log; exit 1; }
tail -1 gpurun_out/r05z2_tests.log
for f in 14311 6119 14311 6119; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-b1 --no-f16-line --fusion $f > gpurun_out/r05z2_$f.json 2> gpurun_out/r05z2_$f.err || { tail -5 gpurun_out/r05z2_$f.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r05z2_$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']), d['ms_per_step'])"
done
