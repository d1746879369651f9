set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_f16_gpu.py > gpurun_out/ff16_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/ff16_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --precision f16 --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --layers > gpurun_out/ff16_bench.json 2> gpurun_out/ff16_bench.err
rc=$?; cut -c1-300 gpurun_out/ff16_bench.json; grep -v amdgpu.ids gpurun_out/ff16_bench.err | head -40; exit $rc
