set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_f16_gpu.py -k "first_conv" > gpurun_out/c1_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/c1_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --precision f16 --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --layers > gpurun_out/c1a.json 2> gpurun_out/c1a.err
rc=$?; echo "rc=$rc $(cut -c100-190 gpurun_out/c1a.json)"; grep -v amdgpu gpurun_out/c1a.err | head -4
