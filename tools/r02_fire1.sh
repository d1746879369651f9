set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_wino_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fire1_tests.log 2>&1
rc=$?; echo "wino tests rc=$rc"; tail -15 gpurun_out/fire1_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --layers > gpurun_out/fire1_bench.json 2> gpurun_out/fire1_bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/fire1_bench.json; grep -v amdgpu.ids gpurun_out/fire1_bench.err
