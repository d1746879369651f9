set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_x3_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/x3_tests.log 2>&1
rc=$?; echo "x3 tests rc=$rc"; tail -5 gpurun_out/x3_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python3 tools/x3_accuracy.py > gpurun_out/x3_acc.json 2> gpurun_out/x3_acc.err
rc=$?; echo "acc rc=$rc"; tail -1 gpurun_out/x3_acc.json
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python3 bench.py --precision f32x3 --steps 10 --warmup 2 --no-cpu-baseline --no-b1 --layers > gpurun_out/bench_x3.json 2> gpurun_out/bench_x3.err
rc=$?; echo "bench rc=$rc"; cut -c1-200 gpurun_out/bench_x3.json; grep -v amdgpu.ids gpurun_out/bench_x3.err | grep "expand3x3\|conv10"
