set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/x3_accuracy.py > gpurun_out/x3_acc.json 2> gpurun_out/x3_acc.err
rc=$?; echo "acc rc=$rc"; cat gpurun_out/x3_acc.json; tail -3 gpurun_out/x3_acc.err
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python3 -u -m pytest tests/test_x3_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "not synth_vs_oracle" > gpurun_out/x3_tests.log 2>&1
rc=$?; echo "x3 tests rc=$rc"; tail -5 gpurun_out/x3_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python3 bench.py --precision f32x3 --steps 10 --warmup 2 --no-cpu-baseline --no-b1 --layers > gpurun_out/bench_x3.json 2> gpurun_out/bench_x3.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/bench_x3.json; grep -v amdgpu.ids gpurun_out/bench_x3.err | tail -40
