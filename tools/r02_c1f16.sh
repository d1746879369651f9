set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_f16_gpu.py -k "first_conv" > gpurun_out/c1_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/c1_pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c1prof -o run -- python3 bench.py --precision f16 --steps 10 --warmup 2 --no-cpu-baseline --no-b1 > gpurun_out/c1_bench.json 2> gpurun_out/c1_bench.err
rc=$?; echo "prof rc=$rc"; find gpurun_out/c1prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-4 {} | head -20'
