set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_wino_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/w7_tests.log 2>&1
rc=$?; echo "wino tests rc=$rc"; tail -3 gpurun_out/w7_tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python3 tools/wino_bench.py --tiles 0,1,2,3 > gpurun_out/w7_bench.txt 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/w7_bench.txt
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 > gpurun_out/w7_graph.json 2> gpurun_out/w7_graph.err
rc=$?; echo "graph rc=$rc"; cut -c1-250 gpurun_out/w7_graph.json
