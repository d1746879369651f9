set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r05a.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke_r05a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests/test_config4_gpu.py tests/test_parity_attrib_gpu.py tests/test_sanitize_gpu.py -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread -rf > $OUT/pytest_new_r05a.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest_new_r05a.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python3 bench.py > $OUT/bench_r05a.json 2> $OUT/bench_r05a.err; rc=$?; echo "bench rc=$rc"; cat $OUT/bench_r05a.json | head -c 1500; tail -3 $OUT/bench_r05a.err
