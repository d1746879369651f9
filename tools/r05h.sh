set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_wino_gpu.py tests/test_model_gpu.py -k "wino or conv_pool or squeezenet" -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread -rf > $OUT/pytest_quick_r05h.log 2>&1; rc=$?; echo "quick pytest rc=$rc"; tail -3 $OUT/pytest_quick_r05h.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_layers.sh r05h f32 base cur c1old base cur c1old > /dev/null 2>&1; grep -E "^\[|expand3x3|conv1" gpurun_out/ab_r05h.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r05h.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke_r05h.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 400 --timeout-method thread -rf > $OUT/pytest_gpu_r05h.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu_r05h.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python3 bench.py > $OUT/bench_r05h.json 2> $OUT/bench_r05h.err; rc=$?; echo "bench rc=$rc"; head -c 300 $OUT/bench_r05h.json; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/split_batch_probe.py --splits 1 2 4 1 2 > $OUT/split_r05h.txt 2>&1; rc=$?; echo "split rc=$rc"; grep splits $OUT/split_r05h.txt
