set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_model_gpu.py -k "pool_expand or pool_squeeze or fire_pool or squeezenet_synth or node_level" tests/test_parity_attrib_gpu.py -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread -rf > $OUT/pytest_r05b.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest_r05b.log | tail -30
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python3 tools/bench_layers.py --tag pe_on > $OUT/layers_r05b.txt 2>&1 && timeout -k 10 300 python3 tools/bench_layers.py --fusion 6119 --tag pe_off >> $OUT/layers_r05b.txt 2>&1 && timeout -k 10 300 python3 tools/bench_layers.py --tag pe_on2 >> $OUT/layers_r05b.txt 2>&1; rc=$?; echo "layers rc=$rc"; cat $OUT/layers_r05b.txt | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --no-b1 --no-cpu-baseline > $OUT/bench_r05b.json 2> $OUT/bench_r05b.err; rc=$?; echo "bench rc=$rc"; head -c 700 $OUT/bench_r05b.json
