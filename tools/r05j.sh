set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_model_gpu.py -k "pool_expand or pool_squeeze" -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread -rf > $OUT/pytest_r05j.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_r05j.log
[ $rc -eq 0 ] || exit $rc
ORE_LIB=$GRAFT_REPO_ROOT/onnx-rusty-inference-engine_amd/lib/exp/libore_lb4.so timeout -k 10 600 python3 -u -m pytest tests/test_model_gpu.py -k "pool_expand" -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread -rf > $OUT/pytest_r05j_lb4.log 2>&1; rc=$?; echo "pytest lb4 rc=$rc"; tail -2 $OUT/pytest_r05j_lb4.log
bash tools/ab_layers.sh r05j f32 base cur lb4 base cur lb4 > /dev/null 2>&1; grep -E "^\[|pool" gpurun_out/ab_r05j.txt
