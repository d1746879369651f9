# pool + squeeze band height A/B: parity of each variant (pool tests), then per-layer timings
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in p13 p14 p23; do
  ORE_LIB=$PWD/onnx-rusty-inference-engine_amd/lib/exp/libore_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_model_gpu.py -k "pool_squeeze or pool_expand" > gpurun_out/r05zi_tests_$v.log 2>&1 || { tail -30 gpurun_out/r05zi_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r05zi_tests_$v.log)"
done
bash tools/ab_layers.sh r05zi f32 cur p13 p14 p23 p14p23 cur
