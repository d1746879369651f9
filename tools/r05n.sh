# band walker: squeeze deferred into the next step; parity + probe
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread \
  tests/test_model_gpu.py tests/test_config4_gpu.py -k "band or conv_pool_squeeze_fused" > gpurun_out/r05n_tests.log 2>&1 || { tail -40 gpurun_out/r05n_tests.log; exit 1; }
tail -2 gpurun_out/r05n_tests.log
for v in ${PROBE_LIBS:-base}; do
  if [ $v = base ]; then lib=""; else lib="onnx-rusty-inference-engine_amd/lib/exp/libore_$v.so"; fi
  echo "== $v"
  ORE_LIB=$lib timeout -k 10 120 python -u tools/band_probe.py || exit 1
done
