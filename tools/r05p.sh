# band walker: batched squeeze reads; parity + probe + stamps
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread \
  tests/test_model_gpu.py tests/test_config4_gpu.py -k "band or conv_pool_squeeze_fused" > gpurun_out/r05p_tests.log 2>&1 || { tail -40 gpurun_out/r05p_tests.log; exit 1; }
tail -2 gpurun_out/r05p_tests.log
timeout -k 10 120 python -u tools/band_probe.py || exit 1
ORE_LIB=onnx-rusty-inference-engine_amd/lib/exp/libore_band_stamps.so timeout -k 10 120 python -u tools/band_probe.py || exit 1
