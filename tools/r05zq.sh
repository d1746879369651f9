# Winograd LDS kernel: biases written to LDS after the first stage's DMAs issue (product) vs before (old):
# Winograd parity tests, prologue stamps, per-layer A/B
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_wino_gpu.py tests/test_config4_gpu.py -k "wino or benched_plan_parity" > gpurun_out/r05zq_tests.log 2>&1 || { tail -30 gpurun_out/r05zq_tests.log; exit 1; }
tail -1 gpurun_out/r05zq_tests.log
ORE_LIB=$PWD/onnx-rusty-inference-engine_amd/lib/exp/libore_stampsn.so timeout -k 10 300 python3 -u tools/stamps.py --tag stamps_bias_after_dma > gpurun_out/r05zq_stamps.txt 2>&1 || { tail -20 gpurun_out/r05zq_stamps.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zq_stamps.txt
bash tools/ab_layers.sh r05zq f32 old cur old cur
