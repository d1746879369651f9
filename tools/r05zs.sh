# Winograd LDS kernel: prologue divisions by float reciprocals (rcp, tools/patches/wino_rcp_div.patch) vs integer
# divisions (cur): parity of rcp + per-layer A/B
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ORE_LIB=$PWD/onnx-rusty-inference-engine_amd/lib/exp/libore_rcp.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_wino_gpu.py tests/test_config4_gpu.py -k "wino or benched_plan_parity" > gpurun_out/r05zs_tests.log 2>&1 || { tail -30 gpurun_out/r05zs_tests.log; exit 1; }
tail -1 gpurun_out/r05zs_tests.log
bash tools/ab_layers.sh r05zs f32 cur rcp cur rcp
