# product pool tests (three pooled rows); Winograd start stagger A/B (timing only)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_model_gpu.py -k "pool_squeeze or pool_expand or squeezenet" > gpurun_out/r05zj_tests.log 2>&1 || { tail -30 gpurun_out/r05zj_tests.log; exit 1; }
tail -1 gpurun_out/r05zj_tests.log
bash tools/ab_layers.sh r05zj f32 cur st1 st2 st3 sth2 ch32 wnt wsc1 cur
