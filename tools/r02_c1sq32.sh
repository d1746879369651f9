set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py -k "squeeze_fused or conv1_squeeze or conv_pool_walk or autotune or squeezenet" > gpurun_out/sq32_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/sq32_pytest.log; [ $rc = 0 ] || exit $rc
for v in 1 0; do
  ORE_C1_SQUEEZE=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --no-f16-line --layers > gpurun_out/sq32.json 2> gpurun_out/sq32_$v.err
  rc=$?; echo "sq=$v rc=$rc $(cut -c100-160 gpurun_out/sq32.json)"; grep -E "conv1|fire2/sq" gpurun_out/sq32_$v.err; [ $rc = 0 ] || exit $rc
done
