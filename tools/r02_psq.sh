set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py -k "pool_squeeze or pool_conv or squeezenet or autotune" > gpurun_out/psq_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/psq_pytest.log; [ $rc = 0 ] || exit $rc
for v in 1 0; do
  ORE_POOL_SQUEEZE=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --no-f16-line --layers > gpurun_out/psq.json 2> gpurun_out/psq_$v.err
  rc=$?; echo "psq=$v rc=$rc $(cut -c100-160 gpurun_out/psq.json)"; grep -E "pool5|fire9/sq" gpurun_out/psq_$v.err; [ $rc = 0 ] || exit $rc
done
