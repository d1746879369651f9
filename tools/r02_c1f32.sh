set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py -k "conv_pool_walk_bit_identical or squeezenet" > gpurun_out/c3_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/c3_pytest.log; [ $rc = 0 ] || exit $rc
for v in default 6; do
  if [ $v = default ]; then unset ORE_CONV_POOL_STREAM; else export ORE_CONV_POOL_STREAM=$v; fi
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --layers > gpurun_out/c3.json 2> gpurun_out/c3_$v.err
  rc=$?; echo "$v rc=$rc $(cut -c100-175 gpurun_out/c3.json)"; grep "conv1 " gpurun_out/c3_$v.err; [ $rc = 0 ] || exit $rc
done
