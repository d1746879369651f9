set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_model_gpu.py -k "fire_pool or concat_pool or autotune or fire_fusion or synth_vs_oracle or pool_squeeze" > gpurun_out/fp32_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/fp32_pytest.log; [ $rc = 0 ] || exit $rc
for v in 1 0; do
  ORE_FIRE_POOL=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --no-f16-line --layers > gpurun_out/fp32.json 2> gpurun_out/fp32_$v.err
  rc=$?; echo "firepool=$v rc=$rc $(cut -c100-160 gpurun_out/fp32.json)"; grep -E "fire4|fire5|pool5" gpurun_out/fp32_$v.err; [ $rc = 0 ] || exit $rc
done
