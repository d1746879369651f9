set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py -k "pool_squeeze or pool_conv" > gpurun_out/psq_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/psq_pytest.log; [ $rc = 0 ] || exit $rc
L=onnx-rusty-inference-engine_amd/lib
for lib in $L/libore.so $L/exp/libore_ps232.so $L/exp/libore_ps432.so $L/exp/libore_ps216.so $L/libore.so; do
  ORE_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --no-f16-line --layers > gpurun_out/psq.json 2> gpurun_out/psq.err
  rc=$?; echo "$(basename $lib) rc=$rc $(cut -c100-160 gpurun_out/psq.json)"; grep -E "pool5" gpurun_out/psq.err; [ $rc = 0 ] || exit $rc
done
