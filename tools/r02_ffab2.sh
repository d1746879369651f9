set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_f16_gpu.py > gpurun_out/ffab2_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/ffab2_pytest.log; [ $rc = 0 ] || exit $rc
L=onnx-rusty-inference-engine_amd/lib
for lib in $L/libore.so $L/exp/libore_ffglob.so $L/libore.so; do
  ORE_LIB=$lib timeout -k 10 200 python3 bench.py --precision f16 --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --layers > gpurun_out/ffab.json 2> gpurun_out/ffab.err
  rc=$?; echo "$(basename $lib) rc=$rc $(cut -c100-160 gpurun_out/ffab.json)"; grep "fire" gpurun_out/ffab.err | grep "+" | awk '{printf "%s %s | ", $1, $3}'; echo; [ $rc = 0 ] || exit $rc
done
