set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export ORE_CONV_POOL_STREAM=6
L=onnx-rusty-inference-engine_amd/lib
for lib in $L/libore.so $L/exp/libore_c3w2.so $L/libore.so; do
  ORE_LIB=$lib timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-b1 --no-f16-line --no-autotune --layers > gpurun_out/c3w.json 2> gpurun_out/c3w.err
  rc=$?; echo "$(basename $lib) rc=$rc $(grep 'conv1 ' gpurun_out/c3w.err)"; [ $rc = 0 ] || exit $rc
done
