set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
L=onnx-rusty-inference-engine_amd/lib
for lib in $L/libore.so $L/exp/libore_nomfma.so $L/exp/libore_nopool.so $L/exp/libore_noload.so; do
  ORE_LIB=$lib timeout -k 10 200 python3 bench.py --precision f16 --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --layers > gpurun_out/c1a.json 2> gpurun_out/c1a.err
  rc=$?; echo "$lib rc=$rc $(grep 'conv1 ' gpurun_out/c1a.err)"; [ $rc = 0 ] || exit $rc
done
