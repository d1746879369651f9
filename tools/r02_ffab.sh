set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
L=onnx-rusty-inference-engine_amd/lib
for lib in $L/libore.so $L/exp/libore_ffold.so $L/exp/libore_ffbd3.so $L/libore.so; do
  ORE_LIB=$lib timeout -k 10 200 python3 bench.py --precision f16 --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --layers > gpurun_out/ffab.json 2> gpurun_out/ffab.err
  rc=$?; echo "$(basename $lib) rc=$rc $(cut -c100-160 gpurun_out/ffab.json)"; grep "fire" gpurun_out/ffab.err | awk '{printf "%s %s | ", $1, $3}'; echo; [ $rc = 0 ] || exit $rc
done
