set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
L=onnx-rusty-inference-engine_amd/lib
for lib in $L/libore.so $L/exp/libore_fireold.so $L/exp/libore_c3w2.so $L/libore.so; do
  ORE_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --no-f16-line --layers > gpurun_out/ab2.json 2> gpurun_out/ab2.err
  rc=$?; echo "$(basename $lib) rc=$rc $(cut -c100-160 gpurun_out/ab2.json)"; grep -E "conv1 |fire" gpurun_out/ab2.err | grep -E "conv1|\+" | awk '{printf "%s %s | ", $1, $3}'; echo; [ $rc = 0 ] || exit $rc
done
