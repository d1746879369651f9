set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
L=onnx-rusty-inference-engine_amd/lib
for lib in $L/libore.so $L/exp/libore_fminb3.so $L/exp/libore_fd3.so $L/libore.so; do
  ORE_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --layers > gpurun_out/fab.json 2> gpurun_out/fab.err
  rc=$?; echo "$(basename $lib) rc=$rc $(cut -c100-160 gpurun_out/fab.json)"; grep "fire" gpurun_out/fab.err | grep "+" | awk '{printf "%s %s | ", $1, $3}'; echo; [ $rc = 0 ] || exit $rc
done
