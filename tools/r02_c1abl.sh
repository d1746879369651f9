set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
L=onnx-rusty-inference-engine_amd/lib
for lib in $L/libore.so $L/exp/libore_cp_oneload.so; do
  ORE_LIB=$lib timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-b1 --layers > gpurun_out/c1abl.json 2> gpurun_out/c1abl.err
  rc=$?; echo "$lib rc=$rc"; grep "conv1 " gpurun_out/c1abl.err
  case $rc in 0) ;; *) exit $rc;; esac
done
