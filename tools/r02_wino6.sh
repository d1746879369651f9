set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
L=onnx-rusty-inference-engine_amd/lib
for lib in $L/libore.so $L/exp/libore_wg_nomfma.so $L/exp/libore_wg_nomfma_nost.so; do
  ORE_LIB=$lib timeout -k 10 120 python3 tools/wino_bench.py --no-direct --tiles 0 --only f4.e3,f8.e3,f9.e3 >> gpurun_out/wino_abl6.txt 2>&1
  rc=$?; echo "$lib rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
grep -v amdgpu.ids gpurun_out/wino_abl6.txt
