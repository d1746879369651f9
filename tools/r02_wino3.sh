set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
L=onnx-rusty-inference-engine_amd/lib
timeout -k 10 300 python3 tools/wino_bench.py > gpurun_out/wino_bench3.txt 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/wino_bench3.txt
case $rc in 0) ;; *) exit $rc;; esac
for lib in $L/exp/libore_wg_noa.so $L/exp/libore_wg_nob.so $L/exp/libore_wg_nost.so $L/exp/libore_wg_all.so; do
  ORE_LIB=$lib timeout -k 10 120 python3 tools/wino_bench.py --no-direct --tiles 0 --only f4.e3,f8.e3,f9.e3 >> gpurun_out/wino_abl3.txt 2>&1
  rc=$?; echo "$lib rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
grep -v amdgpu.ids gpurun_out/wino_abl3.txt
