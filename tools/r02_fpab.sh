set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
L=onnx-rusty-inference-engine_amd/lib
:
:
for lib in $L/exp/libore_fpns.so; do
  ORE_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --no-f16-line --layers > gpurun_out/fpab.json 2> gpurun_out/fpab.err
  rc=$?; echo "$(basename $lib) rc=$rc $(cut -c100-160 gpurun_out/fpab.json)"; grep -E "fire4" gpurun_out/fpab.err; [ $rc = 0 ] || exit $rc
done
PMC_GROUPS=tools/pmc_groups_sq.txt bash tools/pmc.sh fp32
