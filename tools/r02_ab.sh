# A/B of two libore builds in one box: bash tools/r02_ab.sh LIB_A LIB_B [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
A=$1; B=$2; shift 2
for lib in $A $B $A $B; do
  ORE_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --layers "$@" > gpurun_out/ab.json 2> gpurun_out/ab_$(basename $lib).err
  rc=$?; echo "$(basename $lib) rc=$rc $(cut -c100-175 gpurun_out/ab.json)"; [ $rc = 0 ] || exit $rc
done
