# f16: bench under rocprofv3 kernel-trace stats, then the PMC passes (tools/pmc.sh) of the f16 plan
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_f16" -o run -- python3 "$R/bench.py" --precision f16 --steps 20 --warmup 3 --no-cpu-baseline --no-b1 > "$R/gpurun_out/prof_f16_bench.json" 2> "$R/gpurun_out/prof_f16_bench.err")
rc=$?; echo "prof rc=$rc"; [ $rc = 0 ] || exit $rc
PMC_BENCH_ARGS="--precision f16" bash tools/pmc.sh f16r02
