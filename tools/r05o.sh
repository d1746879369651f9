# band walker phase stamps + kernel-trace of the probe
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
ORE_LIB=onnx-rusty-inference-engine_amd/lib/exp/libore_band_stamps.so timeout -k 10 120 python -u tools/band_probe.py || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r05o_prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/band_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/r05o_prof.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT" && f=$(find gpurun_out/r05o_prof -name "*kernel_stats.csv" | head -1) && python - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r["Calls"], r["AverageNs"], r["Name"][:90])
PY
