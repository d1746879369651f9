set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/pool_sq_probe.py || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05w_prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/pool_sq_probe.py" --reps 5 > /dev/null 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT" && f=$(find gpurun_out/r05w_prof -name "*kernel_stats.csv" | head -1) && python - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r["Calls"], r["AverageNs"], r["Name"][:100])
PY
