#!/bin/bash
# PMC passes (tools/pmc_groups_sq.txt, one rocprofv3 --pmc pass per line, --kernel-trace only) over
# tools/bench_ops.py for one layer and a list of forced tiles.
# Usage on the box: bash tools/pmc_ops.sh TAG LAYER TILE...
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; LAYER="$2"; shift 2
OUT="$ROOT/gpurun_out/pmcops_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for T in "$@"; do
  i=0
  while read -r GROUP; do
    [ -z "$GROUP" ] && continue
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $GROUP --kernel-trace --output-format csv -d "$OUT/t${T}_p$i" -o run -- \
      python3 "$ROOT/tools/bench_ops.py" --names "$LAYER" --tile "$T" --reps 5 > "$OUT/t${T}_p$i.log" 2>&1
    rc=$?
    echo "tile $T pass $i rc=$rc"
    case $rc in 0) ;; *) echo "fatal"; exit $rc;; esac
  done < "$ROOT/${PMC_GROUPS:-tools/pmc_groups_sq.txt}"
done
exit 0
