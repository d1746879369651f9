#!/bin/bash
# PMC counter passes over a short bench run (one rocprofv3 --pmc pass per counter group, each
# with --kernel-trace only).  Usage on the box: bash tools/pmc.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-pmc}"
OUT="$ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
sha256sum "$ROOT/onnx-rusty-inference-engine_amd/lib/libore.so" | cut -d' ' -f1 > "$OUT/lib.sha256"
echo "${PMC_COMMIT:-unknown}" > "$OUT/commit"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1
echo "list rc=$?"
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $GROUP --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-step-timing --no-b1 --no-f16-line --streams 1 --dump-steps "$OUT/steps.json" ${PMC_BENCH_ARGS:-} > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i [$GROUP] rc=$rc"
  case $rc in 124|134|137|139) echo "fatal"; exit $rc;; esac
done < "$ROOT/${PMC_GROUPS:-tools/pmc_groups.txt}"
exit 0
