#!/bin/bash
# Whole-step A/B of library builds on bench.py's own schedule (two streams, autotuned), one GPU call.
# Usage (repo root, on the box): [BENCH_ARGS="..."] bash tools/bench_ab.sh TAG NAME...
# (NAME = "cur" for lib/libore.so, else lib/exp/libore_NAME.so).  Output: gpurun_out/benchab_TAG.txt.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
TAG="$1"; shift
OUT="$ROOT/gpurun_out/benchab_$TAG.txt"
mkdir -p "$ROOT/gpurun_out"
: > "$OUT"
for name in "$@"; do
  if [ "$name" = cur ]; then lib="$ROOT/onnx-rusty-inference-engine_amd/lib/libore.so"; else lib="$ROOT/onnx-rusty-inference-engine_amd/lib/exp/libore_$name.so"; fi
  ORE_LIB="$lib" timeout -k 10 240 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-b1 --no-f16-line \
    --no-step-timing ${BENCH_ARGS:-} > "$OUT.tmp" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then cat "$OUT.tmp" >> "$OUT"; echo "[$name] rc=$rc" >> "$OUT"; tail -5 "$OUT"; exit $rc; fi
  python3 -c "import json,sys; r=json.loads([l for l in open('$OUT.tmp') if l.startswith('{')][-1]); print('[$name]', r['value'], 'img/s', r['ms_per_step'], 'ms', r['max_abs_diff_vs_cpu'])" >> "$OUT"
done
rm -f "$OUT.tmp"
cat "$OUT"
exit 0
