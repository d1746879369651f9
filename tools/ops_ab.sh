#!/bin/bash
# Single-layer A/B of library builds in one GPU call: tools/bench_ops.py once per library and pass.
# Usage (repo root, on the box): [OPS_ARGS="--names f4.e3,f8.e3 --tile 40"] bash tools/ops_ab.sh TAG NAME...
# (NAME = "cur" for lib/libore.so, else lib/exp/libore_NAME.so).  Output: gpurun_out/opsab_TAG.txt.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
TAG="$1"; shift
OUT="$ROOT/gpurun_out/opsab_$TAG.txt"
mkdir -p "$ROOT/gpurun_out"
: > "$OUT"
for name in "$@"; do
  if [ "$name" = cur ]; then lib="$ROOT/onnx-rusty-inference-engine_amd/lib/libore.so"; else lib="$ROOT/onnx-rusty-inference-engine_amd/lib/exp/libore_$name.so"; fi
  echo "[$name]" >> "$OUT"
  ORE_LIB="$lib" timeout -k 10 120 python3 tools/bench_ops.py ${OPS_ARGS:---names f4.e3,f8.e3 --tile 40} >> "$OUT" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "[$name] rc=$rc" >> "$OUT"; tail -5 "$OUT"; exit $rc; fi
done
cat "$OUT"
exit 0
