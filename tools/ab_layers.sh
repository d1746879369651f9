#!/bin/bash
# Per-layer A/B of library builds in one GPU call: tools/bench_layers.py once per library.
# Usage (repo root, on the box): bash tools/ab_layers.sh TAG PRECISION NAME... (NAME = "cur" for
# lib/libore.so, else lib/exp/libore_NAME.so).  Output: gpurun_out/ab_TAG.txt.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
TAG="$1"; PREC="$2"; shift 2
OUT="$ROOT/gpurun_out/ab_$TAG.txt"
mkdir -p "$ROOT/gpurun_out"
: > "$OUT"
for name in "$@"; do
  if [ "$name" = cur ]; then lib="$ROOT/onnx-rusty-inference-engine_amd/lib/libore.so"; else lib="$ROOT/onnx-rusty-inference-engine_amd/lib/exp/libore_$name.so"; fi
  ORE_LIB="$lib" timeout -k 10 180 python3 tools/bench_layers.py --precision "$PREC" --tag "$name" >> "$OUT" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "[$name] rc=$rc" >> "$OUT"; tail -5 "$OUT"; exit $rc; fi
done
grep -E "^\[" "$OUT"
exit 0
