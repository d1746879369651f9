#!/bin/bash
# The one parameterised GPU-box pass for experiments (replaces the per-run wrappers of rounds 4-5).
# Usage (repo root, on the box):
#   [TESTS="tests/test_x.py ..."] [TESTK="pytest -k expression"] [TESTLIB=NAME] [PREC=f32|f16] [BENCH=1] bash tools/gpu_ab.sh TAG [NAME...]
# 1. TESTS: pytest on that selection first (with lib NAME when TESTLIB is set; "cur" = lib/libore.so);
# 2. BENCH=1: bench.py once (default library) -> gpurun_out/TAG_bench.json;
# 3. NAMEs: per-layer A/B, tools/ab_layers.sh TAG PREC NAME... (alternate names for repeated pairs).
# Every GPU step has its own time limit and a failure ends the script.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
TAG="$1"; shift
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
PKG="$ROOT/onnx-rusty-inference-engine_amd"
if [ -n "${TESTS:-}" ]; then
  lib=""
  if [ -n "${TESTLIB:-}" ] && [ "$TESTLIB" != cur ]; then lib="$PKG/lib/exp/libore_$TESTLIB.so"; fi
  ORE_LIB="$lib" timeout -k 10 600 python3 -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    $TESTS ${TESTK:+-k "$TESTK"} > "$OUT/${TAG}_tests.log" 2>&1 || { tail -40 "$OUT/${TAG}_tests.log"; exit 1; }
  tail -2 "$OUT/${TAG}_tests.log"
fi
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err" || {
    tail -20 "$OUT/${TAG}_bench.err"; exit 1; }
  cat "$OUT/${TAG}_bench.json"
fi
if [ $# -gt 0 ]; then
  bash tools/ab_layers.sh "$TAG" "${PREC:-f32}" "$@" || exit $?
fi
exit 0
