#!/bin/bash
# One GPU-box pass: smoke, GPU parity tests, a short bench, a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/abort/timeout ends the script (no retries).
# Usage (from the repo root on the box): bash tools/gpu_check.sh [tag] [stages...]
# stages: smoke tests bench bench16 prof (default: smoke tests bench prof)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
TAG="${1:-r01}"
shift || true
STAGES="${*:-smoke tests bench prof}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
fatal() { case "$1" in 124|134|137|139|-6|-11) return 0;; *) return 1;; esac; }
has() { case " $STAGES " in *" $1 "*) return 0;; *) return 1;; esac; }

if has smoke; then
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke_$TAG.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if has tests; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > "$OUT/pytest_gpu_$TAG.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest_gpu_$TAG.log"
  if fatal $rc || [ $rc -gt 1 ]; then exit $rc; fi
fi
if has bench; then
  timeout -k 10 600 python3 bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
  rc=$?; echo "bench rc=$rc"; cat "$OUT/bench_$TAG.json"; tail -5 "$OUT/bench_$TAG.err"
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if has bench16; then
  timeout -k 10 600 python3 bench.py --precision f16 --no-cpu-baseline > "$OUT/bench16_$TAG.json" 2> "$OUT/bench16_$TAG.err"
  rc=$?; echo "bench16 rc=$rc"; cat "$OUT/bench16_$TAG.json"; tail -5 "$OUT/bench16_$TAG.err"
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if has prof; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-b1 --no-f16-line > "$OUT/prof_bench_$TAG.json" 2> "$OUT/prof_$TAG.err"
  rc=$?; echo "prof rc=$rc"; cat "$OUT/prof_bench_$TAG.json"
  find "$OUT/prof_$TAG" -name "*stats*" | head
  if [ $rc -ne 0 ]; then tail -20 "$OUT/prof_$TAG.err"; exit $rc; fi
fi
exit 0
