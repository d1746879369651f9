#!/bin/bash
# End-of-session GPU pass: smoke, GPU tests, bench (f32 + f16 line), bench16, rocprofv3 summary, then
# the PMC passes (f32 and f16) whose traffic JSON bench.py reports.  Usage: bash tools/final_check.sh TAG COMMIT
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
TAG="${1:-final}"; COMMIT="${2:-unknown}"
bash tools/gpu_check.sh "$TAG" smoke tests bench bench16 prof
rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
PMC_COMMIT="$COMMIT" bash tools/pmc.sh "${TAG}_f32" || exit $?
PMC_COMMIT="$COMMIT" PMC_BENCH_ARGS="--precision f16" bash tools/pmc.sh "${TAG}_f16" || exit $?
exit 0
