#!/bin/bash
# Achievable HBM copy bandwidth and MFMA rates on this GPU (tools/peaks.hip).
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$ROOT/gpurun_out"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o "$ROOT/gpurun_out/peaks" "$ROOT/tools/peaks.hip"
timeout -k 10 120 "$ROOT/gpurun_out/peaks"
