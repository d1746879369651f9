#!/bin/bash
# A/B of experiment builds (lib/exp/libore_NAME.so, "cur" = lib/libore.so) on single-conv graphs:
# bash tools/exp_r04.sh TAG "LAYERS" "TILE" NAME...   -> gpurun_out/exp_TAG.txt
set -u
TAG="$1"; LAYERS="$2"; TILE="$3"; shift 3
mkdir -p gpurun_out
OUT=gpurun_out/exp_$TAG.txt
: > $OUT
for lib in "$@"; do
  if [ $lib = cur ]; then L=onnx-rusty-inference-engine_amd/lib/libore.so; else L=onnx-rusty-inference-engine_amd/lib/exp/libore_$lib.so; fi
  echo "== $lib" >> $OUT
  ORE_LIB=$L timeout -k 10 120 python3 tools/bench_ops.py --only conv --names "$LAYERS" --tile "$TILE" --reps 20 >> $OUT 2>&1 || { echo "fail $lib"; cat $OUT; exit 1; }
done
grep -v amdgpu.ids $OUT
