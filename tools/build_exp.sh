#!/bin/bash
# Builds timing-experiment variants of libore.so (kernel parts compiled out) into
# onnx-rusty-inference-engine_amd/lib/exp/; select one with ORE_LIB=<path> (never for parity).
# Usage: bash tools/build_exp.sh NAME "-DFLAG ..."
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
PKG="$ROOT/onnx-rusty-inference-engine_amd"
NAME="$1"; FLAGS="$2"
B="$PKG/build/exp_$NAME"; mkdir -p "$B" "$PKG/lib/exp"
HIPFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 $FLAGS"
/opt/rocm/bin/hipcc $HIPFLAGS -fno-slp-vectorize -c "$PKG/csrc/ore_conv_x3.hip" -o "$B/ore_conv_x3.o" &
for f in ore_kernels ore_conv ore_conv_f16 ore_conv_direct ore_conv_stream ore_fire ore_conv_pool ore_conv_wino ore_fire_f16 ore_conv1_f16 ore_conv1_f32 ore_pool_conv; do /opt/rocm/bin/hipcc $HIPFLAGS -c "$PKG/csrc/$f.hip" -o "$B/$f.o" & done
for f in ore_ops ore_model ore_onnx; do /opt/rocm/bin/hipcc $HIPFLAGS -x hip -c "$PKG/csrc/$f.cpp" -o "$B/$f.o" & done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$PKG/lib/exp/libore_$NAME.so" "$B"/*.o
echo "$PKG/lib/exp/libore_$NAME.so"
