#!/bin/bash
# Builds timing-experiment variants of libore.so (kernel parts compiled out) into
# onnx-rusty-inference-engine_amd/lib/exp/; select one with ORE_LIB=<path> (never for parity).
# Usage: bash tools/build_exp.sh NAME "-DFLAG ..." [source basenames to rebuild; the rest from build/]
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
PKG="$ROOT/onnx-rusty-inference-engine_amd"
NAME="$1"; FLAGS="$2"; ONLY="${3:-}"
B="$PKG/build/exp_$NAME"; rm -rf "$B"; mkdir -p "$B" "$PKG/lib/exp"
HIPFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 $FLAGS"
if [ -n "$ONLY" ]; then make -s -C "$PKG" >/dev/null; cp "$PKG"/build/*.o "$B"/; fi
for src in "$PKG"/csrc/*.hip "$PKG"/csrc/*.cpp; do
  f=$(basename "${src%.*}")
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $f "* ]]; then continue; fi
  case "$src" in
    *ore_fire_f16.hip|*ore_conv_wino.hip) /opt/rocm/bin/hipcc $HIPFLAGS -fno-slp-vectorize -c "$src" -o "$B/$f.o" & ;;
    *.cpp) /opt/rocm/bin/hipcc $HIPFLAGS -x hip -c "$src" -o "$B/$f.o" & ;;
    *) /opt/rocm/bin/hipcc $HIPFLAGS -c "$src" -o "$B/$f.o" & ;;
  esac
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$PKG/lib/exp/libore_$NAME.so" "$B"/*.o
echo "$PKG/lib/exp/libore_$NAME.so"
