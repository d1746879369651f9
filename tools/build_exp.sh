#!/bin/bash
# Builds timing-experiment variants of libore.so into onnx-rusty-inference-engine_amd/lib/exp/; select
# one with ORE_LIB=<path> (never for parity).  The product sources carry no experiment conditionals: an
# experiment is a patch (PATCHES="tools/patches/x.patch ...", applied with -p3 to a copy of csrc/) and/or
# -D flags for that patched copy.
# Usage: [PATCHES="..."] bash tools/build_exp.sh NAME "-DFLAG ..." [source basenames to rebuild; the rest from build/]
#   e.g. PATCHES=tools/patches/stamps.patch bash tools/build_exp.sh stamps "-DORE_STAMPS" ore_conv_wino
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
PKG="$ROOT/onnx-rusty-inference-engine_amd"
NAME="$1"; FLAGS="$2"; ONLY="${3:-}"
B="$PKG/build/exp_$NAME"; rm -rf "$B"; mkdir -p "$B/src" "$PKG/lib/exp"
cp "$PKG"/csrc/* "$B/src/"
for p in ${PATCHES:-}; do
  case "$p" in /*) ;; *) p="$ROOT/$p";; esac
  patch -s -d "$B/src" -p3 < "$p"
done
# -I csrc: the sources' "../../include/ore.h" resolves from there
HIPFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$PKG/csrc $FLAGS"
if [ -n "$ONLY" ]; then make -s -C "$PKG" >/dev/null; cp "$PKG"/build/*.o "$B"/; fi
pids=()
for src in "$B"/src/*.hip "$B"/src/*.cpp; do
  f=$(basename "${src%.*}")
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $f "* ]]; then continue; fi
  case "$src" in
    *ore_fire_f16.hip|*ore_conv_wino.hip) /opt/rocm/bin/hipcc $HIPFLAGS -fno-slp-vectorize -c "$src" -o "$B/$f.o" & ;;
    *.cpp) /opt/rocm/bin/hipcc $HIPFLAGS -x hip -c "$src" -o "$B/$f.o" & ;;
    *) /opt/rocm/bin/hipcc $HIPFLAGS -c "$src" -o "$B/$f.o" & ;;
  esac
  pids+=($!)
done
for pid in "${pids[@]}"; do wait "$pid"; done  # set -e: a failed compile ends the script
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$PKG/lib/exp/libore_$NAME.so" "$B"/*.o
echo "$PKG/lib/exp/libore_$NAME.so"
