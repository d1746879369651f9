# band walker ablations (timing only): atomics / squeeze removed
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=onnx-rusty-inference-engine_amd/lib/exp
for v in base noatom nosq none; do
  if [ $v = base ]; then lib=""; else lib="$L/libore_band_$v.so"; fi
  echo "== $v"
  ORE_LIB=$lib timeout -k 10 120 python -u tools/band_probe.py || exit 1
done
