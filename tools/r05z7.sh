set -u
cd "$GRAFT_REPO_ROOT"
for v in v1 v2 v3 cur; do
  if [ $v = cur ]; then lib=""; else lib="onnx-rusty-inference-engine_amd/lib/exp/libore_$v.so"; fi
  echo "== $v"; ORE_LIB=$lib timeout -k 10 120 python -u tools/band_probe.py || exit 1
done
