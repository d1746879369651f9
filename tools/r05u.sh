# phase stamps of expand1x1 + pool3 + fire5/squeeze
set -u
cd "$GRAFT_REPO_ROOT"
ORE_LIB=onnx-rusty-inference-engine_amd/lib/exp/libore_pool_stamps.so timeout -k 10 180 python -u tools/pool_probe.py || exit 1
