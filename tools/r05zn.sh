# Winograd LDS kernel phase stamps with the store drain (timing only, tools/patches/wino_stamps_drain.patch)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ORE_LIB=$PWD/onnx-rusty-inference-engine_amd/lib/exp/libore_stamps.so timeout -k 10 300 python3 -u tools/stamps.py --tag stamps_drain > gpurun_out/r05zn_stamps.txt 2>&1 || { tail -20 gpurun_out/r05zn_stamps.txt; exit 1; }
cat gpurun_out/r05zn_stamps.txt
