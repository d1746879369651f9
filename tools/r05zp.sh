# Winograd LDS kernel prologue split by a stamp before the first stage's DMAs (timing only)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ORE_LIB=$PWD/onnx-rusty-inference-engine_amd/lib/exp/libore_stampsp.so timeout -k 10 300 python3 -u tools/stamps.py --tag stamps_prologue > gpurun_out/r05zp_stamps.txt 2>&1 || { tail -20 gpurun_out/r05zp_stamps.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r05zp_stamps.txt
