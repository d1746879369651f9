# pool3 + e1 + squeeze: start offset for part of the first resident round (timing only)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_layers.sh r05zm f32 cur ps2 ps3 ps5 psh3 cur
