# Winograd L2 prefetch of a later tile group's first chunks (timing only)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_layers.sh r05zk f32 cur pf32 pf64 pf128 cur
