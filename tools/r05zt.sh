set -u
cd "$GRAFT_REPO_ROOT"
bash tools/final_check.sh r05zt "$(cat gpurun_commit.txt 2>/dev/null || echo unknown)"
