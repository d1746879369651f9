set -u
cd "$GRAFT_REPO_ROOT"
bash tools/final_check.sh r05k 452fc59
