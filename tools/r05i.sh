set -u
cd "$GRAFT_REPO_ROOT"
bash tools/ab_layers.sh r05i f32 cur stag2 stag4 stag6 cur stag2 stag4 stag6 > /dev/null 2>&1; rc=$?; echo "ab rc=$rc"; grep -E "^\[|conv1" gpurun_out/ab_r05i.txt
