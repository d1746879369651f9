# PMC passes over the bench with the band walker (the layer table's mfma% / lds / waits)
set -u
cd "$GRAFT_REPO_ROOT"
PMC_COMMIT=661450a bash tools/pmc.sh r05t_f32 || exit $?
