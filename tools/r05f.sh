set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_wino_gpu.py tests/test_config4_gpu.py -k "not world2" -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread -rf > $OUT/pytest_r05f.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_r05f.log
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/ab_layers.sh r05f f32 base cur base cur > /dev/null 2>&1; grep -E "^\[|expand3x3" gpurun_out/ab_r05f.txt
