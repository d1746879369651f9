set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_model_gpu.py -k "pool_expand or pool_squeeze" tests/test_parity_attrib_gpu.py -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread -rf > $OUT/pytest_r05c.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest_r05c.log | tail -30
case $rc in 0|1) ;; *) exit $rc;; esac
for t in on off on2 off2; do f=""; case $t in off*) f="--fusion 6119";; esac; timeout -k 10 300 python3 tools/bench_layers.py $f --tag $t 2>&1 | grep -v amdgpu.ids | grep -E "^\[|pool|expand1x1" >> $OUT/layers_r05c.txt || exit 1; done; cat $OUT/layers_r05c.txt
