set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_model_gpu.py -k "pool_expand or pool_squeeze" -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread -rf > $OUT/pytest_r05d.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest_r05d.log | tail -10
case $rc in 0|1) ;; *) exit $rc;; esac
: > $OUT/ab_r05d.txt
for t in on off on off; do f=""; [ $t = off ] && f="--fusion 6119"; timeout -k 10 300 python3 bench.py --no-b1 --no-cpu-baseline --no-f16-line --steps 40 $f > $OUT/b.json 2>/dev/null || exit 1; python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$t', d['value'], d['ms_per_step'])" >> $OUT/ab_r05d.txt; done; cat $OUT/ab_r05d.txt
