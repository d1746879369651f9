set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r05g.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke_r05g.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 400 --timeout-method thread -rf > $OUT/pytest_gpu_r05g.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu_r05g.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python3 bench.py > $OUT/bench_r05g.json 2> $OUT/bench_r05g.err; rc=$?; echo "bench rc=$rc"; head -c 400 $OUT/bench_r05g.json; echo
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof_r05g" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-b1 --no-f16-line > "$GRAFT_REPO_ROOT/$OUT/prof_bench_r05g.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof_r05g.err"; rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 tools/split_batch_probe.py --splits 1 2 4 1 2 > $OUT/split_r05g.txt 2>&1; rc=$?; echo "split rc=$rc"; grep splits $OUT/split_r05g.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_layers.sh r05g f32 base cur base cur > /dev/null 2>&1; grep -E "^\[|conv1" gpurun_out/ab_r05g.txt
