set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for st in 1 2 1 2; do
timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-b1 --no-step-timing --streams $st > gpurun_out/st_$st.json 2> gpurun_out/st_$st.err
rc=$?; echo "streams $st rc=$rc $(cut -c100-190 gpurun_out/st_$st.json)"
case $rc in 0) ;; *) exit $rc;; esac
done
