set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --layers > gpurun_out/g1_wino.json 2> gpurun_out/g1_wino.err
rc=$?; echo "wino rc=$rc"; cut -c1-400 gpurun_out/g1_wino.json; grep -v amdgpu.ids gpurun_out/g1_wino.err | grep "expand3x3\|conv1 \|total"
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --no-winograd > gpurun_out/g1_direct.json 2> gpurun_out/g1_direct.err
rc=$?; echo "direct rc=$rc"; cut -c1-300 gpurun_out/g1_direct.json
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --fusion 0 --layers > gpurun_out/g1_wino_f0.json 2> gpurun_out/g1_wino_f0.err
rc=$?; echo "wino fusion0 rc=$rc"; cut -c1-300 gpurun_out/g1_wino_f0.json
