set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/x3_accuracy.py > gpurun_out/x3_acc.json 2> gpurun_out/x3_acc.err
rc=$?; echo "acc rc=$rc"; cat gpurun_out/x3_acc.json; tail -3 gpurun_out/x3_acc.err
case $rc in 124|134|137|139) exit $rc;; esac
ORE_X3_SACC=1 timeout -k 10 300 python3 bench.py --precision f32x3 --steps 10 --warmup 2 --no-cpu-baseline --no-b1 --layers > gpurun_out/bench_x3s.json 2> gpurun_out/bench_x3s.err
rc=$?; echo "bench rc=$rc"; cut -c1-200 gpurun_out/bench_x3s.json; grep -v amdgpu.ids gpurun_out/bench_x3s.err | grep expand3x3
