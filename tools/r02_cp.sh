set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for v in 1024 100000 1024 100000; do
  ORE_CONCAT_POOL_MIN_HW=$v timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-b1 --layers > gpurun_out/cp_$v.json 2> gpurun_out/cp_$v.err
  rc=$?; echo "min_hw $v rc=$rc $(cut -c100-190 gpurun_out/cp_$v.json)"
  case $rc in 0) ;; *) exit $rc;; esac
done
grep -v amdgpu.ids gpurun_out/cp_100000.err | grep "fire4\|pool3\|fire5/sq"
