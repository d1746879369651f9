set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for sh in default 2,4 3,3 3,5 4,3 4,5; do
  if [ $sh = default ]; then unset ORE_FIRE_POOL_SHAPE; else export ORE_FIRE_POOL_SHAPE=$sh; fi
  timeout -k 10 200 python3 bench.py --precision f16 --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --layers > gpurun_out/fps.json 2> gpurun_out/fps.err
  rc=$?; echo "shape $sh rc=$rc $(cut -c100-175 gpurun_out/fps.json)"; [ $rc = 0 ] || exit $rc
  grep "+pool+" gpurun_out/fps.err
done
