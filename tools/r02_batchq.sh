# per-layer time vs batch: wave-quantisation tails show as per-image time jumps
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for prec in f32 f16; do
for b in 128 192 224 256 320; do
  timeout -k 10 200 python3 bench.py --precision $prec --batch $b --steps 10 --warmup 2 --no-cpu-baseline --no-b1 --layers > gpurun_out/bq.json 2> gpurun_out/bq_${prec}_$b.err
  rc=$?; echo "$prec b=$b rc=$rc $(cut -c100-160 gpurun_out/bq.json)"; [ $rc = 0 ] || exit $rc
done
done
