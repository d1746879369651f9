# Winograd persistent + phase offset A/B (timing only, ORE_LIB experiment builds)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in base wpp0 wpp1 wpp2 base; do
  if [ $v = base ]; then lib=""; else lib="onnx-rusty-inference-engine_amd/lib/exp/libore_$v.so"; fi
  ORE_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-b1 --no-f16-line --layers > gpurun_out/r05z1_$v.json 2> gpurun_out/r05z1_$v.err || { tail -5 gpurun_out/r05z1_$v.err; exit 1; }
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/r05z1_{v}.json").read().strip().splitlines()[-1])
lines = [l for l in open(f"gpurun_out/r05z1_{v}.err") if "expand3x3" in l]
print(f"[{v}] {d['value']:.0f} img/s {d['ms_per_step']} ms |", " | ".join(l.split()[0].split('/')[0] + " " + l.split()[2] for l in lines))
PY
done
