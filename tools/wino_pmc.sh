# rocprofv3 counter passes over tools/wino_one.py (one kernel); usage: bash tools/wino_pmc.sh TAG [wino_one args]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; shift
OUT="$ROOT/gpurun_out/wpmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $GROUP --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$ROOT/tools/${WPMC_SCRIPT:-wino_one.py}" "$@" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i [$GROUP] rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done < "$ROOT/tools/${WPMC_GROUPS:-wino_pmc_groups.txt}"
exit 0
