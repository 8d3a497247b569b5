#!/bin/bash
# r03am: leaf kernel choice at small batches: 16-wide-tile kernel forced (ATO_KKT_S16_MIN=0) vs the
# default threshold (six-tile kernel below 1536 workgroups), factor timing
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03am
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03am] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03am] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
}
for b in 1 4 8 16 24 30; do
  step def_b$b 120 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/def_b$b.json
  ATO_KKT_S16_MIN=0 step s16_b$b 120 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/s16_b$b.json
done
grep -H '"factor_ms"' $OUT/*.json
echo done
