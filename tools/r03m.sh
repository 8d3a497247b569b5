#!/bin/bash
# r03m: KKT factor with lower-only extraction (layout-independent factors), 16-wide leaves above
# a batch threshold, one-wave three-tile fronts, side-stream class overlap: parity tests, factor
# timing A/B against HEAD's library, batched-solve A/B (200 iterations)
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03m
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03m] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03m] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
BASE=$PWD/tools/diag/_lib/libato_base.so

step pytest_kkt 300 python -u -m pytest tests/test_gpu_kkt.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed" $OUT/pytest_kkt.log | tail -2
for b in 512 256 128 64 1; do
  step kkt_cur_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_cur_b$b.json
  ATO_LIB_PATH=$BASE step kkt_base_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_base_b$b.json
done
for b in 512 256 128; do
  ATO_KKT_S16_MIN=1000000000 step kkt_nos16_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_nos16_b$b.json
  ATO_KKT_S16_MIN=1 step kkt_alls16_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_alls16_b$b.json
done

grep -H '"factor_ms"' $OUT/kkt_*.json
step kktprof 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kktprof -o run -- python tools/bench_kkt.py --batch 512 --reps 7
for v in base cur; do
  if [ $v = base ]; then lp=$BASE; else lp=; fi
  ATO_LIB_PATH=$lp step solve_$v 600 python tools/solve_batched.py --batch 512 --max-iter 200 --cold --no-host --out $OUT/solve_$v.json
  grep -o '"solve_s": [0-9.]*' $OUT/solve_$v.json
done
echo done
