#!/bin/bash
# r03d: blocked interval-leaf factor kernel -- bitwise A/B tests, factor timing A/B, cold solve A/B, kernel trace
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03d
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>: stop the session on crash-like exits
  local name=$1 secs=$2; shift 2
  echo "[r03d] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03d] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
ATO_UNIT_ORDER=class step eval_class 200 python bench.py --no-solve --no-cpu-baseline
tail -c 600 $OUT/eval_class.log
step eval_interval 200 python bench.py --no-solve --no-cpu-baseline
tail -c 600 $OUT/eval_interval.log
ATO_UNIT_ORDER=class step pmc_fetch_class 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_class -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-solve
step pmc_fetch_interval 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_interval -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-solve
step pmc_write_interval 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_interval -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-solve
step mb_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/mb_fetch -o run -- ./tools/mb_store
step mb_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/mb_write -o run -- ./tools/mb_store
step kkt_tests 300 python -u -m pytest tests/test_gpu_kkt.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed|Error" $OUT/kkt_tests.log | tail -5
for B in 512 64 1; do
  ATO_KKT_BLOCKED=0 step kkt_w_$B 120 python tools/bench_kkt.py --batch $B --reps 7
  tail -1 $OUT/kkt_w_$B.log
  ATO_KKT_BLOCKED=1 step kkt_b_$B 120 python tools/bench_kkt.py --batch $B --reps 7
  tail -1 $OUT/kkt_b_$B.log
done
step kkt_prof 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kkt_prof -o run -- python tools/bench_kkt.py --batch 512 --reps 7
ATO_KKT_BLOCKED=1 step solve_b 600 python tools/solve_batched.py --batch 512 --max-iter 1000 --no-host --cold --out $OUT/laps_b.json
tail -3 $OUT/solve_b.log
echo done
