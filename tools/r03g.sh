#!/bin/bash
# r03g: evaluation-kernel unit orders (time and FETCH per launch)
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03g
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>: stop the session on crash-like exits
  local name=$1 secs=$2; shift 2
  echo "[r03g] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03g] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
for o in class interval longfirst interval class longfirst; do
  ATO_UNIT_ORDER=$o step eval_$o 120 python bench.py --no-solve --no-cpu-baseline --eval-steps 100
  grep -o '"kernel_avg_us": [0-9.]*' $OUT/eval_$o.log
  cp $OUT/eval_$o.log $OUT/eval_${o}_$(date +%s%N).log
done
for o in interval longfirst; do
  ATO_UNIT_ORDER=$o step pmc_$o 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_$o -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-solve
done
for o in interval longfirst; do
  ATO_UNIT_ORDER=$o step b4096_$o 120 python bench.py --no-solve --no-cpu-baseline --batch 4096 --eval-steps 30
  grep -o '"kernel_avg_us": [0-9.]*' $OUT/b4096_$o.log
done
echo done
