#!/bin/bash
# r03i: full GPU tests, default bench, evaluation kernel trace + PMC traffic, Hessian unit-order A/B
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03i
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>: stop the session on crash-like exits
  local name=$1 secs=$2; shift 2
  echo "[r03i] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03i] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed" $OUT/pytest_gpu.log | tail -2
step hess_lf 120 python tools/bench_hess.py --batch 512
cat $OUT/hess_lf.log | tail -1
ATO_LONGFIRST_MAX_B=0 step hess_il 120 python tools/bench_hess.py --batch 512
cat $OUT/hess_il.log | tail -1
step evalprof 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/evalprof -o run -- python bench.py --no-solve --no-cpu-baseline --eval-steps 100
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-solve
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-solve
step mb_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/mb_fetch -o run -- ./tools/mb_store
step mb_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/mb_write -o run -- ./tools/mb_store
step bench 900 python bench.py
tail -c 3000 $OUT/bench.log
echo done
