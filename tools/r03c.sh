#!/bin/bash
# r03 profiling: time split of the cold-start batched solve, its kernel trace, eval timing check
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03c
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>: stop the session on crash-like exits
  local name=$1 secs=$2; shift 2
  echo "[r03c] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03c] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
step evalcheck 200 python bench.py --no-solve --no-cpu-baseline
tail -c 1500 $OUT/evalcheck.log
step api 300 python -u -m pytest tests/test_gpu_api.py -m gpu -q -s --timeout 280 --timeout-method thread -p no:cacheprovider
grep -E "warm start|passed|failed" $OUT/api.log
ATO_IPM_PROFILE=1 step laps 600 python tools/solve_batched.py --batch 512 --max-iter 1000 --no-host --cold --out $OUT/laps.json
step solveprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/solveprof -o run -- python tools/solve_batched.py --batch 512 --max-iter 300 --no-host --cold --out $OUT/solveprof.json
echo done
