#!/bin/bash
# r03ae: full GPU tests, smoke and the default bench with the KKT solves deferred until the inertia passes are done
# bench's evaluation kernel, kernel trace of the KKT factor
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03ae
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03ae] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03ae] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed" $OUT/pytest_gpu.log | tail -2
step smoke 300 python -c 'import __graft_entry__ as g; g.smoke()'
tail -2 $OUT/smoke.log
step bench 900 python bench.py
tail -c 400 $OUT/bench.log
step evalprof 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/evalprof -o run -- python bench.py --no-solve --no-cpu-baseline
grep -o '"kernel_avg_us": [0-9.]*' $OUT/evalprof.log
grep k_eval_paired $OUT/evalprof/run_kernel_stats.csv | cut -d, -f2-4
echo done
