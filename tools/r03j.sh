#!/bin/bash
# r03j: evaluation-kernel event timing (events without the system fence) against the kernel trace
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03j
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03j] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03j] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
step evalprof 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/evalprof -o run -- python bench.py --no-solve --no-cpu-baseline
grep -o '"kernel_avg_us": [0-9.]*' $OUT/evalprof.log
grep k_eval_paired $OUT/evalprof/run_kernel_stats.csv | cut -d, -f2-4
step eval 120 python bench.py --no-solve --no-cpu-baseline
grep -o '"kernel_avg_us": [0-9.]*' $OUT/eval.log
step evalprof4096 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/evalprof4096 -o run -- python bench.py --no-solve --no-cpu-baseline --batch 4096 --eval-steps 30
grep -o '"kernel_avg_us": [0-9.]*' $OUT/evalprof4096.log
grep k_eval_paired $OUT/evalprof4096/run_kernel_stats.csv | cut -d, -f2-4
echo done
