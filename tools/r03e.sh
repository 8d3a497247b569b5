#!/bin/bash
# r03e: config-5 parity (fig-8 fp32, B = 8192) + its bench line and kernel trace; solve pass statistics
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03e
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>: stop the session on crash-like exits
  local name=$1 secs=$2; shift 2
  echo "[r03e] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03e] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
step config5 300 python -u -m pytest tests/test_gpu_config5.py -m gpu -x -v -s --timeout 240 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed|Error|worst" $OUT/config5.log | tail -5
step bench_c5 200 python bench.py --no-solve --no-cpu-baseline --track fig8 --dtype f32 --batch 8192 --eval-steps 50
tail -c 700 $OUT/bench_c5.log
step prof_c5 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- python bench.py --no-solve --no-cpu-baseline --track fig8 --dtype f32 --batch 8192 --eval-steps 50
step bench_c5_f64 200 python bench.py --no-solve --no-cpu-baseline --track fig8 --dtype f64 --batch 8192 --eval-steps 30
tail -c 400 $OUT/bench_c5_f64.log
ATO_IPM_PROFILE=1 step solve 600 python tools/solve_batched.py --batch 512 --max-iter 1000 --no-host --cold --out $OUT/laps.json
tail -c 300 $OUT/solve.log
echo done
