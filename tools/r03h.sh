#!/bin/bash
# r03h: fp32 quad-store writer -- parity (fp32 vs fp64 and goldens) and A/B against the paired writer
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03h
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>: stop the session on crash-like exits
  local name=$1 secs=$2; shift 2
  echo "[r03h] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03h] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
step tests 300 python -u -m pytest tests/test_gpu_config5.py tests/test_gpu_parity.py tests/test_gpu_golden.py -m gpu -x -v -s --timeout 240 --timeout-method thread -p no:cacheprovider -k "config5 or fp32 or f32 or full_size or paired"
grep -E "passed|failed|Error|worst" $OUT/tests.log | tail -5
for r in 1 2; do
  step c5_quad_$r 120 python bench.py --no-solve --no-cpu-baseline --track fig8 --dtype f32 --batch 8192 --eval-steps 50
  grep -o '"kernel_avg_us": [0-9.]*' $OUT/c5_quad_$r.log
  ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_pairf32.so step c5_pair_$r 120 python bench.py --no-solve --no-cpu-baseline --track fig8 --dtype f32 --batch 8192 --eval-steps 50
  grep -o '"kernel_avg_us": [0-9.]*' $OUT/c5_pair_$r.log
done
step b512_quad 120 python bench.py --no-solve --no-cpu-baseline --dtype f32 --eval-steps 100
grep -o '"kernel_avg_us": [0-9.]*' $OUT/b512_quad.log
ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_pairf32.so step b512_pair 120 python bench.py --no-solve --no-cpu-baseline --dtype f32 --eval-steps 100
grep -o '"kernel_avg_us": [0-9.]*' $OUT/b512_pair.log
step prof_c5 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- python bench.py --no-solve --no-cpu-baseline --track fig8 --dtype f32 --batch 8192 --eval-steps 50
for B in 512 1024 2048 4096; do
  step lf_b$B 120 python bench.py --no-solve --no-cpu-baseline --batch $B --eval-steps 60
  grep -o '"kernel_avg_us": [0-9.]*' $OUT/lf_b$B.log
  ATO_LONGFIRST_MAX_B=0 step il_b$B 120 python bench.py --no-solve --no-cpu-baseline --batch $B --eval-steps 60
  grep -o '"kernel_avg_us": [0-9.]*' $OUT/il_b$B.log
done
for v in gradfirst links5; do
  for B in 512 4096; do
    ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_$v.so step ${v}_b$B 120 python bench.py --no-solve --no-cpu-baseline --batch $B --eval-steps 60
    grep -o '"kernel_avg_us": [0-9.]*' $OUT/${v}_b$B.log
  done
done
echo done
