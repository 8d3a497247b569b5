#!/bin/bash
# r03al: leaf factor in two phases (tiles left of S not updated once the pivots pass tile S),
# S = 6 and 7 against HEAD: KKT parity tests on the variant library and factor timing
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03al
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03al] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03al] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
}
L=$PWD/tools/diag/_lib
ATO_LIB_PATH=$L/libato_s6.so step pytest_kkt_s6 300 python -u -m pytest tests/test_gpu_kkt.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed" $OUT/pytest_kkt_s6.log | tail -2
for rep in 1 2; do
for b in 512 64; do
  step kkt_cur_b${b}_$rep 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_cur_b${b}_$rep.json
  for v in s6 s7; do
    ATO_LIB_PATH=$L/libato_$v.so step kkt_${v}_b${b}_$rep 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_${v}_b${b}_$rep.json
  done
done
done
grep -H '"factor_ms"' $OUT/kkt_*.json
echo done
