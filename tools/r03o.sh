#!/bin/bash
# r03o: leaf-kernel scalar trims (non-unrolled live scan, live counter, update from the pivot's tile)
# against the r03n library: KKT parity tests and factor timing
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03o
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03o] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03o] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
step pytest_kkt 300 python -u -m pytest tests/test_gpu_kkt.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed" $OUT/pytest_kkt.log | tail -2
for rep in 1 2; do
for b in 512 128; do
  step kkt_cur_b${b}_$rep 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_cur_b${b}_$rep.json
  ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_r03n.so step kkt_r03n_b${b}_$rep 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_r03n_b${b}_$rep.json
done
done
grep -H '"factor_ms"' $OUT/kkt_*.json
echo done
