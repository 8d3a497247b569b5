#!/bin/bash
# r03q: row groups of the 16-wide-tile Schur update (NG = 4 current, 2, 3) against r03n
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03q
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03q] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03q] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
}
step pytest_kkt 300 python -u -m pytest tests/test_gpu_kkt.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed" $OUT/pytest_kkt.log | tail -2
for rep in 1 2; do
  step kkt_cur_$rep 200 python tools/bench_kkt.py --batch 512 --reps 7 --out $OUT/kkt_cur_$rep.json
  for v in ng2 ng3 r03n; do
    ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_$v.so step kkt_${v}_$rep 200 python tools/bench_kkt.py --batch 512 --reps 7 --out $OUT/kkt_${v}_$rep.json
  done
done
grep -H '"factor_ms"' $OUT/kkt_*.json
echo done
