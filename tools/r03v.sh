#!/bin/bash
# r03v: switch-dispatched column extraction in the 16-wide-tile leaf kernel against r03r: KKT
# tests, factor timing, SALU / VALU / branch counts of the leaf kernel; restoration test at IPOPT's max_iter
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03v
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03v] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03v] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
step pytest_kkt 300 python -u -m pytest tests/test_gpu_kkt.py tests/test_gpu_batched_ipm.py::test_batched_device_restoration_follows_single_instance -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed" $OUT/pytest_kkt.log | tail -2
for rep in 1 2; do
  step kkt_cur_$rep 200 python tools/bench_kkt.py --batch 512 --reps 7 --out $OUT/kkt_cur_$rep.json
  ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_r03u.so step kkt_r03u_$rep 200 python tools/bench_kkt.py --batch 512 --reps 7 --out $OUT/kkt_r03u_$rep.json
  ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_y.so step kkt_y_$rep 200 python tools/bench_kkt.py --batch 512 --reps 7 --out $OUT/kkt_y_$rep.json
done
for b in 1 64; do
  step kkt_cur_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_cur_b$b.json
  ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_r03u.so step kkt_r03u_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_r03u_b$b.json
done
grep -H '"factor_ms"' $OUT/kkt_*.json
step pmc_cur 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES --output-format csv -d $OUT/pmc_cur -o run -- python tools/bench_kkt.py --batch 512 --reps 2
ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_r03u.so step pmc_r03u 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES --output-format csv -d $OUT/pmc_r03u -o run -- python tools/bench_kkt.py --batch 512 --reps 2
echo done
