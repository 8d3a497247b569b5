#!/bin/bash
# r03ab: leaf kernel scalar trims (branchless search keys, predicated factor-column store) against HEAD
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03ab
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03ab] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03ab] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
L=$PWD/tools/diag/_lib
for rep in 1 2; do
  step kkt_cur_$rep 200 python tools/bench_kkt.py --batch 512 --reps 7 --out $OUT/kkt_cur_$rep.json
  for v in tr; do
    ATO_LIB_PATH=$L/libato_$v.so step kkt_${v}_$rep 200 python tools/bench_kkt.py --batch 512 --reps 7 --out $OUT/kkt_${v}_$rep.json
  done
done
grep -H '"factor_ms"' $OUT/kkt_*.json
for v in tr; do
  ATO_LIB_PATH=$L/libato_$v.so step pmc_$v 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES --output-format csv -d $OUT/pmc_$v -o run -- python tools/bench_kkt.py --batch 512 --reps 2
done
echo done
step pmc_cur 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES --output-format csv -d $OUT/pmc_cur -o run -- python tools/bench_kkt.py --batch 512 --reps 2
