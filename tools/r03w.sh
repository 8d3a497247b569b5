#!/bin/bash
# r03w: leaf row factors with the pivot-type branch hoisted (u1) against HEAD; default bench on HEAD
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03w
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03w] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03w] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
for rep in 1 2; do
  step kkt_cur_$rep 200 python tools/bench_kkt.py --batch 512 --reps 7 --out $OUT/kkt_cur_$rep.json
  ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_u1.so step kkt_u1_$rep 200 python tools/bench_kkt.py --batch 512 --reps 7 --out $OUT/kkt_u1_$rep.json
done
grep -H '"factor_ms"' $OUT/kkt_*.json
step kktprof 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kktprof -o run -- python tools/bench_kkt.py --batch 512 --reps 7
step bench 900 python bench.py
tail -c 600 $OUT/bench.log
echo done
