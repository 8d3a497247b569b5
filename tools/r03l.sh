#!/bin/bash
# r03l: 16-wide-tile leaf factor kernel + per-class level launches: KKT parity tests, then factor
# timing A/B (current, W=2 build, no 16-wide class, no class split) and a kernel trace
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03l
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03l] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03l] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
step pytest_kkt 300 python -u -m pytest tests/test_gpu_kkt.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed" $OUT/pytest_kkt.log | tail -2
for b in 512 64 1; do
  step kkt_cur_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_cur_b$b.json
  ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_w2.so step kkt_w2_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_w2_b$b.json
  ATO_KKT_S16=0 step kkt_nos16_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_nos16_b$b.json
  ATO_KKT_SPLIT=0 step kkt_nosplit_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_nosplit_b$b.json
done
grep -H '"factor_ms"' $OUT/kkt_*.json
step kktprof 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kktprof -o run -- python tools/bench_kkt.py --batch 512 --reps 7
ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_w2.so step kktprof_w2 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kktprof_w2 -o run -- python tools/bench_kkt.py --batch 512 --reps 7
echo done
