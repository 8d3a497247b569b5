#!/bin/bash
# r03aa: leaf update without tile guards (two row groups) as the default; the same for the generic
# kernel (wnoskip) at B = 512, 64, 1; KKT parity tests
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03aa
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03aa] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03aa] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
L=$PWD/tools/diag/_lib
step pytest_kkt 300 python -u -m pytest tests/test_gpu_kkt.py tests/test_gpu_batched_ipm.py::test_batched_device_restoration_follows_single_instance -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed" $OUT/pytest_kkt.log | tail -2
for b in 512 64 1; do
  step kkt_cur_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_cur_b$b.json
  ATO_LIB_PATH=$L/libato_wnoskip.so step kkt_wnoskip_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --out $OUT/kkt_wnoskip_b$b.json
done
grep -H '"factor_ms"' $OUT/kkt_*.json
echo done
