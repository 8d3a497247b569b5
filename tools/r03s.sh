#!/bin/bash
# r03s: restoration-test seeds on the new factor; the rest of the GPU tests; solve time split; bench
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03s
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03s] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03s] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
step seeds 300 python -u tools/diag/resto_seeds.py
cat $OUT/seeds.log | grep seed
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_batched_ipm.py::test_batched_device_restoration_follows_single_instance
grep -E "passed|failed" $OUT/pytest_gpu.log | tail -2
ATO_IPM_PROFILE=1 step solvelaps 600 python tools/solve_batched.py --batch 512 --max-iter 200 --cold --no-host --out $OUT/solvelaps.json
step bench 900 python bench.py
tail -c 600 $OUT/bench.log
echo done
