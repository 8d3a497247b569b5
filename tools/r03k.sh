#!/bin/bash
# r03k: HEAD check after the container rebuild: full GPU tests and the default bench
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03k
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>: stop the session on crash-like exits
  local name=$1 secs=$2; shift 2
  echo "[r03k] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03k] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed" $OUT/pytest_gpu.log | tail -2
step bench 900 python bench.py
tail -c 3000 $OUT/bench.log
echo done
