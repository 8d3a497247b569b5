#!/bin/bash
# r03an: 16-wide-tile leaf kernel from 4 x CUs workgroups (was 6 x CUs): full GPU tests, smoke,
# default bench
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03an
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03an] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03an] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
grep -E "passed|failed" $OUT/pytest_gpu.log | tail -2
step smoke 300 python -c 'import __graft_entry__ as g; g.smoke()'
step bench 900 python bench.py
tail -c 300 $OUT/bench.log
echo done
