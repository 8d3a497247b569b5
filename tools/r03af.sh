#!/bin/bash
# r03af: time split (ATO_IPM_PROFILE laps) and kernel trace of a 200-iteration cold solve on HEAD
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03af
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03af] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03af] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
ATO_IPM_PROFILE=1 step solvelaps 600 python tools/solve_batched.py --batch 512 --max-iter 200 --cold --no-host --out $OUT/solvelaps.json
step solveprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/solveprof -o run -- python tools/solve_batched.py --batch 512 --max-iter 200 --cold --no-host --out $OUT/solveprof.json
echo done
