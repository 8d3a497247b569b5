#!/bin/bash
# r03x: kernel trace of a 200-iteration cold-start batched solve on HEAD (where the GPU time goes now)
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03x
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03x] $(date +%T) $name"
  timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03x] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
step solveprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/solveprof -o run -- python tools/solve_batched.py --batch 512 --max-iter 200 --cold --no-host --out $OUT/solveprof.json
echo done
