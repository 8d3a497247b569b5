#!/bin/bash
# r03ak: kernel statistics of a 200-iteration cold batched solve on HEAD (where the GPU time goes now)
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03ak
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/solveprof -o run -- python tools/solve_batched.py --batch 512 --max-iter 200 --cold --no-host --out $OUT/solveprof.json > $OUT/solveprof.log 2>&1
rc=$?
echo "solveprof rc=$rc"
find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
exit $rc
