#!/bin/bash
# r03 GPU session: all GPU tests, the default bench (batched SQP + eval roofline), rocprof of the eval
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_obstacles.py tests/test_gpu_batched_ipm.py tests/test_gpu_api.py tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 
rc=$?
if [ $rc -ne 0 ]; then
  echo "tests rc=$rc"; grep -E "^(FAILED|ERROR)|^E " $OUT/pytest_gpu.log | head -40
  case $rc in 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
fi
tail -3 $OUT/pytest_gpu.log
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
tail -c 3000 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-solve --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
find $OUT -name '*_trace.csv' -delete
echo done
