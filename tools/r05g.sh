#!/bin/bash
# round-5 GPU session: re-run the failed GPU tests, the config-5 solve, the saddle-front threshold A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05g}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_batched_ipm.py tests/test_gpu_scripts.py tests/test_gpu_solve_config5.py \
    -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "${SEL:-config3_full or solve_b8192}" > $OUT/pytest_sel.log 2>&1
rc=$?
echo "pytest rc=$rc" | tee -a $OUT/steps.log
case $rc in 124|134|137|139|135|136) exit $rc ;; esac
exit 0
