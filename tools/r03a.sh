set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r03a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03a/pytest_gpu.log 2>&1 || { echo "tests rc=$?"; exit 1; }
timeout -k 10 900 python -u tools/solve_batched.py --batch 512 --max-iter 1000 --no-host --cold --out gpurun_out/r03a/solve_cold_b512.json > gpurun_out/r03a/solve_cold.log 2>&1; echo "solve rc=$?"
