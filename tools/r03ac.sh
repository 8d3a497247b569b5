#!/bin/bash
# r03ac: instruction mix (SQ counters) of every kernel of a short cold-start batched solve
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03ac
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03ac] $(date +%T) $name"
  timeout -s KILL "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03ac] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
}
step pmc 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES --output-format csv -d $OUT/pmc -o run -- python tools/solve_batched.py --batch 512 --max-iter 25 --cold --no-host --out $OUT/solve.json
python tools/diag/pmc_summary.py $OUT/pmc/run_counter_collection.csv 30 > $OUT/pmc_summary.txt
rm -f $OUT/pmc/run_counter_collection.csv
cat $OUT/pmc_summary.txt
echo done
