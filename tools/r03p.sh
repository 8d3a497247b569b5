#!/bin/bash
# r03p: SQ counters of the KKT factor kernels (instruction mix and wait states), B = 512
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03p
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "[r03p] $(date +%T) $name"
  timeout -s KILL "$secs" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[r03p] $name rc=$rc"
  case $rc in 0) ;; 124|137|134|139|136|135) echo "crash-like exit: stopping"; exit $rc ;; esac
  find $OUT \( -name '*_trace.csv' -o -name '*.db' \) -delete 2>/dev/null
}
step listpmc 60 rocprofv3 -L
pick() { local r=""; for c in "$@"; do grep -qw "$c" $OUT/listpmc.log && r="$r $c"; done; echo $r; }
A=$(pick SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY)
B=$(pick SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU)
echo "A: $A"; echo "B: $B"
step pmc_a 90 rocprofv3 --pmc $A --output-format csv -d $OUT/pmc_a -o run -- python tools/bench_kkt.py --batch 512 --reps 2
step pmc_b 90 rocprofv3 --pmc $B --output-format csv -d $OUT/pmc_b -o run -- python tools/bench_kkt.py --batch 512 --reps 2
echo done
