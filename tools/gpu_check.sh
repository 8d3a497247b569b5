#!/bin/bash
# GPU session script for gpurun: parity tests, smoke, bench, rocprof kernel trace.
# Each GPU step has its own time limit; the script stops at the first crash-like exit
# (abort / segfault / timeout / kill) and otherwise records failures and continues.
# Usage: tools/gpu_check.sh <tag> [steps...]   steps: tests smoke bench prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
shift || true
STEPS=${*:-tests smoke bench prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
status=0

run() {  # run <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    echo "[gpu_check] $(date +%T) start $name" | tee -a "$OUT/steps.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[gpu_check] $(date +%T) end $name rc=$rc" | tee -a "$OUT/steps.log"
    # keep the summaries only: full traces would push gpurun_out/ past its 64 MiB copy-back limit
    find "$OUT" \( -name '*_trace.csv' -o -name '*.db' -o -name '*.rocpd' \) -delete 2>/dev/null
    case $rc in
        0) ;;
        124|137|134|139|136|135) echo "[gpu_check] crash-like exit, stopping" | tee -a "$OUT/steps.log"; exit $rc ;;
        *) status=$rc ;;
    esac
}

for s in $STEPS; do
    case $s in
        tests) run pytest_gpu 1000 python -u -m pytest tests -m gpu --maxfail=6 -v --capture=sys --timeout 300 --timeout-method thread -p no:cacheprovider ${GPU_TESTS:-} ;;
        ab)    run ab_new 900 python -u tools/solver_ab.py --what fig8,config3 --tag new --out "$OUT/ab_new.json"
               # the baseline arm needs the round-4 tree in tools/r04_baseline (git- and gpurun-ignored, so absent
               # on a fresh box): without it the arm would import the current package and compare new with new
               if [ -d tools/r04_baseline/aircraft_trajectory_optimization_amd ]; then
                   PYTHONPATH=$PWD/tools/r04_baseline run ab_r04 900 python -u tools/solver_ab.py --what fig8,config3 --tag r04 --out "$OUT/ab_r04.json"
               else
                   echo "[gpu_check] ab: tools/r04_baseline missing, baseline arm not run" | tee -a "$OUT/steps.log"; status=2
               fi ;;
        abl)   i=0
               for o in ${AB_ARMS:-'{}' '{"soft_resto_pderror_reduction_factor": 0}' '{"constr_mult_reset_threshold": 1000}' \
                        '{"soft_resto_pderror_reduction_factor": 0, "constr_mult_reset_threshold": 1000}'}; do
                   i=$((i+1))
                   ATO_AB_OPTS="$o" run abl_$i 900 python -u tools/solver_ab.py --what ${AB_WHAT:-fig8,fig8k4,config3} --tag "$o" --out "$OUT/abl_$i.json"
               done ;;
        sadtau) for t in 0 1e2 1e4 1e6; do
                   ATO_KKT_SADDLE_TAU=$t run kkt_sad_tau$t 200 python tools/bench_kkt.py --batch 512 --reps 5 --saddle 1 --out "$OUT/kkt_sad_tau$t.json"
               done
               run kkt_bk 200 python tools/bench_kkt.py --batch 512 --reps 5 --saddle 0 --out "$OUT/kkt_bk.json"
               for t in 1e2 1e4; do
                   ATO_KKT_SADDLE=1 ATO_KKT_SADDLE_TAU=$t run c3_sad_tau$t 600 python -u tools/solver_ab.py --what config3 --tag "saddle tau $t" --out "$OUT/c3_sad_tau$t.json"
               done ;;
        bench5solve) run bench5_dcm_solve 1100 python -u bench.py --track fig8 --pose dcm --batch ${B5:-8192} --max-iter ${B5_MAXIT:-150} --no-cpu-baseline --progress 20 ;;
        jtyab) run pytest_jty 200 python -u -m pytest tests/test_gpu_ipm_kernels.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k js_jty
               for v in 0 1; do
                   ATO_IPM_FUSED_JTY=$v run solve_jty$v 600 python tools/solve_batched.py --batch 512 --max-iter 1000 --cold --no-host --out "$OUT/solve_jty$v.json"
               done ;;
        bench5j32) run bench5_dcm_jac32 1100 python -u bench.py --track fig8 --pose dcm --batch ${B5:-8192} --max-iter ${B5_MAXIT:-150} --jac32 --tol 1e-6 --no-cpu-baseline --progress 20 ;;
        bench4) run bench4_obstacles 900 python bench.py --track obstacles --batch 512 --no-cpu-baseline ;;
        abnew) run ab_new 900 python -u tools/solver_ab.py --what ${AB_WHAT:-fig8,config3} --tag new --out "$OUT/ab_new.json" ;;
        smoke) run smoke 300 python -c 'import __graft_entry__ as g; g.smoke()' ;;
        bench) run bench 900 python bench.py ;;
        bench32) run bench_f32 300 python bench.py --steps 50 --warmup 10 --dtype f32 --no-cpu-baseline --no-solve ;;
        benchim) run bench_im 300 python bench.py --steps 50 --warmup 10 --layout instance --no-cpu-baseline --no-solve ;;
        benchbig) run bench_b4096 300 python bench.py --steps 20 --warmup 5 --batch 4096 --no-cpu-baseline --no-solve ;;
        prof)  run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
                   python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-solve ;;
        pmc)   run pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
                   python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-solve
               run pmc_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
                   python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-solve ;;
        pmcsq) run pmc_sq 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
                   SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d "$OUT/pmc_sq" -o run -- \
                   python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-solve
               run pmc_tcc 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmc_tcc" -o run -- \
                   python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-solve ;;
        kkt)   run kkt_b512 200 python tools/bench_kkt.py --batch 512 --out "$OUT/kkt_b512.json"
               run kkt_b64 200 python tools/bench_kkt.py --batch 64 --out "$OUT/kkt_b64.json"
               run kkt_b1 200 python tools/bench_kkt.py --batch 1 --out "$OUT/kkt_b1.json"
               run kkt_chain_b512 200 python tools/bench_kkt.py --batch 512 --ordering chain --out "$OUT/kkt_chain_b512.json"
               run kkt_chain_b1 200 python tools/bench_kkt.py --batch 1 --ordering chain --out "$OUT/kkt_chain_b1.json" ;;
        ipmtests) run pytest_ipm 600 python -u -m pytest tests/test_gpu_batched_ipm.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
        kktvar) for v in $(ls tools/diag/_lib/libato_*.so | grep -v stamps); do
                   n=$(basename "$v" .so)
                   for b in 512 1; do
                       ATO_LIB_PATH=$PWD/$v run "kkt_${n}_b$b" 200 python tools/bench_kkt.py --batch $b --reps 7 --out "$OUT/kkt_${n}_b$b.json"
                   done
               done
               for b in 512 1; do run kkt_cur_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --out "$OUT/kkt_cur_b$b.json"; done ;;
        evalvar) for v in $(ls tools/diag/_lib/libato_*.so | grep -v stamps); do
                   n=$(basename "$v" .so)
                   ATO_LIB_PATH=$PWD/$v run "bench_$n" 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-solve
               done
               run bench_cur 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-solve ;;
        kktphase) ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_stamps.so run kkt_phase 120 python tools/diag/kkt_phase.py
               ATO_PHASE_B=512 ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_stamps.so run kkt_phase512 120 python tools/diag/kkt_phase.py ;;
        kktab) for b in 512 64 1; do
                   ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_base.so run kkt_base_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --out "$OUT/kkt_base_b$b.json"
                   run kkt_cur_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --out "$OUT/kkt_cur_b$b.json"
               done ;;
        sadab) for b in 512 64 1; do
                   run kkt_bk_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --saddle 0 --out "$OUT/kkt_bk_b$b.json"
                   run kkt_sad_b$b 200 python tools/bench_kkt.py --batch $b --reps 7 --saddle 1 --out "$OUT/kkt_sad_b$b.json"
               done ;;
        sadphase) ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_stamps.so run saddle_phase 120 python tools/diag/saddle_phase.py
               ATO_PHASE_B=1 ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_stamps.so run saddle_phase_b1 120 python tools/diag/saddle_phase.py ;;
        sadprof) run saddle_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/saddle_prof" -o run -- \
                   python tools/bench_kkt.py --batch 512 --reps 5 --saddle 1 --out "$OUT/saddle_prof.json" ;;
        solvesad) for v in 0 1; do
                   ATO_KKT_SADDLE=$v run solve_sad$v 600 python tools/solve_batched.py --batch 512 --max-iter 1000 --cold --no-host --out "$OUT/solve_sad$v.json"
               done ;;
        cpc5)  run bench5_cpc_f32 300 python bench.py --track fig8 --pose dcm --cpc --dtype f32 --batch 8192 --no-solve --no-cpu-baseline --eval-steps 50
               run bench5_cpc_f64 300 python bench.py --track fig8 --pose dcm --cpc --dtype f64 --batch 8192 --no-solve --no-cpu-baseline --eval-steps 50
               run prof5_cpc 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof5_cpc" -o run -- \
                   python bench.py --track fig8 --pose dcm --cpc --dtype f32 --batch 8192 --no-solve --no-cpu-baseline --eval-steps 30 ;;
        kktq)  run kkt_b512 200 python tools/bench_kkt.py --batch 512 --out "$OUT/kkt_b512.json"
               run kkt_b1 200 python tools/bench_kkt.py --batch 1 --out "$OUT/kkt_b1.json" ;;
        ipmktests) run pytest_ipmk 300 python -u -m pytest tests/test_gpu_ipm_kernels.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ;;
        kkttests) run pytest_kkt 300 python -u -m pytest tests/test_gpu_kkt.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ;;
        solve) run solve_b512 600 python tools/solve_batched.py --batch 512 --max-iter 200 --no-host --out "$OUT/solve_b512.json" ;;
        solveprof) run solveprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/solveprof" -o run -- \
                   python tools/solve_batched.py --batch 512 --max-iter 60 --no-host --out "$OUT/solveprof.json" ;;
        solvelaps) ATO_IPM_PROFILE=1 run solvelaps 600 python tools/solve_batched.py --batch 512 --max-iter 60 --no-host --out "$OUT/solvelaps.json" ;;
        solvelaps200) ATO_IPM_PROFILE=1 run solvelaps200 600 python tools/solve_batched.py --batch 512 --max-iter 200 --no-host --out "$OUT/solvelaps200.json" ;;
        solveab) for v in base cur base cur; do
                   if [ $v = base ]; then lp=$PWD/tools/diag/_lib/libato_base.so; else lp=; fi
                   ATO_LIB_PATH=$lp run solve_$v 600 python tools/solve_batched.py --batch 512 --max-iter 200 --no-host --out "$OUT/solve_$v.json"
                   cp "$OUT/solve_$v.json" "$OUT/solve_${v}_$(date +%s).json"
               done ;;
        config5) run pytest_config5 600 python -u -m pytest tests/test_gpu_config5.py -x -v -s --timeout 400 --timeout-method thread -p no:cacheprovider ;;
        bench5) run bench5_dcm_f32 300 python bench.py --track fig8 --pose dcm --dtype f32 --batch 8192 --no-solve --no-cpu-baseline --eval-steps 50
               run bench5_dcm_f64 300 python bench.py --track fig8 --pose dcm --dtype f64 --batch 8192 --no-solve --no-cpu-baseline --eval-steps 50
               run bench5_esp_f32 300 python bench.py --track fig8 --pose esp --dtype f32 --batch 8192 --no-solve --no-cpu-baseline --eval-steps 50 ;;
        prof5) run prof5 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof5" -o run -- \
                   python bench.py --track fig8 --pose dcm --dtype f32 --batch 8192 --no-solve --no-cpu-baseline --eval-steps 30 ;;
        solvelapscold) ATO_IPM_PROFILE=1 run solvelaps_cold 600 python tools/solve_batched.py --batch 512 --max-iter 200 --cold --no-host --out "$OUT/solvelaps_cold.json" ;;
        solveprofnd) HIP_ENABLE_DEFERRED_LOADING=0 run solveprof_cold_nodefer 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/solveprof_cold_nodefer" -o run -- \
                   python tools/solve_batched.py --batch 512 --max-iter 200 --cold --no-host --out "$OUT/solveprof_cold_nodefer.json" ;;
        solveprofcold) run solveprof_cold 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/solveprof_cold" -o run -- \
                   python tools/solve_batched.py --batch 512 --max-iter 200 --cold --no-host --out "$OUT/solveprof_cold.json" ;;
        s16ab) i=0
               for v in 1536 1024 1536 1024; do
                   i=$((i+1))
                   ATO_KKT_S16_MIN=$v run solve_s16min${v}_$i 600 python tools/solve_batched.py --batch 512 --max-iter 200 --cold --no-host --out "$OUT/solve_s16min${v}_$i.json"
               done ;;
        opcount) run opcount_device 300 python tools/diag/ipm_opcount.py --device -v ;;
        c5ab)  run c5_dcm 600 python -u tools/solve_config5.py --batch ${B5:-1024} --out "$OUT/c5_dcm.json"
               ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_dcmPm.so run c5_dcm_Pmodel 600 python -u tools/solve_config5.py --batch ${B5:-1024} --out "$OUT/c5_dcm_Pmodel.json" ;;
        c5esp) run c5_esp 600 python -u tools/solve_config5.py --batch ${B5:-1024} --pose esp --out "$OUT/c5_esp.json" ;;
        cpcsolve) run cpc_dcm 500 python -u tools/solve_cpc.py --batch ${BC:-64} --out "$OUT/cpc_dcm.json"
               run cpc_esp 500 python -u tools/solve_cpc.py --batch ${BC:-64} --pose esp --out "$OUT/cpc_esp.json" ;;
        listpmc) run listpmc 120 rocprofv3 -L ;;
        mb)    run mb_store 120 ./tools/mb_store ;;
        tileab) for t in 0 8 16 4; do
                    ATO_EVAL_TILE=$t run eval_tile${t}_b4096 300 python bench.py --steps 20 --warmup 5 --batch 4096 --no-cpu-baseline --no-solve --eval-steps 30
                done
                ATO_EVAL_TILE=8 ATO_EVAL_TILE_LF=0 run eval_tile8im_b4096 300 python bench.py --steps 20 --warmup 5 --batch 4096 --no-cpu-baseline --no-solve --eval-steps 30
                for t in 0 8; do
                    ATO_EVAL_TILE=$t run eval_tile${t}_f32_b8192 300 python bench.py --track fig8 --pose dcm --dtype f32 --batch 8192 --no-solve --no-cpu-baseline --eval-steps 50
                done ;;
        c3ab)  for v in base cur; do
                   if [ $v = base ]; then lp=$PWD/tools/diag/_lib/libato_base.so; else lp=; fi
                   ATO_LIB_PATH=$lp ATO_KKT_SPECULATE=0 run pytest_c3_$v 300 python -u -m pytest tests/test_gpu_batched_ipm.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider -k config3_full
               done ;;
        hessab) ATO_LIB_PATH=$PWD/tools/diag/_lib/libato_base.so run hess_base 200 python tools/diag/hess_ab.py "$OUT/hess_base.npz"
                run hess_cur 200 python tools/diag/hess_ab.py "$OUT/hess_cur.npz"
                ATO_HESS_MASK=1 run hess_mask 200 python tools/diag/hess_ab.py "$OUT/hess_mask.npz" ;;
        c3b128) run solve_c3_b128 300 python tools/solve_batched.py --batch 128 --max-iter 1000 --cold --no-host --out "$OUT/solve_c3_b128.json" ;;
        nanab) for v in base cur; do
                   if [ $v = base ]; then lp=$PWD/tools/diag/_lib/libato_base.so; else lp=; fi
                   ATO_LIB_PATH=$lp ATO_DEBUG_HESS_NONFINITE=1 run solve_nan_$v 300 python tools/solve_batched.py --batch 64 --max-iter 1000 --cold --no-host --out "$OUT/solve_nan_$v.json"
               done ;;
        pmctile) for t in 0 8; do
                   ATO_EVAL_TILE=$t run pmc_fetch_tile$t 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_tile$t" -o run -- \
                       python bench.py --steps 10 --warmup 3 --batch 4096 --no-cpu-baseline --no-solve --eval-steps 10
                done ;;
        scripts) run pytest_scripts 900 python -u -m pytest tests/test_gpu_scripts.py -x -v -s --timeout 800 --timeout-method thread -p no:cacheprovider ;;
        mbscale) run mb_store_scale 120 ./tools/mb_store_scale
               run bench_b4096 300 python bench.py --steps 20 --warmup 5 --batch 4096 --no-cpu-baseline --no-solve --eval-steps 30 ;;
        mbpmc) run mb_fetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/mb_fetch" -o run -- ./tools/mb_store
               run mb_write 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/mb_write" -o run -- ./tools/mb_store ;;
        units) for k in 0 1 2 3 4 12 34; do
                   export ATO_DEBUG_UNITS=$k
                   run bench_units$k 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-solve
                   unset ATO_DEBUG_UNITS
               done ;;
        *) echo "unknown step $s" ;;
    esac
done
exit $status
