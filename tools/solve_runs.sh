#!/bin/bash
# interior-point solves on the GPU evaluator (each step time-limited; stop at the first crash-like exit)
set -u
mkdir -p gpurun_out/solve
ONLY=${1:-}
run() {  # run <name> <seconds> <args...>
    local name=$1 secs=$2
    shift 2
    if [ -n "$ONLY" ] && [ "$ONLY" != "$name" ]; then return; fi
    timeout -k 10 "$secs" python tools/solve_one.py "$@" --out "gpurun_out/solve/$name.json" --verbose \
        > "gpurun_out/solve/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    case $rc in 0|1) ;; *) exit $rc ;; esac
}
run race_50x4_point 300 --model point --N 50 --K 4
run race_50x4_ws 600 --N 50 --K 4 --ws --max-iter 1000
run race_50x4_cold 600 --N 50 --K 4 --max-iter 1000
run fig8_50x7_cold 900 --track fig8 --N 50 --K 7 --max-iter 1000
run race_script_param_rk4_ws 1150 --N 70 --K 7 --rk4 --ws --max-iter 1000
run race_script_global_rk4_ws 1150 --frame global --N 70 --K 7 --rk4 --ws --max-iter 1000
