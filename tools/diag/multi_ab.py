'''
Per-instance comparison of the line search's batched backtracking (BatchedInteriorPoint.LS_MULTI_K) against
the trial-by-trial loop on config-3 cold starts, several solves in one process: statuses, iteration counts and
laps per instance, so that a difference can be told from run-to-run variation (the asynchronous restoration
phases are collected when they finish).
    python tools/diag/multi_ab.py --batch 128 --ks 0 8 0 8 --out gpurun_out/x.json
'''
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=128)
    ap.add_argument('--max-iter', type=int, default=1000)
    ap.add_argument('--ks', type=int, nargs='+', default=[0, 8, 0, 8])
    ap.add_argument('--async-phases', type=int, default=None)
    ap.add_argument('--out', required=True)
    a = ap.parse_args()
    import numpy as np
    import torch
    from aircraft_trajectory_optimization_amd.raceline.batched_solve import solve_shard
    from aircraft_trajectory_optimization_amd.solver.batched_ipm import BatchedInteriorPoint
    from aircraft_trajectory_optimization_amd.solver.ipm import IPMOptions
    from aircraft_trajectory_optimization_amd.tracks import make_spec
    if a.async_phases is not None:
        BatchedInteriorPoint.ASYNC_PHASES = a.async_phases
    spec = make_spec(track='race', model='drone', frame='parametric', N=50, K=4, use_quat=True, global_r=True)
    runs = []
    for k in a.ks:
        BatchedInteriorPoint.LS_MULTI_K = k
        t0 = time.time()
        res, solver, _ = solve_shard(spec, list(range(a.batch)), IPMOptions(max_iter=a.max_iter))
        torch.cuda.synchronize()
        dt = time.time() - t0
        laps = res.x[:spec.N].sum(0).cpu().numpy()
        runs.append({'k': k, 'seconds': dt, 'status': list(res.status), 'iters': [int(i) for i in res.iters],
                     'laps': laps.tolist(), 'ls_trials': solver.stats.get('ls_trials'),
                     'ls_multi': solver.stats.get('ls_multi')})
        print(f'K={k}: {dt:.1f} s', {s: res.status.count(s) for s in sorted(set(res.status))},
              'sum it', sum(runs[-1]['iters']), 'ls', runs[-1]['ls_trials'], runs[-1]['ls_multi'], flush=True)
        solver.kkt.close()
        del solver
        torch.cuda.empty_cache()
    base = runs[0]
    for r in runs[1:]:
        d = [b for b in range(a.batch) if r['iters'][b] != base['iters'][b] or r['status'][b] != base['status'][b]]
        dl = max((abs(r['laps'][b] - base['laps'][b]) for b in range(a.batch) if b not in d), default=0.0)
        print(f'K={r["k"]} vs K={base["k"]}: {len(d)} instances differ in status / iterations {d[:20]}, '
              f'max lap difference elsewhere {dl:.3e}', flush=True)
    json.dump(runs, open(a.out, 'w'))


if __name__ == '__main__':
    main()
