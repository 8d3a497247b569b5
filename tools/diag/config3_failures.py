'''
Where the config-3 instances that do not converge spend their iterations: the
bench workload (racetrack 50 x 4 cold starts, seeds 0..B-1, IPOPT's max_iter 1000) solved on the device,
then per instance -- from the solver's per-instance counters (BatchedInteriorPoint.per_instance) and its
last history row -- restoration phases and the iterations inside them, watchdog starts / reverts, soft
restoration steps, KKT failures (no direction), filter resets, and the final barrier parameter, scaled
optimality error and primal / dual infeasibility. Instances are put into failure classes; JSON out.

    python tools/diag/config3_failures.py --batch 512 --out gpurun_out/diag/c3_failures.json
'''
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def classify(row):
    ''' the failure class of a non-converged instance (first match) '''
    it = max(row['iterations'], 1)
    if row['resto_iterations'] >= 0.5 * it:
        return 'restoration-bound (>= half the iterations inside restoration phases)'
    if row['E0'] <= 1e-6:
        return 'stalled near a KKT point (E0 <= 1e-6, not converged to tol)'
    if row['mu'] > 1e-4:
        return 'barrier not decreased (mu > 1e-4 at the end)'
    if row['watchdog_reverted'] >= 10:
        return 'watchdog cycling (>= 10 reverts)'
    return 'slow progress (none of the above)'


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=512)
    ap.add_argument('--max-iter', type=int, default=1000)
    ap.add_argument('--opts', default='{}', help='IPMOptions overrides (JSON)')
    ap.add_argument('--out', default='')
    a = ap.parse_args()
    import torch
    from aircraft_trajectory_optimization_amd.raceline.batched_solve import solve_shard
    from aircraft_trajectory_optimization_amd.solver.ipm import IPMOptions
    from aircraft_trajectory_optimization_amd.tracks import make_spec
    spec = make_spec(track='race', model='drone', frame='parametric', N=50, K=4, use_quat=True, global_r=True)
    t0 = time.perf_counter()
    res, solver, _ = solve_shard(spec, list(range(a.batch)),
                                 IPMOptions(**{**json.loads(a.opts), 'max_iter': a.max_iter}))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    pi = solver.per_instance
    last = solver.history[-1]                     # [f, inf_pr, inf_du, mu, E0, restorations][instance]
    rows = []
    for b, st in enumerate(res.status):
        r = {'seed': b, 'status': st, 'iterations': int(res.iters[b]), 'mu': float(last[3, b]), 'E0': float(last[4, b]),
             'inf_pr': float(last[1, b]), 'inf_du': float(last[2, b])}
        for k, v in pi.items():
            r[k] = int(v[b])
        rows.append(r)
    groups = {}
    for r in rows:
        groups.setdefault(r['status'], []).append(r)
    keys = ['iterations', 'restorations', 'resto_iterations', 'watchdog_started', 'watchdog_reverted',
            'soft_resto_steps', 'kkt_failures', 'filter_resets']
    summary = {}
    for st, rs in sorted(groups.items()):
        summary[st] = {'count': len(rs), **{k: {'median': float(np.median([r[k] for r in rs])),
                                               'mean': float(np.mean([r[k] for r in rs]))} for k in keys}}
    fail = [r for r in rows if r['status'] not in ('optimal', 'acceptable')]
    classes = {}
    for r in fail:
        c = classify(r)
        r['class'] = c
        classes.setdefault(c, []).append(r['seed'])
    out = {'batch': a.batch, 'max_iter': a.max_iter, 'options': json.loads(a.opts), 'solve_s': dt,
           'statuses': {k: len(v) for k, v in groups.items()}, 'by_status': summary,
           'failure_classes': {k: {'count': len(v), 'seeds': v} for k, v in classes.items()},
           'failed': fail}
    txt = json.dumps(out, indent=1)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or '.', exist_ok=True)
        with open(a.out, 'w', encoding='utf-8') as fh:
            fh.write(txt)
    print(json.dumps({k: out[k] for k in ('statuses', 'solve_s')}))
    for st, v in summary.items():
        print(st, json.dumps(v))
    for k, v in classes.items():
        print(f'{len(v):4d}  {k}')


if __name__ == '__main__':
    main()
