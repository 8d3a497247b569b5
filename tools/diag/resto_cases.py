'''
DIAGNOSTIC ONLY: batched vs single-instance solves of race N=5, K=2 cold starts (the
restoration test problem) for a few perturbation seeds.   python tools/diag/resto_cases.py (GPU)
'''
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), 'tests'))


def main():
    from test_gpu_batched_ipm import _host_solve
    from aircraft_trajectory_optimization_amd.solver.ipm import IPMOptions
    from aircraft_trajectory_optimization_amd.solver.batched_ipm import device_solver
    from aircraft_trajectory_optimization_amd.tracks import make_spec
    spec = make_spec(track='race', N=5, K=2)
    opts = IPMOptions(max_iter=300)
    r = _host_solve(spec, spec.w0, spec.lbw, spec.ubw, opts)
    print('host w0', r.status, r.iters, r.x[:spec.N].sum(), r.stats, flush=True)
    for seed in range(4):
        rng = np.random.default_rng(seed)
        W = np.repeat(spec.w0[None], 3, axis=0)
        W[1, :spec.N] *= 1 + 0.1 * rng.uniform(-1, 1, spec.N)
        W[2, :spec.N] *= 1 + 0.1 * rng.uniform(-1, 1, spec.N)
        res = device_solver(spec, 3, spec.lbw, spec.ubw, opts).solve(W)
        print('seed', seed, res.status, [int(i) for i in res.iters], res.stats,
              [float(res.x[:spec.N, b].sum()) for b in range(3)], flush=True)
        for b in (1, 2):
            h = _host_solve(spec, W[b], spec.lbw, spec.ubw, opts)
            print('   host', b, h.status, h.iters, h.x[:spec.N].sum(), h.stats.get('restorations'), flush=True)


if __name__ == '__main__':
    main()
