import sys, numpy as np, torch
sys.path.insert(0, '.')
from aircraft_trajectory_optimization_amd.solver.ipm import IPMOptions
from aircraft_trajectory_optimization_amd.solver.batched_ipm import device_solver
from aircraft_trajectory_optimization_amd.tracks import make_spec
spec = make_spec(track='race', N=5, K=2)
B = 2
rng = np.random.default_rng(0)
W = np.repeat(spec.w0[None], B, axis=0)
W[1, :spec.N] *= 1 + 0.1 * rng.uniform(-1, 1, spec.N)
for rep in range(3):
    res = device_solver(spec, B, spec.lbw, spec.ubw, IPMOptions(max_iter=300)).solve(W)
    print(rep, res.status, [int(i) for i in res.iters], res.stats, float(res.x[:spec.N, 0].sum()), flush=True)
