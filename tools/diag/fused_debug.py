'''DIAGNOSTIC (GPU): batched point-mass solve with and without the fused IPM kernels, history diff'''
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from aircraft_trajectory_optimization_amd.raceline.batch_instances import perturbed_warm_starts
from aircraft_trajectory_optimization_amd.solver.batched_ipm import device_solver
from aircraft_trajectory_optimization_amd.solver.ipm import IPMOptions
from aircraft_trajectory_optimization_amd.tracks import make_spec
spec = make_spec(track='race', model='point', use_quat=False, N=10, K=3)
B = 4
W, LBW, UBW = perturbed_warm_starts(spec, B)
hs = []
for fused in (True, False):
    sol = device_solver(spec, B, LBW, UBW, IPMOptions(max_iter=int(sys.argv[1]) if len(sys.argv) > 1 else 8))
    if not fused:
        sol.vk = None
    r = sol.solve(W)
    hs.append(sol.history)
    print('fused' if fused else 'torch', r.status, r.iters, r.stats)
h0, h1 = hs
for i in range(min(len(h0), len(h1))):
    print(i, 'f', h0[i, 0, 0], h1[i, 0, 0], 'pr', h0[i, 1, 0], h1[i, 1, 0], 'du', h0[i, 2, 0], h1[i, 2, 0],
          'mu', h0[i, 3, 0], h1[i, 3, 0])
