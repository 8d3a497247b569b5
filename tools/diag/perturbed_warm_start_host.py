import sys, time
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
import numpy as np
from tests.helpers import HostEvaluator
from aircraft_trajectory_optimization_amd.solver.ipm import InteriorPointSolver, IPMOptions
from aircraft_trajectory_optimization_amd.tracks import make_spec, make_warm_spec
from aircraft_trajectory_optimization_amd.raceline.batch_instances import perturbed_warm_starts
N, K, seed, dcm = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4] == 'dcm'
kw = dict(track='fig8', frame='parametric', N=N, K=K, use_quat=True, global_r=True)
ps = make_spec(**{**kw, 'model': 'point', 'use_quat': False})
pev = HostEvaluator(ps)
pr = InteriorPointSolver(pev, ps.lbw, ps.ubw, pev.lbg, pev.ubg, IPMOptions(max_iter=500)).solve(ps.w0)
spec = make_warm_spec(pr.x, **{**kw, 'use_dcm': dcm})
W, L, U = perturbed_warm_starts(spec, seed + 1, scale=float(sys.argv[5]) if len(sys.argv) > 5 else 1.0)
ev = HostEvaluator(spec)
t = time.time()
r = InteriorPointSolver(ev, L[seed], U[seed], ev.lbg, ev.ubg, IPMOptions(max_iter=400)).solve(W[seed])
print('RESULT', r.status, r.iters, r.x[:N].sum(), r.stats, time.time() - t)
