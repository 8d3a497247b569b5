import sys, time
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
import numpy as np
from tests.helpers import HostEvaluator
from aircraft_trajectory_optimization_amd.solver.ipm import InteriorPointSolver, IPMOptions
from aircraft_trajectory_optimization_amd.tracks import make_spec, make_warm_spec
from aircraft_trajectory_optimization_amd.raceline.warmstart import drone_guess
N, K = 50, 4
kw = dict(track='fig8', frame='parametric', N=N, K=K, use_quat=True, global_r=True)
ps = make_spec(**{**kw, 'model': 'point', 'use_quat': False})
pev = HostEvaluator(ps)
pr = InteriorPointSolver(pev, ps.lbw, ps.ubw, pev.lbg, pev.ubg, IPMOptions(max_iter=500)).solve(ps.w0)
node = ps.N + np.arange(ps.P) * ps.nv
print('point', pr.status, pr.x[:N].sum(), 'y', pr.x[node+1].min(), pr.x[node+1].max(), 'n', pr.x[node+2].min(), pr.x[node+2].max())
yb = float(sys.argv[1])
L, U = ps.lbw.copy(), ps.ubw.copy()
L[node + 1], U[node + 1] = -yb, yb
pr = InteriorPointSolver(pev, L, U, pev.lbg, pev.ubg, IPMOptions(max_iter=500)).solve(ps.w0)
print('point narrowed', pr.status, pr.iters, pr.x[:N].sum())
spec = make_warm_spec(pr.x, **{**kw, 'use_dcm': sys.argv[2] == 'dcm'})
dn = spec.N + np.arange(spec.P) * spec.nv
spec.lbw[dn + 1], spec.ubw[dn + 1] = -yb, yb
ev = HostEvaluator(spec)
t = time.time()
r = InteriorPointSolver(ev, spec.lbw, spec.ubw, ev.lbg, ev.ubg, IPMOptions(max_iter=400)).solve(spec.w0)
print('RESULT', r.status, r.iters, r.x[:N].sum(), r.stats.get('restorations'), time.time() - t)
