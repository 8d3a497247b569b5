"""
DIAGNOSTIC (CPU): solve accuracy of the saddle-front elimination against Bunch-Kaufman, both in
the test emulation (tests/kkt_emulation.py), on the KKT matrices of a single-instance racetrack
cold-start solve (every fifth factorisation): max |K x - b| / max |b| and the inertia of each.

    python tools/diag/saddle_accuracy.py SEED MAX_ITER N      e.g. 0 40 12
"""
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.helpers import product_spec, HostEvaluator, var_stages
from aircraft_trajectory_optimization_amd.raceline.instances import seeded_instances
from aircraft_trajectory_optimization_amd.solver.ipm import InteriorPointSolver, IPMOptions
from aircraft_trajectory_optimization_amd.solver.kkt_plan import collocation_saddle, build_plan
from tests.kkt_emulation import Factor
N = int(sys.argv[3]) if len(sys.argv) > 3 else 12
spec = product_spec(track='race', N=N, K=4)
ev = HostEvaluator(spec)
sad = collocation_saddle(spec.N, spec.K1, spec.nv, spec.nz, ev.ng, ev.j_row_ptr, ev.j_col)
st = var_stages(spec)
p0 = build_plan(ev.nw, ev.ng, st, ev.j_row_ptr, ev.j_col, ev.h_row_ptr, ev.h_col)
p1 = build_plan(ev.nw, ev.ng, st, ev.j_row_ptr, ev.j_col, ev.h_row_ptr, ev.h_col, saddle=sad)
W, L, U = seeded_instances(spec, [int(sys.argv[1])])
s = InteriorPointSolver(ev, L[0], U[0], ev.lbg, ev.ubg, IPMOptions(max_iter=int(sys.argv[2])))
orig = s._factor
n, m = ev.nw, ev.ng
jr = np.repeat(np.arange(m), np.diff(ev.j_row_ptr))
hr = np.repeat(np.arange(n), np.diff(ev.h_row_ptr))
rec = []
cnt = [0]
def fac(K):
    cnt[0] += 1
    if cnt[0] % 5 == 0:
        K = sp.csr_matrix(K)
        H = np.asarray(K[hr, ev.h_col]).ravel()
        dx = K.diagonal()[:n].copy()
        H = np.where(hr == ev.h_col, 0.0, H)      # diagonal goes to dx (H holds off-diagonals + its diag)
        Hd = np.asarray(K[hr, ev.h_col]).ravel()
        J = np.asarray(K[n + jr, ev.j_col]).ravel()
        dr = K.diagonal()[n:].copy()
        rhs = np.random.default_rng(cnt[0]).standard_normal(n + m)
        out = []
        for p in (p0, p1):
            f = Factor(p, H, J, dx, dr)
            x = f.solve(rhs)
            out.append((np.abs(K @ x - rhs).max() / np.abs(rhs).max(), f.inertia, len(getattr(f, 'sad', {}))))
        rec.append(out)
        print(cnt[0], out, flush=True)
    return orig(K)
s._factor = fac
r = s.solve(W[0])
print(r.status, r.iters)
