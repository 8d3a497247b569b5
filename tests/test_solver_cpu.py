'''
Host solver pieces on CPU (the evaluator here is the CPU build of the programs, test-only):
  * the block-tridiagonal KKT factorisation against a dense solve and dense eigenvalue inertia
  * the interior-point solver on a point-mass raceline: converges to a KKT point
    (IPOPT's optimality test), which is independent of how it got there
'''
import numpy as np
import pytest
import scipy.sparse as sp

from aircraft_trajectory_optimization_amd.solver.ipm import InteriorPointSolver, IPMOptions, _lower_to_full
from aircraft_trajectory_optimization_amd.solver.kkt_blocks import BlockKKT
from tests.helpers import HostEvaluator, product_spec, random_w, var_stages


@pytest.mark.parametrize('cfg', [dict(track='fig8', N=5, K=3), dict(track='race', frame='global', N=7, K=2),
                                 dict(track='race', N=7, K=2, rk4=True)],
                         ids=['fig8-colloc', 'race-global', 'race-rk4'])
def test_block_kkt_matches_dense(cfg):
    spec = product_spec(**cfg)
    ev = HostEvaluator(spec)
    rng = np.random.default_rng(0)
    w = random_w(spec, rng)
    _, _, _, jv = ev.eval(w)
    W = _lower_to_full(ev.nw, ev.h_row_ptr, ev.h_col, ev.hess(w, rng.standard_normal(ev.ng), 1.0))
    jr = np.repeat(np.arange(ev.ng), np.diff(ev.j_row_ptr))
    J = sp.csr_matrix((jv, (jr, ev.j_col)), shape=(ev.ng, ev.nw))
    D = np.abs(rng.standard_normal(ev.ng)) * 1e-3
    K = sp.bmat([[W + sp.diags(np.abs(rng.standard_normal(ev.nw))), J.T], [J, -sp.diags(D)]]).tocsc()
    bk = BlockKKT(ev.nw, ev.ng, var_stages(spec), ev.j_row_ptr, ev.j_col, ev.h_row_ptr, ev.h_col)
    fac, inertia = bk.factor(K)
    rhs = rng.standard_normal(ev.nw + ev.ng)
    Kd = K.toarray()
    x = fac.solve(rhs)
    assert np.abs(Kd @ x - rhs).max() <= 1e-8 * np.abs(rhs).max()
    eig = np.linalg.eigvalsh(Kd)
    assert inertia == ((eig > 0).sum(), (eig < 0).sum(), 0)


def test_ipm_point_mass_converges_to_kkt_point():
    spec = product_spec(track='race', model='point', use_quat=False, N=10, K=3)
    ev = HostEvaluator(spec)
    solver = InteriorPointSolver(ev, spec.lbw, spec.ubw, ev.lbg, ev.ubg, IPMOptions(max_iter=200))
    res = solver.solve(spec.w0)
    assert res.status == 'optimal', res.status
    # KKT certificate in unscaled quantities
    f, g, gf, jv = ev.eval(res.x)
    jr = np.repeat(np.arange(ev.ng), np.diff(ev.j_row_ptr))
    J = sp.csr_matrix((jv, (jr, ev.j_col)), shape=(ev.ng, ev.nw))
    viol = np.maximum(ev.lbg - g, 0) + np.maximum(g - ev.ubg, 0)
    assert viol.max() <= 1e-6
    assert np.all(res.x >= spec.lbw - 1e-12) and np.all(res.x <= spec.ubw + 1e-12)
    dual = gf + J.T @ res.lam_g + res.lam_x
    assert np.abs(dual).max() <= 1e-5 * max(1.0, np.abs(gf).max())
    lap = res.x[:spec.N].sum()
    assert 4.0 < lap < 7.0


def test_ipm_drone_with_point_mass_warm_start():
    ''' use_ws path (drone_raceline.py:158-274): point-mass solve, attitude / rate / thrust guess,
    then the quaternion drone NLP converges to an IPOPT-tolerance KKT point '''
    from aircraft_trajectory_optimization_amd.tracks import make_warm_spec
    kw = dict(track='fig8', frame='parametric', N=16, K=3)
    ps = product_spec(model='point', use_quat=False, **kw)
    pev = HostEvaluator(ps)
    pres = InteriorPointSolver(pev, ps.lbw, ps.ubw, pev.lbg, pev.ubg, IPMOptions(max_iter=300)).solve(ps.w0)
    assert pres.status == 'optimal'
    ds = make_warm_spec(pres.x, **kw)
    q = ds.w0[ds.N + 3:ds.N + 7]
    assert abs(np.linalg.norm(q) - 1) < 1e-12          # a proper rotation, not the cold-start (1,0,0,0) flip
    ev = HostEvaluator(ds)
    res = InteriorPointSolver(ev, ds.lbw, ds.ubw, ev.lbg, ev.ubg, IPMOptions(max_iter=300)).solve(ds.w0)
    assert res.status == 'optimal', res.status
    f, g, gf, jv = ev.eval(res.x)
    viol = np.maximum(ev.lbg - g, 0) + np.maximum(g - ev.ubg, 0)
    assert viol.max() <= 1e-6
    jr = np.repeat(np.arange(ev.ng), np.diff(ev.j_row_ptr))
    J = sp.csr_matrix((jv, (jr, ev.j_col)), shape=(ev.ng, ev.nw))
    dual = gf + J.T @ res.lam_g + res.lam_x
    assert np.abs(dual).max() <= 1e-5 * max(1.0, np.abs(gf).max())


def test_ipm_open_line_point_mass_starts_and_ends_at_rest():
    ''' open (non-periodic) line (A14): the point mass starts and ends at rest with vertical thrust
    (base_raceline.py:516-543, point_raceline.py:15-45) and the solve reaches a KKT point '''
    spec = product_spec(track='race', model='point', use_quat=False, N=10, K=3, closed=False)
    ev = HostEvaluator(spec)
    res = InteriorPointSolver(ev, spec.lbw, spec.ubw, ev.lbg, ev.ubg, IPMOptions(max_iter=300)).solve(spec.w0)
    assert res.status == 'optimal', res.status
    f, g, gf, jv = ev.eval(res.x)
    viol = np.maximum(ev.lbg - g, 0) + np.maximum(g - ev.ubg, 0)
    assert viol.max() <= 1e-6
    jr = np.repeat(np.arange(ev.ng), np.diff(ev.j_row_ptr))
    J = sp.csr_matrix((jv, (jr, ev.j_col)), shape=(ev.ng, ev.nw))
    dual = gf + J.T @ res.lam_g + res.lam_x
    assert np.abs(dual).max() <= 1e-5 * max(1.0, np.abs(gf).max())
    v0 = res.x[spec.col_z(0, 0, 3):spec.col_z(0, 0, 6)]
    assert np.linalg.norm(v0) <= 1e-3                    # |v_g|^2 <= 0 at the start
    u0 = res.x[spec.col_z(0, 0, 6):spec.col_z(0, 0, 8)]
    assert np.abs(u0).max() <= 1e-6                       # horizontal thrust components
