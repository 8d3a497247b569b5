'''
Independent optimality pin of the interior-point solver (SURVEY 8(c) pins 5-6): the solution it
returns is checked with the ORACLE's NLP functions only (oracle/ref_transcription.py, itself pinned
to the reference's own transcription), not with the product's evaluator:
  * first order: primal feasibility, the stationarity of the Lagrangian (complex-step gradient of
    f + lam^T g) and complementarity, in unscaled quantities;
  * second order: the Hessian of the Lagrangian (central differences of the oracle's exact
    Lagrangian gradient) is positive definite on the null space of the active constraints'
    Jacobian, i.e. x is a strict local minimiser, not just a KKT point.
IPOPT itself cannot run here, so lap-time parity with it is unpinned; a KKT point
with positive-definite reduced Hessian is what IPOPT's own termination certifies. (scipy's
trust-constr and SLSQP were tried as cross-solvers on these problems and stalled: xtol
termination far from any KKT point, incompatible QP subproblems.)
'''
import numpy as np
import pytest

from aircraft_trajectory_optimization_amd.solver.ipm import InteriorPointSolver, IPMOptions
from tests.helpers import HostEvaluator, kkt_certificate, oracle_nlp, product_spec


# unscaled (the solver, like IPOPT, converges in gradient-scaled rows: a row scaled by 1e-2 meets the
# scaled tolerance 1e-8 at 1e-6 unscaled); IPOPT's own unscaled defaults are looser (constr_viol_tol 1e-4, dual_inf_tol 1, compl_inf_tol 1e-4,
# on top of tol = 1e-8 for the scaled overall error)
TOL = {'primal': 1e-5, 'dual': 1e-6, 'compl': 1e-6}


def _solve(spec, w0=None, lbw=None, ubw=None, max_iter=600):
    ev = HostEvaluator(spec)
    lbw = spec.lbw if lbw is None else lbw
    ubw = spec.ubw if ubw is None else ubw
    return InteriorPointSolver(ev, lbw, ubw, ev.lbg, ev.ubg, IPMOptions(max_iter=max_iter)).solve(
        spec.w0 if w0 is None else w0)


def reduced_hessian_eigs(nlp, x, lam_g, lam_x, lbw, ubw, act_tol=1e-7):
    ''' eigenvalues of Z^T (grad^2 L) Z, Z spanning the null space of the active constraints '''
    J = nlp.jac_dense(x)
    eq = nlp.lbg == nlp.ubg
    active = eq | (np.abs(lam_g) > act_tol)
    rows = [J[active]]
    bnd = (np.abs(lam_x) > act_tol) | (np.asarray(lbw) == np.asarray(ubw))
    if bnd.any():
        E = np.zeros((int(bnd.sum()), nlp.nw))
        E[np.arange(E.shape[0]), np.nonzero(bnd)[0]] = 1.0
        rows.append(E)
    A = np.concatenate(rows)
    _, sv, Vt = np.linalg.svd(A)
    rank = int((sv > 1e-9 * sv[0]).sum())
    Z = Vt[rank:].T
    if Z.shape[1] == 0:
        return np.array([np.inf]), 0
    HZ = nlp.hvp(x, lam_g, 1.0, Z, eps=1e-5)
    R = Z.T @ HZ
    return np.linalg.eigvalsh((R + R.T) / 2), Z.shape[1]


@pytest.mark.parametrize('cfg', [dict(track='race', model='point', use_quat=False, N=6, K=3),
                                 dict(track='fig8', model='point', use_quat=False, N=8, K=2)],
                         ids=['race-point', 'fig8-point'])
def test_point_mass_solution_is_a_strict_local_minimum(cfg):
    spec = product_spec(**cfg)
    res = _solve(spec)
    assert res.status == 'optimal'
    nlp = oracle_nlp(**cfg)
    c = kkt_certificate(nlp, res.x, res.lam_g, res.lam_x, spec.lbw, spec.ubw)
    assert c['primal'] <= TOL['primal'] and c['dual'] <= TOL['dual'] and c['compl'] <= TOL['compl'], c
    eig, dim = reduced_hessian_eigs(nlp, res.x, res.lam_g, res.lam_x, spec.lbw, spec.ubw)
    assert dim > 0 and eig.min() > 0, (dim, eig[:5])


def test_drone_warm_start_solution_is_a_strict_local_minimum():
    from aircraft_trajectory_optimization_amd.tracks import make_warm_spec
    kw = dict(track='race', frame='parametric', N=6, K=3)
    pspec = product_spec(model='point', use_quat=False, **kw)
    pres = _solve(pspec)
    assert pres.status == 'optimal'
    spec = make_warm_spec(pres.x, **kw)
    res = _solve(spec)
    assert res.status == 'optimal'
    nlp = oracle_nlp(quat_flip=spec.quat_flip, **kw)
    c = kkt_certificate(nlp, res.x, res.lam_g, res.lam_x, spec.lbw, spec.ubw)
    assert c['primal'] <= TOL['primal'] and c['dual'] <= TOL['dual'] and c['compl'] <= TOL['compl'], c
    eig, dim = reduced_hessian_eigs(nlp, res.x, res.lam_g, res.lam_x, spec.lbw, spec.ubw)
    assert dim > 0 and eig.min() > 0, (dim, eig[:5])
