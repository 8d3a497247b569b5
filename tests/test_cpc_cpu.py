'''
CPC gate progress (config 5's formulation beside the DCM pose; build-side, Foehn et al. 2021).
PARITY UNPINNED: the reference only displays a CPC trajectory loaded from CSV
(drone3d/utils/cpc_utils.py:14-101, scripts/fig_8_cpc.py:22-26); no reference code states the
progress NLP, so the product's segment programs (the CPU build of the kernels' code) are checked
against the oracle's numpy restatement of the same rows (oracle/ref_transcription.py, `cpc`), and the
guess is checked to satisfy the rows it is built to satisfy.

Rows (global frame, after all other node rows): per node q, complementarity
mu_j (|p_q - w_j|^2 - nu_j) = 0, order lambda_j - lambda_{j+1} <= 0, progress
lambda_{q+1,j} - lambda_{q,j} + mu_{q,j} = 0; one total time (every h equal); no gate rows.
'''
import numpy as np
import pytest

from tests.helpers import HostCheck, csr_dense, oracle_nlp, product_spec, random_w

CASES = [dict(track='fig8', frame='global', N=8, K=3, use_dcm=True),
         dict(track='fig8', frame='global', N=8, K=2),
         dict(track='fig8', frame='global', N=8, K=1, rk4=True, use_dcm=True),
         dict(track='race', frame='global', N=7, K=2, model='point', use_quat=False)]
IDS = ['dcm-colloc', 'esp-colloc', 'dcm-rk4', 'point']


def _pair(cfg, tol=0.3):
    spec = product_spec(**cfg, cpc={'waypoints': None, 'tol': tol})
    nlp = oracle_nlp(**cfg, cpc=spec.cpc)
    return spec, nlp


def _point(spec, rng):
    w = random_w(spec, rng)
    c0 = spec.cpc_off
    M = spec.cpc_m
    blk = w[c0:].reshape(spec.P, 3, M)
    blk[:, 0] = rng.random((spec.P, M))                      # lambda
    blk[:, 1] = rng.random((spec.P, M))                      # mu
    blk[:, 2] = rng.random((spec.P, M)) * spec.cpc['tol'] ** 2
    w[c0:] = blk.reshape(-1)
    return w


@pytest.mark.parametrize('cfg', CASES, ids=IDS)
def test_cpc_programs_match_oracle(cfg):
    spec, nlp = _pair(cfg)
    hc = HostCheck(spec.native_spec())
    assert (hc.nw, hc.ng) == (nlp.nw, nlp.ng) == (spec.nw, nlp.ng)
    np.testing.assert_array_equal(hc.lbg, nlp.lbg)
    np.testing.assert_array_equal(hc.ubg, nlp.ubg)
    rng = np.random.default_rng(3)
    W = np.stack([_point(spec, rng) for _ in range(3)])
    g, J, f, gf = hc.eval(W)
    for b in range(len(W)):
        go = nlp.g(W[b])
        np.testing.assert_allclose(g[b], go, rtol=0, atol=1e-12 * max(1.0, np.abs(go).max()))
        Jo = nlp.jac_dense(W[b])
        np.testing.assert_allclose(csr_dense(hc.row_ptr, hc.col, J[b], hc.ng, hc.nw), Jo, rtol=0,
                                   atol=1e-12 * max(1.0, np.abs(Jo).max()))
        assert abs(f[b] - nlp.f(W[b])) <= 1e-12 * max(1.0, abs(nlp.f(W[b])))
        np.testing.assert_allclose(gf[b], nlp.grad_f(W[b]), rtol=0, atol=1e-12 * max(1.0, np.abs(gf[b]).max()))


def test_cpc_hessian_matches_oracle():
    ''' the bilinear complementarity rows in the Hessian of the Lagrangian (seeded dual passes) '''
    from tests.helpers import sym_dense
    cfg = CASES[0]
    spec, nlp = _pair(cfg)
    hc = HostCheck(spec.native_spec())
    rng = np.random.default_rng(5)
    w = _point(spec, rng)
    lam = rng.standard_normal(hc.ng)
    rp, col, _ = hc.hess_pattern()
    H = sym_dense(rp, col, hc.hess(w, lam, 0.7)[0], hc.nw)
    V = rng.standard_normal((hc.nw, 3))
    HV = nlp.hvp(w, lam, 0.7, V)
    np.testing.assert_allclose(H @ V, HV, rtol=0, atol=1e-6 * max(1.0, np.abs(HV).max()))


def test_cpc_layout_and_guess():
    ''' one total time, no gate rows, the progress block after the node variables; the guess passes
    every waypoint in order, satisfies the progress and order rows exactly and the complementarity
    rows wherever the guessed path comes within tol of its waypoint '''
    spec, nlp = _pair(CASES[0], tol=10.0)
    assert spec.gates == [] and spec.phase_len == spec.N
    M, P = spec.cpc_m, spec.P
    assert M == 8 and spec.nw == spec.N + P * spec.nv + P * 3 * M
    blk = spec.w0[spec.cpc_off:].reshape(P, 3, M)
    lam, mu, nu = blk[:, 0], blk[:, 1], blk[:, 2]
    assert (lam[0] == 1).all() and (lam[-1] == 0).all()
    assert (np.diff(lam, axis=0) <= 0).all() and (mu.sum(0) == 1).all()
    np.testing.assert_array_equal(lam[1:] - lam[:-1] + mu[:-1], 0.0)          # progress rows
    assert (lam[:, :-1] - lam[:, 1:] <= 0).all()                               # order rows
    pos = np.array([spec.w0[spec.col_z(q // spec.K1, q % spec.K1):][:3] for q in range(P)])
    d2 = ((pos[:, None, :] - spec.cpc['waypoints'][None]) ** 2).sum(-1)
    assert np.abs(mu * (d2 - nu)).max() <= 1e-12                               # complementarity
    c = slice(spec.cpc_off, None)
    assert (spec.lbw[c] <= spec.w0[c]).all() and (spec.w0[c] <= spec.ubw[c]).all()


def test_cpc_refuses_parametric_frame():
    with pytest.raises(NotImplementedError):
        product_spec(track='fig8', N=8, K=3, cpc={'waypoints': None})
