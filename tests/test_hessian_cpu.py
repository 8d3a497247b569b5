'''
Hessian of the Lagrangian (sigma grad^2 f + sum_i lam_i grad^2 g_i), CPU build of the same
programs (tests/native/hostcheck.cpp) against the oracle: Hessian-vector products by central
differences of the oracle's complex-step Lagrangian gradient (truncation O(eps^2) ~ 1e-8
relative at eps = 1e-5, so the tolerance is 1e-6 relative), and the structure covers every
second derivative the oracle sees.
'''
import numpy as np
import pytest

from tests.helpers import HostCheck, oracle_nlp, product_spec, random_w, sym_dense

CASES = [
    dict(track='race', N=4, K=2),
    dict(track='fig8', N=3, K=3, use_quat=False),
    dict(track='race', N=4, K=2, global_r=False),
    dict(track='race', frame='global', N=7, K=2),
    dict(track='race', frame='global', N=7, K=2, use_quat=False),
    dict(track='race', model='point', use_quat=False, N=4, K=2),
    dict(track='race', model='point', frame='global', use_quat=False, N=7, K=2),
    dict(track='race', N=7, K=2, rk4=True),
    dict(track='race', frame='global', N=7, K=2, rk4=True),
    dict(track='fig8', N=4, K=3, quat_flip=True),
    dict(track='race', N=4, K=3, closed=False),
    dict(track='race', frame='global', N=6, K=2, use_quat=False, closed=False),
    dict(track='race', model='point', use_quat=False, N=4, K=2, closed=False),
]


def _id(c):
    return '-'.join(f'{k}={v}' for k, v in c.items())


@pytest.mark.parametrize('cfg', CASES, ids=_id)
def test_hessian_vector_products(cfg):
    rng = np.random.default_rng(5)
    spec = product_spec(**cfg)
    nlp = oracle_nlp(**cfg)
    hc = HostCheck(spec.native_spec())
    rp, col, nc = hc.hess_pattern()
    assert nc >= 1 and rp[-1] == len(col)
    w = random_w(nlp, rng)
    lam = rng.standard_normal(hc.ng)
    sigma = 0.7
    H = sym_dense(rp, col, hc.hess(w, lam, sigma)[0], hc.nw)
    V = rng.standard_normal((hc.nw, 2))
    ref = nlp.hvp(w, lam, sigma, V)
    np.testing.assert_allclose(H @ V, ref, rtol=0, atol=1e-6 * max(1.0, np.abs(ref).max()))


def test_hessian_structure_covers_oracle():
    ''' every column of the finite-difference Hessian lies inside the analysed pattern '''
    cfg = dict(track='race', N=3, K=2)
    rng = np.random.default_rng(9)
    spec = product_spec(**cfg)
    nlp = oracle_nlp(**cfg)
    hc = HostCheck(spec.native_spec())
    rp, col, _ = hc.hess_pattern()
    P = sym_dense(rp, col, np.ones(len(col)), hc.nw) != 0
    w = random_w(nlp, rng)
    lam = rng.standard_normal(hc.ng)
    Hfd = nlp.hvp(w, lam, 1.0, np.eye(hc.nw))
    scale = np.abs(Hfd).max()
    assert np.abs(Hfd[~P]).max() <= 1e-6 * scale


def test_hessian_objective_only():
    ''' lam = 0: sigma grad^2 f, the input-cost block h_n B_k (R + R^T) and its h coupling '''
    cfg = dict(track='race', N=4, K=2)
    rng = np.random.default_rng(2)
    spec = product_spec(**cfg)
    nlp = oracle_nlp(**cfg)
    hc = HostCheck(spec.native_spec())
    rp, col, _ = hc.hess_pattern()
    w = random_w(nlp, rng)
    H = sym_dense(rp, col, hc.hess(w, np.zeros(hc.ng), 2.0)[0], hc.nw)
    V = rng.standard_normal((hc.nw, 1))
    ref = nlp.hvp(w, np.zeros(hc.ng), 2.0, V)
    np.testing.assert_allclose(H @ V, ref, rtol=0, atol=1e-9 * max(1.0, np.abs(ref).max()))
