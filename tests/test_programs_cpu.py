'''
CPU check of the C++ segment programs (compiled for the host by the test-only harness
tests/native/hostcheck.cpp) against the oracle: row count, lbg/ubg, g, dense Jacobian,
f and grad f, for every model / frame / attitude variant the library supports.
The same programs run in the HIP kernels; tests/test_gpu_parity.py repeats this on the GPU.
'''
import numpy as np
import pytest

from tests.helpers import HostCheck, csr_dense, oracle_nlp, product_spec, random_w

VARIANTS = []
for _track in ('race', 'fig8'):
    for _model, _frame, _quat, _gr in [('drone', 'parametric', True, True), ('drone', 'parametric', False, True),
                                       ('drone', 'parametric', True, False), ('drone', 'parametric', False, False),
                                       ('drone', 'global', True, True), ('drone', 'global', False, True),
                                       ('point', 'parametric', False, True), ('point', 'parametric', False, False),
                                       ('point', 'global', False, True)]:
        VARIANTS.append(dict(track=_track, model=_model, frame=_frame, use_quat=_quat, global_r=_gr,
                             N=7 if _frame == 'global' else 4, K=2))
VARIANTS.append(dict(track='race', fix_gate_center=True, N=4, K=3))
VARIANTS.append(dict(track='fig8', quat_flip=True, N=4, K=3))
VARIANTS.append(dict(track='fig8', N=3, K=7))
# RK4 multiple shooting (use_rk4; scripts/race.py): N x K steps of one node each
for _model, _frame, _quat, _gr in [('drone', 'parametric', True, True), ('drone', 'parametric', False, True),
                                   ('drone', 'parametric', True, False), ('drone', 'global', True, True),
                                   ('drone', 'global', False, True), ('point', 'parametric', False, True),
                                   ('point', 'global', False, True)]:
    VARIANTS.append(dict(track='race', model=_model, frame=_frame, use_quat=_quat, global_r=_gr, N=7, K=2, rk4=True))
VARIANTS.append(dict(track='fig8', N=8, K=2, rk4=True, quat_flip=True))
# open (non-periodic) lines: initial / terminal rows instead of the closure, the final gate at zF
for _model, _frame, _quat in [('drone', 'parametric', True), ('drone', 'parametric', False),
                              ('drone', 'global', True), ('drone', 'global', False),
                              ('point', 'parametric', False), ('point', 'global', False)]:
    VARIANTS.append(dict(track='race', model=_model, frame=_frame, use_quat=_quat, closed=False,
                         N=6 if _frame == 'global' else 4, K=3))
# build-side DCM pose (config 5): restated in the oracle, pinned by equivalence (tests/test_dcm_cpu.py)
for _frame, _gr, _extra in [('parametric', True, {}), ('parametric', False, {}), ('global', True, {}),
                            ('parametric', True, {'closed': False}), ('global', True, {'closed': False}),
                            ('parametric', True, {'rk4': True}), ('global', True, {'rk4': True})]:
    VARIANTS.append(dict(track='race', model='drone', frame=_frame, use_dcm=True, global_r=_gr,
                         N=7 if (_frame == 'global' or _extra.get('rk4')) else 4, K=2 if _extra.get('rk4') else 3,
                         **_extra))


def _id(c):
    return '-'.join(f'{k}={v}' for k, v in c.items())


@pytest.mark.parametrize('cfg', VARIANTS, ids=_id)
def test_programs_match_oracle(cfg):
    rng = np.random.default_rng(7)
    spec = product_spec(**cfg)
    nlp = oracle_nlp(**cfg)
    hc = HostCheck(spec.native_spec())
    assert hc.nw == nlp.nw and hc.ng == nlp.ng
    np.testing.assert_array_equal(hc.lbg, nlp.lbg)
    np.testing.assert_array_equal(hc.ubg, nlp.ubg)
    np.testing.assert_allclose(spec.w0, nlp.w0, rtol=1e-13, atol=1e-13)
    np.testing.assert_array_equal(spec.lbw, nlp.lbw)
    np.testing.assert_array_equal(spec.ubw, nlp.ubw)
    w = random_w(nlp, rng)
    g, J, f, gf = hc.eval(w)
    go = nlp.g(w)
    Jo = nlp.jac_dense(w)
    scale_g = max(1.0, np.abs(go).max())
    scale_J = max(1.0, np.abs(Jo).max())
    np.testing.assert_allclose(g[0], go, rtol=0, atol=1e-12 * scale_g)
    P = csr_dense(hc.row_ptr, hc.col, np.ones(hc.nnz), hc.ng, hc.nw)
    assert not np.any((Jo != 0) & (P == 0)), 'oracle Jacobian has entries outside the pattern'
    np.testing.assert_allclose(csr_dense(hc.row_ptr, hc.col, J[0], hc.ng, hc.nw), Jo, rtol=0, atol=1e-12 * scale_J)
    assert abs(f[0] - nlp.f(w)) <= 1e-12 * max(1.0, abs(nlp.f(w)))
    np.testing.assert_allclose(gf[0], nlp.grad_f(w), rtol=0, atol=1e-12)


def test_csr_pattern_well_formed():
    spec = product_spec(N=6, K=4)
    hc = HostCheck(spec.native_spec())
    assert hc.row_ptr[0] == 0 and hc.row_ptr[-1] == hc.nnz
    assert np.all(np.diff(hc.row_ptr) >= 1)
    for r in range(hc.ng):
        c = hc.col[hc.row_ptr[r]:hc.row_ptr[r + 1]]
        assert np.all(np.diff(c) > 0) and c.min() >= 0 and c.max() < hc.nw


def test_benchmark_problem_sizes():
    ''' 50 x 4 x 13 racetrack (SURVEY 8 layout table): nw = 5300 '''
    spec = product_spec(N=50, K=4)
    hc = HostCheck(spec.native_spec())
    assert hc.nw == 5300
    nlp = oracle_nlp(N=50, K=4)
    assert hc.ng == nlp.ng
    assert 45000 < hc.nnz < 60000


def test_full_size_jvp_cpu():
    ''' full benchmark size: J v against complex-step directional derivatives of the oracle '''
    rng = np.random.default_rng(3)
    spec = product_spec(N=50, K=4)
    nlp = oracle_nlp(N=50, K=4)
    hc = HostCheck(spec.native_spec())
    w = random_w(nlp, rng)
    g, J, _, _ = hc.eval(w)
    np.testing.assert_allclose(g[0], nlp.g(w), rtol=0, atol=1e-11)
    V = rng.standard_normal((hc.nw, 3))
    Jv = np.stack([np.add.reduceat(J[0] * V[hc.col, j], hc.row_ptr[:-1]) for j in range(3)], axis=1)
    ref = nlp.jvp(w, V)
    np.testing.assert_allclose(Jv, ref, rtol=0, atol=1e-10 * max(1.0, np.abs(ref).max()))
