'''
Parity against the REFERENCE's own transcription.

tests/golden/transcription/*.npz were produced by tests/golden/make_transcription_golden.py,
which runs the reference's drone3d raceline / dynamics / centerline code itself (against an
arithmetic-only CasADi stand-in; CasADi is not installable here) and evaluates the
NLP it builds. These tests pin, case by case (closed / open lines, parametric / global frames,
quaternion / Euler attitude, global / relative attitude, drone / point mass, collocation K = 2..7
and RK4, fixed gate centres, obstacle spheres, point-mass warm starts):
  * the row order and bounds: lbg / ubg element for element, and lbw / ubw / w0,
  * g(w), the dense Jacobian, f(w) and grad f(w) at two seeded points,
for the oracle (oracle/ref_transcription.py) and for the product's segment programs compiled for
the host (the same C++ the HIP kernels run; tests/test_gpu_golden.py repeats this through
ato_eval on the GPU).

Tolerance (fp64): |x - reference| <= 1e-12 * max(1, max |reference|) per quantity; the only
differences are summation and association order. RK4 cases of the product use 1e-10: the step
Jacobian is a forward-mode dual-number derivative through four chained model evaluations (the
reference and the oracle take the complex-step derivative of the same expressions), and on the
figure-8 the parametric s-rate 1 / (1 + k_y n - k_n y) magnifies the association-order differences
(entries up to 6e5 at the seeded points).
'''
import numpy as np
import pytest

from aircraft_trajectory_optimization_amd.tracks import make_warm_spec
from tests.helpers import HostCheck, csr_dense, golden_case, golden_jacobian, golden_names, oracle_nlp, \
    product_spec

NAMES = [n for n in golden_names() if not n.endswith('_refused')]
WARM = [n for n in NAMES if '_warm_' in n]


def _close(a, b, tol=1e-12):
    np.testing.assert_allclose(a, b, rtol=0, atol=tol * max(1.0, float(np.max(np.abs(b)))))


def _bounds_equal(a, b):
    np.testing.assert_array_equal(np.asarray(a, float), np.asarray(b, float))


def _spec(name):
    d, kw = golden_case(name)
    if '_warm_' in name:
        cfg = {k: v for k, v in kw.items() if k not in ('quat_flip', 'euler_wraps')}
        spec = make_warm_spec(d['x_point'], **cfg)
    else:
        spec = product_spec(**kw)
    return d, kw, spec


@pytest.mark.parametrize('name', NAMES)
def test_oracle_matches_reference_transcription(name):
    d, kw = golden_case(name)
    nlp = oracle_nlp(**kw)
    assert (nlp.nw, nlp.ng) == (int(d['nw']), int(d['ng']))
    _bounds_equal(nlp.lbg, d['lbg'])
    _bounds_equal(nlp.ubg, d['ubg'])
    if '_warm_' not in name:
        _bounds_equal(nlp.lbw, d['lbw'])
        _bounds_equal(nlp.ubw, d['ubw'])
        _close(nlp.w0, d['w0'])
    for i, w in enumerate(d['W']):
        _close(nlp.g(w), d['G'][i])
        _close(nlp.jac_dense(w), golden_jacobian(d, i))
        _close(nlp.f(w), d['F'][i])
        _close(nlp.grad_f(w), d['GF'][i])


@pytest.mark.parametrize('name', NAMES)
def test_product_programs_match_reference_transcription(name):
    d, kw, spec = _spec(name)
    hc = HostCheck(spec.native_spec())
    assert (hc.nw, hc.ng) == (int(d['nw']), int(d['ng']))
    _bounds_equal(hc.lbg, d['lbg'])
    _bounds_equal(hc.ubg, d['ubg'])
    _bounds_equal(spec.lbw, d['lbw'])
    _bounds_equal(spec.ubw, d['ubw'])
    _close(spec.w0, d['w0'])
    g, J, f, gf = hc.eval(d['W'])
    tol = 1e-10 if kw.get('rk4') else 1e-12
    P = csr_dense(hc.row_ptr, hc.col, np.ones(hc.nnz), hc.ng, hc.nw)
    for i in range(len(d['W'])):
        Jref = golden_jacobian(d, i)
        assert not np.any((Jref != 0) & (P == 0)), 'reference Jacobian entries outside the product pattern'
        _close(g[i], d['G'][i], tol)
        _close(csr_dense(hc.row_ptr, hc.col, J[i], hc.ng, hc.nw), Jref, tol)
        _close(f[i], d['F'][i], tol)
        _close(gf[i], d['GF'][i], tol)


@pytest.mark.parametrize('name', WARM)
def test_warm_start_guess_matches_reference(name):
    ''' drone_raceline.py:158-274: position, attitude (sign / wrap continuity), body velocity, body
    rates, rotor thrusts and step sizes from the point-mass solution; closure sign / wraps '''
    d, kw, spec = _spec(name)
    _close(spec.w0, d['w0'])
    _bounds_equal(spec.lbw, d['lbw'])
    _bounds_equal(spec.ubw, d['ubw'])
    assert spec.quat_flip == kw.get('quat_flip', False)
    assert spec.euler_wraps == kw.get('euler_wraps', 0.0)


def test_warm_start_refusal_matches_reference():
    ''' the reference raises for an Euler guess whose heading jumps (drone_raceline.py:223-235);
    so does the product, for the same point-mass solution '''
    for name in [n for n in golden_names() if n.endswith('_refused')]:
        d, kw = golden_case(name)
        assert str(d['error']).startswith('NotImplementedError')
        cfg = {k: v for k, v in kw.items() if k not in ('quat_flip', 'euler_wraps')}
        with pytest.raises(NotImplementedError):
            make_warm_spec(d['x_point'], **cfg)


def test_golden_set_covers_the_row_families():
    ''' the fixture set spans every transcription variant the product supports '''
    seen = {n for n in NAMES}
    for needle in ('_K7', '_rk4', '_open_', '_global_', '_ypr_', '_rel_', '_point_', '_spheres_', '_warm_',
                   'fixcenter', 'fig8_', 'race_', 'obst_'):
        assert any(needle in n for n in seen), needle
