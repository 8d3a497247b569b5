'''
Parity with the REFERENCE's own transcription at the bench's size (racetrack 50x4, the headline
config, and its obstacle-sphere variant): tests/golden/directional/*.npz, written by
tests/golden/make_transcription_golden.py (DIRECTIONAL), hold the reference NLP's bounds, w0,
g and f at two seeded points and the directional derivatives J V and grad f . V along four seeded
unit directions (complex step through the reference's expression graph; a dense 4.8k x 5.3k
Jacobian is not stored).

Checked here: the oracle (oracle/ref_transcription.py, its jvp) and the product's segment
programs compiled for the CPU (tests/native/hostcheck.cpp: CSR J times V). The GPU path is
tests/test_gpu_golden.py. Tolerance 1e-12 * max(1, max |reference|) per quantity, as the small cases.
'''
import numpy as np
import pytest

from tests.helpers import (DIRECTIONAL_DIR, HostCheck, csr_matvec, directional_names, golden_case, oracle_nlp,
                           product_spec)

NAMES = directional_names()


def _close(a, b, tol=1e-12):
    np.testing.assert_allclose(a, b, rtol=0, atol=tol * max(1.0, float(np.max(np.abs(b)))))


def _case(name):
    return golden_case(name, DIRECTIONAL_DIR)


def test_directional_set_is_the_bench_size():
    assert 'race_param_esp_N50K4' in NAMES
    for name in NAMES:
        d, kw = _case(name)
        assert (kw['N'], kw['K']) == (50, 4)
        assert d['V'].shape == (int(d['nw']), 4)
        np.testing.assert_allclose(np.linalg.norm(d['V'], axis=0), 1.0, rtol=1e-14)


@pytest.mark.parametrize('name', NAMES)
def test_oracle_matches_reference_at_bench_size(name):
    d, kw = _case(name)
    nlp = oracle_nlp(**kw)
    assert (nlp.nw, nlp.ng) == (int(d['nw']), int(d['ng']))
    np.testing.assert_array_equal(nlp.lbg, d['lbg'])
    np.testing.assert_array_equal(nlp.ubg, d['ubg'])
    np.testing.assert_array_equal(nlp.lbw, d['lbw'])
    np.testing.assert_array_equal(nlp.ubw, d['ubw'])
    _close(nlp.w0, d['w0'])
    for i, w in enumerate(d['W']):
        _close(nlp.g(w), d['G'][i])
        _close(nlp.f(w), d['F'][i])
        _close(nlp.jvp(w, d['V']), d['JV'][i])
        _close(nlp.grad_f(w) @ d['V'], d['GFV'][i])


@pytest.mark.parametrize('name', NAMES)
def test_product_programs_match_reference_at_bench_size(name):
    d, kw = _case(name)
    spec = product_spec(**kw)
    hc = HostCheck(spec.native_spec())
    assert (hc.nw, hc.ng) == (int(d['nw']), int(d['ng']))
    np.testing.assert_array_equal(hc.lbg, d['lbg'])
    np.testing.assert_array_equal(hc.ubg, d['ubg'])
    np.testing.assert_array_equal(spec.lbw, d['lbw'])
    np.testing.assert_array_equal(spec.ubw, d['ubw'])
    _close(spec.w0, d['w0'])
    g, J, f, gf = hc.eval(d['W'])
    for i in range(len(d['W'])):
        _close(g[i], d['G'][i])
        _close(f[i], d['F'][i])
        _close(csr_matvec(hc.row_ptr, hc.col, J[i], d['V']), d['JV'][i])
        _close(gf[i] @ d['V'], d['GFV'][i])
