'''
Config 5's instance batch (raceline/batch_instances.py corridor_bounds, raceline/warmstart.py
drone_guess_batch): the vectorised drone guess equals drone_guess row by row for every pose, and the
corridors bound the lateral offset as documented.
'''
import numpy as np
import pytest

from aircraft_trajectory_optimization_amd.raceline.batch_instances import corridor_bounds
from aircraft_trajectory_optimization_amd.raceline.warmstart import drone_guess, drone_guess_batch
from aircraft_trajectory_optimization_amd.tracks import make_spec


def _points(ps, B, seed=0):
    ''' B point-mass "solutions": the default guess with smooth random perturbations (positive speeds,
    thrust with a vertical component) -- drone_guess only reads them '''
    rng = np.random.default_rng(seed)
    X = np.repeat(ps.w0[None], B, axis=0)
    X[:, :ps.N] *= rng.uniform(0.9, 1.1, (B, ps.N))
    node = ps.N + np.arange(ps.P) * ps.nv
    for i in (1, 2):
        X[:, node + i] += rng.normal(0, 0.1, (B, ps.P))
    X[:, node + 3] += rng.uniform(1.0, 3.0, (B, ps.P))
    X[:, node[:, None] + np.arange(4, 6)] += rng.normal(0, 0.5, (B, ps.P, 2))
    X[:, node[:, None] + np.arange(6, 9)] += rng.normal(0, 1.0, (B, ps.P, 3))
    X[:, node + 8] += 9.81
    X[:, node[:, None] + np.arange(9, 12)] += rng.normal(0, 1.0, (B, ps.P, 3))
    return X


@pytest.mark.parametrize('pose', ['dcm', 'quat', 'euler'])
@pytest.mark.parametrize('track,frame', [('fig8', 'parametric'), ('race', 'parametric'), ('race', 'global')])
def test_drone_guess_batch_equals_rowwise(pose, track, frame):
    kw = dict(track=track, frame=frame, N=6, K=3, global_r=(frame == 'parametric' and track == 'fig8'),
              use_quat=pose != 'euler', use_dcm=pose == 'dcm')
    ps = make_spec(**{**kw, 'model': 'point', 'use_quat': False, 'use_dcm': False})
    ds = make_spec(**{**kw, 'model': 'drone'})
    XP = _points(ps, 5)
    try:
        rows = [drone_guess(ds, ps, x) for x in XP]
    except NotImplementedError:
        with pytest.raises(NotImplementedError):
            drone_guess_batch(ds, ps, XP)
        return
    W, L, U, flip, wraps = drone_guess_batch(ds, ps, XP)
    for b, (w0, lb, ub, fl, wr) in enumerate(rows):
        np.testing.assert_allclose(W[b], w0, rtol=1e-13, atol=1e-13)
        np.testing.assert_array_equal(L[b], lb)
        np.testing.assert_array_equal(U[b], ub)
        assert bool(flip[b]) == fl and float(wraps[b]) == wr


def test_corridor_bounds():
    spec = make_spec(track='fig8', model='point', frame='parametric', N=10, K=3, use_quat=False, global_r=True)
    L, U = corridor_bounds(spec, [0, 1, 2, 3])
    node = spec.N + np.arange(spec.P) * spec.nv
    np.testing.assert_array_equal(L[0], spec.lbw)
    np.testing.assert_array_equal(U[0], spec.ubw)
    for b in (1, 2, 3):
        w = U[b, node + 1]
        assert np.all(w >= 0.7 - 1e-12) and np.all(w <= 1.4 + 1e-12)
        np.testing.assert_array_equal(L[b, node + 1], -w)
        other = np.setdiff1d(np.arange(spec.nw), node + 1)
        np.testing.assert_array_equal(L[b, other], spec.lbw[other])
        np.testing.assert_array_equal(U[b, other], spec.ubw[other])
    assert not np.array_equal(U[1], U[2])
