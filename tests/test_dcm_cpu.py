'''
Config 5's direction-cosine-matrix (DCM / SO(3)) pose: build-side, since the reference has ESP and
YPR attitudes only (drone3d/dynamics/rotations.py:19-24). Parity with the reference is unpinned by
construction; the DCM path is pinned by EQUIVALENCE with the reference-pinned ESP path:

  * the ODE: on states mapped through R = R(q) (rotations.py:44-80), the position, velocity and
    body-rate rows of the two models agree, and the DCM attitude rate R [w]x equals the rate of
    R(q(t)) along the ESP quaternion rate M(q) w -- for the global, global_r and relative frames;
  * the NLP: a DCM solve warm-started from the same point-mass raceline reaches the ESP solve's
    lap time, and its attitudes stay on SO(3) (the continuity operator's fixed point).

The C++ segment programs of the DCM pose are checked against the oracle's DCM restatement in
tests/test_programs_cpu.py (and on the GPU in tests/test_gpu_config5.py).
'''
import numpy as np
import pytest

from aircraft_trajectory_optimization_amd.solver.ipm import InteriorPointSolver, IPMOptions
from oracle import ref_models
from tests.helpers import HostEvaluator, oracle_line, product_spec

VEH = dict(m=1.0, g=9.81, b1=0.1, b2=0.2, b3=0.3, I1=1e-3, I2=1.2e-3, I3=1.7e-3, l=0.15, k=0.05,
           bw1=1e-4, bw2=2e-4, bw3=3e-4)


def _esp_to_dcm(z):
    ''' ESP state (13, B) -> DCM state (18, B): R = R(q) row-major '''
    R = ref_models.esp_R(z[3:7])
    return np.concatenate([z[:3], R.reshape(9, -1), z[7:]])


@pytest.mark.parametrize('frame,global_r', [('global', True), ('parametric', True), ('parametric', False)])
def test_dcm_ode_matches_esp_on_mapped_states(frame, global_r):
    rng = np.random.default_rng(11)
    B = 16
    z = rng.standard_normal((13, B))
    # unit quaternions: the reference's R(q) (rotations.py:50-66) is a rotation only for |q| = 1 (its
    # diagonal keeps the 1 of the unit-quaternion formula while dividing by |q|^2)
    z[3:7] /= np.linalg.norm(z[3:7], axis=0)
    z[1:3] *= 0.3
    u = 2 + rng.random((4, B))
    geo = None
    if frame == 'parametric':
        line = oracle_line('fig8')
        geo = line.frame(0.37 * (line.smax - line.smin))
    fe = ref_models.drone_zdot(z, u, VEH, True, frame, global_r, geo)
    zd = _esp_to_dcm(z)
    fd = ref_models.drone_zdot(zd, u, VEH, 'dcm', frame, global_r, geo)
    # position, body velocity and body-rate rows: identical physics
    np.testing.assert_allclose(fd[:3], fe[:3], rtol=0, atol=1e-13 * max(1, np.abs(fe[:3]).max()))
    np.testing.assert_allclose(fd[12:], fe[7:], rtol=0, atol=1e-12 * max(1, np.abs(fe[7:]).max()))
    # attitude: d/dt R(q) along q' = M(q) w_eff (complex step of R(q) in direction q'), against R [w_eff]x
    hstep = 1e-30
    Rdot = np.imag(ref_models.esp_R(z[3:7] + 1j * hstep * fe[3:7])) / hstep
    np.testing.assert_allclose(fd[3:12], Rdot.reshape(9, -1), rtol=0, atol=1e-12 * max(1, np.abs(Rdot).max()))


def _warm_solve(use_dcm, kw, x_point):
    from aircraft_trajectory_optimization_amd.tracks import make_warm_spec
    ds = make_warm_spec(x_point, use_dcm=use_dcm, **kw)
    ev = HostEvaluator(ds)
    res = InteriorPointSolver(ev, ds.lbw, ds.ubw, ev.lbg, ev.ubg, IPMOptions(max_iter=400)).solve(ds.w0)
    return ds, res


def test_dcm_warm_start_solve_matches_esp_lap_time():
    '''
    fig-8 (scripts/fig_8.py's track), parametric pose with global_r, N = 16, K = 4, both attitude
    parameterisations warm-started from the same point-mass solution. The two NLPs discretise the same
    continuous problem with different attitude polynomials (the interior collocation nodes of either
    leave the rotation manifold by the stage error), so their lap times differ by a discretisation
    error that shrinks with the mesh: measured 4.9e-3 s at N = 16, K = 3; 5.7e-4 s at 16 x 4; 2.5e-4 s
    at 32 x 3 (CPU). Bound here: the north star's 1e-3 s. The 50 x 4 fig-8 gap is measured on the GPU
    (tests/test_gpu_config5.py).
    '''
    kw = dict(track='fig8', frame='parametric', N=16, K=4)
    ps = product_spec(model='point', use_quat=False, **kw)
    pev = HostEvaluator(ps)
    pres = InteriorPointSolver(pev, ps.lbw, ps.ubw, pev.lbg, pev.ubg, IPMOptions(max_iter=300)).solve(ps.w0)
    assert pres.status == 'optimal'
    es, eres = _warm_solve(False, kw, pres.x)
    ds, dres = _warm_solve(True, kw, pres.x)
    assert eres.status == 'optimal' and dres.status == 'optimal', (eres.status, dres.status)
    lap_e, lap_d = eres.x[:es.N].sum(), dres.x[:ds.N].sum()
    assert abs(lap_e - lap_d) <= 1e-3, (lap_e, lap_d)
    # interval-start attitudes (outputs of the continuity operator): on SO(3), and close to R(q) of
    # the ESP solution
    err_orth, err_R = 0.0, 0.0
    for n in range(1, ds.N):
        R = dres.x[ds.col_z(n, 0, 3):ds.col_z(n, 0, 12)].reshape(3, 3)
        err_orth = max(err_orth, np.abs(R.T @ R - np.eye(3)).max())
        q = eres.x[es.col_z(n, 0, 3):es.col_z(n, 0, 7)]
        err_R = max(err_R, np.abs(ref_models.esp_R(q[:, None])[:, :, 0] - R).max())
    assert err_orth <= 1e-8, err_orth
    assert err_R <= 2e-2, err_R


def test_dcm_through_the_raceline_api(monkeypatch):
    ''' the reference's solver class with DroneConfig(use_dcm=True): point-mass warm start, solve,
    unpacked states (the attitude field holds the quaternion of R) '''
    from aircraft_trajectory_optimization_amd.pytypes import DroneConfig
    from aircraft_trajectory_optimization_amd.raceline import solvers
    from aircraft_trajectory_optimization_amd.raceline.config import ParametricRacelineConfig
    from aircraft_trajectory_optimization_amd.tracks import make_line
    monkeypatch.setattr(solvers._Raceline, 'evaluator_factory', HostEvaluator)
    line = make_line('fig8')
    cfg = ParametricRacelineConfig(verbose=False, N=12, K=4)
    cfg.closed = True
    cfg.fixed_gates = line.config.s[:-1]
    solver = solvers.ParametricDroneRaceline(line, cfg, DroneConfig(global_r=True, use_dcm=True), generate_ws=True)
    assert solver.spec.nz == 18 and solver.model.nz == 18
    res = solver.solve()
    assert res.feasible
    assert len(res.states) == 12 * 5
    for s in res.states:
        assert abs(np.linalg.norm(s.q.to_vec()) - 1) < 1e-9
        assert abs(np.linalg.norm(s.r.to_vec()) - 1) < 1e-9
    assert abs(res.time - np.sum(res.step_sizes)) < 1e-12
