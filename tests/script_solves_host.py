'''
Host-side companions of tests/test_gpu_scripts.py: the same script-level solves (race.py's RK4
N = 70 drone solves, obstacles.py's N = 100 drone solve, fig_8.py's four N = 50 solves) through the
reference API, with the CPU build of the segment programs as the evaluator and the single-instance
host-KKT solver
(solver/ipm.py). The lap times they print are test_gpu_scripts.HOST_LAP. The obstacle tube uses the
oracle's mesh distance here (no device; the GPU mesh distance is pinned to it in test_gpu_parity.py).

    python tests/script_solves_host.py race_parametric | race_global | obstacles |
        fig8_cold_quat | fig8_cold_euler | fig8_param_ws | fig8_global_ws
'''
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from aircraft_trajectory_optimization_amd.raceline import solvers  # noqa: E402
from tests.helpers import HostEvaluator  # noqa: E402


def _oracle_mesh():
    from aircraft_trajectory_optimization_amd.obstacles.mesh_obstacle import MeshObstacle
    from oracle.ref_mesh import signed_distance as oracle_sd
    from tests.helpers import REPO
    mesh = np.load(f'{REPO}/aircraft_trajectory_optimization_amd/assets/arena_track_obstacles_multistory.npz')
    V, F = mesh['vertices'].astype(float), mesh['faces'].astype(np.int64)
    env = MeshObstacle.__new__(MeshObstacle)
    env.signed_distance = lambda x: oracle_sd(np.asarray(x, float), V, F)
    env.closest_point = lambda x: (np.zeros_like(np.atleast_2d(x)), None)
    return env


def main(which):
    from aircraft_trajectory_optimization_amd.tracks import make_line
    solvers._Raceline.evaluator_factory = HostEvaluator
    t0 = time.time()
    if which.startswith('fig8_'):
        from aircraft_trajectory_optimization_amd.utils.solve_util import solve_util
        kind = which[5:]
        s, r = solve_util(line=make_line('fig8'), global_frame=kind == 'global_ws', drone=True,
                          use_quaternion=kind != 'cold_euler', global_r=True, use_ws=kind.endswith('ws'), N=50,
                          verbose=False)
    elif which.startswith('race_'):
        from aircraft_trajectory_optimization_amd.utils.solve_util import solve_util
        s, r = solve_util(line=make_line('race'), global_frame=which == 'race_global', drone=True, use_ws=True,
                          use_quaternion=True, use_rk4=True, N=70, verbose=False)
    else:
        from aircraft_trajectory_optimization_amd.pytypes import DroneConfig
        from aircraft_trajectory_optimization_amd.raceline.config import ParametricRacelineConfig
        line = make_line('obstacles')
        line.config.gate_s = None
        config = ParametricRacelineConfig(verbose=False, N=100)
        config.closed = True
        s = solvers.ParametricObstacleDroneRaceline(line, config, DroneConfig(global_r=True, use_quat=True,
                                                                              collision_radius=0.4),
                                                    _oracle_mesh(), generate_ws=True)
        r = s.solve()
    ws = s.ws_raceline.time if s.ws_raceline is not None else None
    print(f'{which}: feasible {r.feasible} lap {r.time!r} (point mass {ws!r}), '
          f'iterations {s.result.iters}, wall {time.time() - t0:.1f} s', flush=True)


if __name__ == '__main__':
    main(sys.argv[1])
