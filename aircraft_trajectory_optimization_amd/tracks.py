'''
The reference's scenario tracks and a one-call problem builder.

  RACE   scripts/race.py:12-14 (square gates)
  FIG8   scripts/fig_8.py:10-12 (circle gates)
  OBST   scripts/obstacles.py:14-16
'''
import numpy as np

from aircraft_trajectory_optimization_amd.centerlines.base_centerline import GateShape
from aircraft_trajectory_optimization_amd.centerlines.spline_centerline import SplineCenterline, \
    SplineCenterlineConfig
from aircraft_trajectory_optimization_amd.pytypes import DroneConfig, PointConfig
from aircraft_trajectory_optimization_amd.raceline.config import GlobalRacelineConfig, ParametricRacelineConfig
from aircraft_trajectory_optimization_amd.raceline.problem import ProblemSpec

RACE = np.array([[-1.1, 9.2, 9.2, -4.5, -4.5, 4.75, -2.8],
                 [-1.6, 6.6, -4, -6, -6, -0.9, 6.8],
                 [3.6, 1.0, 1.2, 3.5, 0.8, 1.2, 1.2]])
FIG8 = np.array([[0, 5, 0, -5, 0, 5, 0, -5],
                 [0, 1, 2, 1, 0, -1, -2, -1],
                 [10, 5, 0, -5, -10, -5, 0, 5]], dtype=float)
OBST = np.array([[-5, -2.75, -0.66, 2.95, 8.67, 9.2, 1.57, -2.39, -4.7, -2.39, 4.23, -2.66],
                 [4.5, -0.08, -1.36, 1.25, 6.69, -3.6, -6.43, -6, -6.43, -6.23, -0.66, 6.66],
                 [1.2, 2.815, 3.9, 2.815, 1.0, 1.0, 2.815, 3.9, 2.815, 1.0, 1.0, 1.0]])
TRACKS = {'race': (RACE, 'square'), 'fig8': (FIG8, 'circle'), 'obstacles': (OBST, 'circle')}


def make_line(track: str, closed: bool = True) -> SplineCenterline:
    ''' spline centreline of a named scenario (closed as in the scripts, or open: the waypoints
    as an open line, the demo of point_raceline.py:170-178) '''
    x, shape = TRACKS[track]
    cfg = SplineCenterlineConfig(x=np.array(x, float))
    cfg.closed = bool(closed)
    cfg.gate_shape = GateShape.SQUARE if shape == 'square' else GateShape.CIRCLE
    return SplineCenterline(cfg)


def make_spec(track='race', model='drone', frame='parametric', N=50, K=4, use_quat=True, global_r=True,
              fix_gate_center=False, quat_flip=False, spheres=None, v0=1.0, h0=1, rk4=False,
              euler_wraps=0.0, closed=True, use_dcm=False, cpc=None) -> ProblemSpec:
    ''' ProblemSpec of a scenario the way solve_util configures it (utils/solve_util.py:29-75) '''
    line = make_line(track, closed)
    if frame == 'parametric':
        cfg = ParametricRacelineConfig(verbose=False, N=N, K=K, v0=v0, h0=h0, use_rk4=rk4)
        cfg.closed = line.config.closed
        cfg.fixed_gates = line.config.s[:-1] if line.config.closed else line.config.s
    else:
        cfg = GlobalRacelineConfig(verbose=False, N=N, K=K, v0=v0, h0=h0, use_rk4=rk4)
        cfg.closed = line.config.closed
        cfg.gate_xi, cfg.gate_xj, cfg.gate_xk = line.config.x
    cfg.fix_gate_center = fix_gate_center
    if model == 'drone':
        veh = DroneConfig(global_r=True if frame == 'global' else global_r, use_quat=use_quat, use_dcm=use_dcm)
    else:
        veh = PointConfig(global_r=global_r)
    return ProblemSpec(line, cfg, veh, frame, quat_flip=quat_flip, euler_wraps=euler_wraps, sphere_table=spheres,
                       cpc=cpc)


def make_warm_spec(x_point, **kw) -> ProblemSpec:
    ''' drone ProblemSpec warm-started from a point-mass solution x_point of the same scenario
    (the point problem is make_spec(model='point', ...) with the same track / frame / N / K) '''
    from aircraft_trajectory_optimization_amd.raceline.warmstart import drone_guess
    point = make_spec(**{**kw, 'model': 'point', 'use_quat': False, 'use_dcm': False})
    drone0 = make_spec(**{**kw, 'model': 'drone'})
    w0, lbw, ubw, flip, wraps = drone_guess(drone0, point, np.asarray(x_point, float))
    drone = make_spec(**{**kw, 'model': 'drone', 'quat_flip': flip, 'euler_wraps': wraps})
    drone.w0, drone.lbw, drone.ubw = w0, lbw, ubw
    return drone
