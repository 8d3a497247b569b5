'''
One-call solver factory (drone3d/utils/solve_util.py:11-82): picks the global / parametric,
drone / point-mass raceline for a centreline and solves it.
'''
from typing import Tuple

from aircraft_trajectory_optimization_amd.pytypes import DroneConfig, PointConfig
from aircraft_trajectory_optimization_amd.raceline.config import GlobalRacelineConfig, \
    ParametricRacelineConfig, RacelineResults
from aircraft_trajectory_optimization_amd.raceline.solvers import GlobalDroneRaceline, GlobalPointRaceline, \
    ParametricDroneRaceline, ParametricPointRaceline


def solve_util(line, global_frame: bool, drone: bool, use_quaternion: bool = False, global_r: bool = True,
               use_ws: bool = False, solve: bool = True, fix_gate_center: bool = False, verbose: bool = True,
               use_rk4: bool = False, N=50, v0=1.0) -> Tuple[object, RacelineResults]:
    ''' same arguments, defaults and configuration as the reference '''
    if global_frame:
        config = GlobalRacelineConfig(verbose=verbose, N=N, v0=v0, use_rk4=use_rk4)
        config.closed = line.config.closed
        config.gate_xi = line.config.x[0]
        config.gate_xj = line.config.x[1]
        config.gate_xk = line.config.x[2]
        config.fix_gate_center = fix_gate_center
        if drone:
            solver = GlobalDroneRaceline(line, config, DroneConfig(global_r=True, use_quat=use_quaternion),
                                         generate_ws=use_ws)
        else:
            solver = GlobalPointRaceline(line, config, PointConfig(global_r=True))
    else:
        config = ParametricRacelineConfig(verbose=verbose, N=N, v0=v0, use_rk4=use_rk4)
        config.closed = line.config.closed
        config.fixed_gates = line.config.s[:-1] if line.config.closed else line.config.s
        config.fix_gate_center = fix_gate_center
        if drone:
            solver = ParametricDroneRaceline(line, config, DroneConfig(global_r=global_r, use_quat=use_quaternion),
                                             generate_ws=use_ws)
        else:
            solver = ParametricPointRaceline(line, config, PointConfig(global_r=global_r))
    raceline = solver.solve() if solve else solver.get_ws()
    return solver, raceline
