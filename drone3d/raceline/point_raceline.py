''' drone3d.raceline.point_raceline (reference: drone3d/raceline/point_raceline.py) '''
from aircraft_trajectory_optimization_amd.raceline.solvers import GlobalPointRaceline, \
    ParametricPointRaceline  # noqa: F401
from aircraft_trajectory_optimization_amd.raceline.solvers import ParametricObstaclePointRaceline  # noqa: F401
