''' drone3d.raceline.drone_raceline (reference: drone3d/raceline/drone_raceline.py) '''
from aircraft_trajectory_optimization_amd.raceline.solvers import GlobalDroneRaceline, \
    ParametricDroneRaceline  # noqa: F401
from aircraft_trajectory_optimization_amd.raceline.solvers import _DroneRaceline as DroneRaceline  # noqa: F401
from aircraft_trajectory_optimization_amd.raceline.solvers import ParametricObstacleDroneRaceline  # noqa: F401
