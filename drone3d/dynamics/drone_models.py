''' drone3d.dynamics.drone_models (reference: drone3d/dynamics/drone_models.py) '''
from aircraft_trajectory_optimization_amd.dynamics.drone_models import DroneModel, ParametricDroneModel  # noqa: F401
