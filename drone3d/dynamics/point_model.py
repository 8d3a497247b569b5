''' drone3d.dynamics.point_model (reference: drone3d/dynamics/point_model.py) '''
from aircraft_trajectory_optimization_amd.dynamics.point_model import ParametricPointModel, PointModel  # noqa: F401
