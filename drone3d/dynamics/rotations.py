''' drone3d.dynamics.rotations (reference: drone3d/dynamics/rotations.py) '''
from aircraft_trajectory_optimization_amd.dynamics.rotations import Parameterization, Reference, Rotation  # noqa: F401
