''' drone3d.utils.discretization_utils (reference: drone3d/utils/discretization_utils.py) '''
from aircraft_trajectory_optimization_amd.utils.discretization_utils import *  # noqa: F401,F403
