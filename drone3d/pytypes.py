''' drone3d.pytypes (reference: drone3d/pytypes.py) '''
from aircraft_trajectory_optimization_amd.pytypes import *  # noqa: F401,F403
