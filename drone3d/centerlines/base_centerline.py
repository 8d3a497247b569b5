''' drone3d.centerlines.base_centerline (reference: drone3d/centerlines/base_centerline.py) '''
from aircraft_trajectory_optimization_amd.centerlines.base_centerline import *  # noqa: F401,F403
from aircraft_trajectory_optimization_amd.centerlines.base_centerline import BaseCenterline, \
    BaseCenterlineConfig, GateShape  # noqa: F401
