''' drone3d.centerlines.spline_centerline (reference: drone3d/centerlines/spline_centerline.py) '''
from aircraft_trajectory_optimization_amd.centerlines.spline_centerline import *  # noqa: F401,F403
from aircraft_trajectory_optimization_amd.centerlines.spline_centerline import SplineCenterline, \
    SplineCenterlineConfig  # noqa: F401
