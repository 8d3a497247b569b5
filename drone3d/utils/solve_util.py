''' drone3d.utils.solve_util (reference: drone3d/utils/solve_util.py) '''
from aircraft_trajectory_optimization_amd.utils.solve_util import solve_util  # noqa: F401
