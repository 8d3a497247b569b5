''' drone3d.utils.cpc_utils (reference: drone3d/utils/cpc_utils.py) '''
from aircraft_trajectory_optimization_amd.utils.cpc_utils import package_cpc_data_as_raceline  # noqa: F401
