''' drone3d.utils.load_utils (reference: drone3d/utils/load_utils.py) '''
from aircraft_trajectory_optimization_amd.utils.load_utils import get_assets_file, get_assets_folder  # noqa: F401
