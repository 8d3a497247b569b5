''' asset paths (drone3d/utils/load_utils.py:4-10) '''
import os


def get_assets_folder() -> str:
    ''' the package's assets folder '''
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'assets')


def get_assets_file(file: str) -> str:
    ''' path of an asset file '''
    return os.path.join(get_assets_folder(), file)
