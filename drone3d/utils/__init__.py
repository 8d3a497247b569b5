''' drone3d.utils (re-exports; see drone3d/__init__.py) '''
