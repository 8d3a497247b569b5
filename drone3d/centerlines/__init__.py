''' drone3d.centerlines (re-exports; see drone3d/__init__.py) '''
