''' drone3d.obstacles (re-exports; see drone3d/__init__.py) '''
