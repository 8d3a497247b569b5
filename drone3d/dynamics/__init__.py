''' drone3d.dynamics (re-exports; see drone3d/__init__.py) '''
