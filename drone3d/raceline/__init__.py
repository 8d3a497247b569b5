''' drone3d.raceline (re-exports; see drone3d/__init__.py) '''
