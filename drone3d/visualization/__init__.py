''' drone3d.visualization (re-exports; see drone3d/__init__.py) '''
