'''
drone3d -- the reference's import surface (drone3d.pytypes, drone3d.raceline.*,
drone3d.utils.solve_util, ...) mapped onto aircraft_trajectory_optimization_amd, so code written
against the reference (scripts/race.py, fig_8.py) imports unchanged. Every module here only
re-exports; the implementation (HIP evaluation library, interior-point solver) lives in
aircraft_trajectory_optimization_amd.
'''
