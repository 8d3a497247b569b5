''' drone3d.visualization.drone_raceline_fig -- headless stand-in for the OpenGL viewer
(reference: drone3d/visualization/drone_raceline_fig.py). This build has no windowing stack;
the "window" prints a per-raceline summary and returns. '''
from aircraft_trajectory_optimization_amd.visualization.headless import DroneRacelineWindow  # noqa: F401
