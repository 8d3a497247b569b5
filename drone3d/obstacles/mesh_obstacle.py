''' drone3d.obstacles.mesh_obstacle (reference: drone3d/obstacles/mesh_obstacle.py) '''
from aircraft_trajectory_optimization_amd.obstacles.mesh_obstacle import MeshObstacle, ObstacleFreeTube  # noqa: F401
