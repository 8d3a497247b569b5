'''
Mesh obstacle environment and obstacle-free tube (drone3d/obstacles/mesh_obstacle.py:18-237).

MeshObstacle loads the arena mesh (assets/arena_track_obstacles_multistory.npz, converted from
the reference's OBJ by tools/convert_mesh.py) into libato (ato_mesh_create); every distance
query runs in the HIP kernel ato_mesh_signed_distance (no trimesh). The tube is the reference's
brute-force largest-empty-sphere search (nr = 5 radii x nth = 8 angles around each node in the
(e_y, e_n) plane, :110-145); ObstacleFreeTube turns it into the per-node sphere rows
(y - dy)^2 + (n - dn)^2 <= max(r - r_c, 0.01)^2 (:219-237) as the ProblemSpec sphere table.
'''
import ctypes
import os
from typing import Dict, Optional, Tuple

import numpy as np

from aircraft_trajectory_optimization_amd import native

ASSETS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'assets')
_DEFAULT_FILENAME = 'arena_track_obstacles_multistory.npz'


class MeshObstacle:
    ''' triangle-mesh obstacle with GPU signed-distance queries '''

    def __init__(self, filename: str = _DEFAULT_FILENAME, color=None):
        import torch
        self.filename = filename
        path = filename if os.path.isabs(filename) else os.path.join(ASSETS, filename)
        data = np.load(path)
        self.vertices = np.ascontiguousarray(data['vertices'], np.float64)
        self.faces = np.ascontiguousarray(data['faces'], np.int32)
        self.color = color if color is not None else [1, 0, 0, 1]
        self.lib = native.load()
        if not torch.cuda.is_available():
            raise RuntimeError('MeshObstacle needs a HIP device')
        self._torch = torch
        self.device = torch.device('cuda', torch.cuda.current_device())
        h = ctypes.c_void_p()
        rc = self.lib.ato_mesh_create(self.vertices.ctypes.data, len(self.vertices), self.faces.ctypes.data,
                                      len(self.faces), ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(f'ato_mesh_create failed: {self.lib.ato_last_error().decode()}')
        self.handle = h

    def __del__(self):
        try:
            if getattr(self, 'handle', None):
                self.lib.ato_mesh_destroy(self.handle)
        except Exception:  # pylint: disable=broad-except
            pass

    def _query(self, x: np.ndarray, closest: bool) -> Tuple[np.ndarray, Optional[np.ndarray]]:
        torch = self._torch
        x = np.ascontiguousarray(np.atleast_2d(x), np.float64).reshape(-1, 3)
        n = len(x)
        xt = torch.as_tensor(x, device=self.device)
        d = torch.empty(n, dtype=torch.float64, device=self.device)
        c = torch.empty((n, 3), dtype=torch.float64, device=self.device) if closest else None
        rc = self.lib.ato_mesh_signed_distance(self.handle, n, xt.data_ptr(), d.data_ptr(),
                                               c.data_ptr() if closest else None,
                                               torch.cuda.current_stream(self.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f'ato_mesh_signed_distance failed: {self.lib.ato_last_error().decode()}')
        return d.cpu().numpy(), (c.cpu().numpy() if closest else None)

    def signed_distance(self, x: np.ndarray) -> np.ndarray:
        ''' positive outside the obstacles (mesh_obstacle.py:38-41) '''
        return self._query(x, False)[0]

    def closest_point(self, x: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        ''' closest surface points and (unsigned) distances '''
        d, c = self._query(x, True)
        return c, np.abs(d)

    def check_line_for_collisions(self, line, n: int = 1000) -> float:
        s = np.linspace(line.s_min(), line.s_max(), n)
        return float(self.signed_distance(np.array([line.p2xc(sk) for sk in s])).min())

    def check_for_collisions(self, x: np.ndarray, sep_radius: float = 0.3) -> bool:
        return bool((self.signed_distance(x) >= sep_radius).all())

    def search_largest_sphere(self, x0, ey, en, r_max: float = 0.5, nr: int = 5, nth: int = 8):
        ''' brute-force search for the largest empty sphere near each point (mesh_obstacle.py:110-145) '''
        d0 = self.signed_distance(x0)
        r = np.linspace(r_max, 0, nr, endpoint=False)
        th = np.linspace(0, 2 * np.pi, nth, endpoint=False)
        R, TH = np.meshgrid(r, th)
        R, TH = R.reshape(-1), TH.reshape(-1)
        X = np.kron(x0, np.ones((R.shape[0], 1))) + np.kron(ey, (R * np.cos(TH))[:, None]) + \
            np.kron(en, (R * np.sin(TH))[:, None])
        D = self.signed_distance(X).reshape((-1, nr * nth)).T
        idxs = D.argmax(axis=0)
        dn = D.max(axis=0)
        rn, thn = R[idxs], TH[idxs]
        xn = x0 + rn[:, None] * (ey * np.cos(thn[:, None]) + en * np.sin(thn[:, None]))
        x, rr = xn.copy(), dn.copy()
        x[d0 >= dn] = x0[d0 >= dn]
        rr[d0 >= dn] = d0[d0 >= dn]
        pts, _ = self.closest_point(x)
        return x, rr, pts

    def compute_plannning_tube(self, line, s: np.ndarray, collision_r: float) -> 'ObstacleFreeTube':
        ''' obstacle-free tube at the given path lengths (mesh_obstacle.py:50-76) '''
        s = np.asarray(s, float)
        x = np.array([line.p2xc(sk) for sk in s])
        ey = np.array([line.p2ey(sk) for sk in s])
        en = np.array([line.p2en(sk) for sk in s])
        center, r, tangent = self.search_largest_sphere(x, ey, en)
        ball_y = np.sum((center - x) * ey, axis=1)
        ball_n = np.sum((center - x) * en, axis=1)
        return ObstacleFreeTube(line, center, r, tangent, np.array([s, ball_y, ball_n]).T, collision_r)


class ObstacleFreeTube:
    ''' per-node spheres of the tube (mesh_obstacle.py:194-237) '''

    def __init__(self, line, ball_center, ball_r, ball_tangent_pts, ball_p, collision_r):
        from scipy.spatial import KDTree
        self.line = line
        self.ball_center, self.ball_r = ball_center, ball_r
        self.ball_tangent_pts, self.ball_p = ball_tangent_pts, ball_p
        self.ball_kd_tree = KDTree(ball_p[:, :1])
        self.collision_r = collision_r

    def sphere(self, s: float) -> Tuple[float, float, float]:
        ''' (dy, dn, available radius) of the sphere nearest to s '''
        _, i = self.ball_kd_tree.query([s])
        return self.ball_p[i, 1], self.ball_p[i, 2], max(self.ball_r[i] - self.collision_r, 0.01)

    def sphere_table(self, node_s: np.ndarray) -> np.ndarray:
        ''' [P, 3] table consumed by the sphere rows of the HIP programs '''
        return np.array([self.sphere(s) for s in node_s], float)

    def perturbed_tables(self, node_s: np.ndarray, seeds) -> np.ndarray:
        '''
        Config 4's batch of perturbed tubes (build-defined, the reference solves one tube):
        instance b draws, with numpy.random.default_rng(b), for every sphere of the tube a radius
        change U[-0.05, 0.05] and centre offsets (dy, dn) ~ N(0, 0.05^2); each node then takes its
        nearest sphere as sphere() does. Returns (B, P, 3) tables of (dy, dn, available radius).
        '''
        _, idx = self.ball_kd_tree.query(np.asarray(node_s, float)[:, None])
        nb = len(self.ball_r)
        out = []
        for b in seeds:
            rng = np.random.default_rng(b)
            dr = rng.uniform(-0.05, 0.05, nb)
            dd = rng.normal(0.0, 0.05, (nb, 2))
            r = np.maximum(self.ball_r + dr - self.collision_r, 0.01)
            out.append(np.stack([self.ball_p[idx, 1] + dd[idx, 0], self.ball_p[idx, 2] + dd[idx, 1], r[idx]], axis=1))
        return np.array(out, float)

    def get_vertex_objects(self, ubo=None) -> Dict[str, 'TubeDrawable']:
        ''' the drawables the reference's viewer adds for the tube (mesh_obstacle.py:239-275), as data:
        instance centres, scales and (planning tube) orientations '''
        # pylint: disable=unused-argument
        P = self.ball_center.shape[0]
        Rp = np.stack([self.line.p2Rp(float(s)) for s in self.ball_p[:, 0]]) if P else np.zeros((0, 3, 3))
        return {
            'Planning Tube': TubeDrawable(self.ball_center, np.maximum(self.ball_r - self.collision_r, 0.01), Rp),
            'Free-Space Spheres': TubeDrawable(self.ball_center, self.ball_r),
            'Sphere Centers': TubeDrawable(self.ball_center, np.full(P, 0.05)),
            'Sphere Contact Points': TubeDrawable(self.ball_tangent_pts, np.full(P, 0.05)),
        }


class TubeDrawable:
    ''' instanced drawable as plain data (no renderer in this build) '''

    def __init__(self, centers, scales, orientations=None):
        self.centers = np.asarray(centers, float)
        self.scales = np.asarray(scales, float)
        self.orientations = orientations
