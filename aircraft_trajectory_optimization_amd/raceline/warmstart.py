'''
Point-mass warm start of the drone NLP (use_ws / generate_ws; drone_raceline.py:32-40,
:158-274, base_raceline.py:731-736).

A point-mass raceline over the same track and discretisation is solved first; every drone
collocation node then gets
  * position from the point-mass node state,
  * attitude from the point-mass thrust direction (e3) and velocity (e1, made orthogonal), with
    quaternion signs kept continuous along the lap (and the closure sign derived from the first
    and last node), or Euler angles with 2 pi unwrapping,
  * body velocity R^T v_g and body rates R^T (T x dT) / |T|^2,
  * rotor thrusts |T| / 4, and the point-mass step sizes (bounds h/100 .. 10 h).
'''
from typing import Tuple

import numpy as np
from scipy.spatial.transform import Rotation

from aircraft_trajectory_optimization_amd.pytypes import DroneConfig
from aircraft_trajectory_optimization_amd.raceline.problem import ProblemSpec


def _point_frame(spec: ProblemSpec, n: int, k: int) -> np.ndarray:
    ''' rotation of the point model's velocity / thrust frame to the global frame
    (point_model.py: R = I for global orientation, R_p(s) otherwise) '''
    if spec.param and not spec.vehicle.global_r:
        return spec.line.p2Rp(spec.get_s(n, k))
    return np.eye(3)


def drone_guess(drone: ProblemSpec, point: ProblemSpec, x_point: np.ndarray) \
        -> Tuple[np.ndarray, np.ndarray, np.ndarray, bool, float]:
    '''
    Drone (w0, lbw, ubw, quat_flip, euler_wraps) from a point-mass solution x_point over the
    same N, K. `drone` provides indexing, bounds and the default guess.
    '''
    if (drone.N, drone.K) != (point.N, point.K):
        raise ValueError('warm start needs the same discretisation')
    veh: DroneConfig = drone.vehicle
    closed = bool(drone.config.closed)
    w0, lbw, ubw = drone.w0.copy(), drone.lbw.copy(), drone.ubw.copy()
    N, K1 = drone.N, drone.K1
    h = x_point[:N]
    w0[:N] = h
    lbw[:N] = h / 100
    ubw[:N] = h * 10
    first_r = last_r = None
    for n in range(N):
        for k in range(K1):
            pi = point.N + (n * K1 + k) * point.nv
            zp = x_point[pi:pi + 6]
            up = x_point[pi + 6:pi + 9]
            dup = x_point[pi + 9:pi + 12]
            Rw = _point_frame(point, n, k)
            T = Rw @ up
            vg = Rw @ zp[3:6]
            if closed:
                e1 = vg / np.linalg.norm(vg)
                e3 = T / np.linalg.norm(T)
                e1 = e1 - e3 * (e1 @ e3)
                e1 = e1 / np.linalg.norm(e1)
                e2 = np.cross(e3, e1)
                R = np.array([e1, e2, e3]).T
            else:
                b = np.array([0., 0., 1.])
                t = T / np.linalg.norm(T)
                v = -np.cross(t, b)
                s = np.linalg.norm(v)
                c = t @ b
                hat = np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])
                R = np.eye(3) + hat + hat @ hat * (1 - c) / s ** 2
            if not veh.global_r:
                R = drone.line.p2Rp(drone.get_s(n, k)).T @ R
            if getattr(veh, 'use_dcm', False):               # build-side DCM pose: R itself
                r = R.reshape(-1)
            elif veh.use_quat:
                r = Rotation.from_matrix(R).as_quat()          # (x, y, z, w) = (qi, qj, qk, qr)
                if last_r is not None and np.linalg.norm(r - last_r) >= 1:
                    r = -r
            else:
                r = np.flip(Rotation.from_matrix(R).as_euler('xyz', degrees=False))
                if last_r is not None and np.linalg.norm(r - last_r) > 1:
                    if r[0] - last_r[0] > np.pi:
                        r[0] -= 2 * np.pi
                    elif r[0] - last_r[0] <= -np.pi:
                        r[0] += 2 * np.pi
                    if np.linalg.norm(r - last_r) > 1:
                        raise NotImplementedError('Warmstart continuity failed for euler angles, try quaternion')
            if first_r is None:
                first_r = r
            last_r = r
            vb = R.T @ vg
            dT = Rw @ dup
            wb = R.T @ np.cross(T, dT) / np.linalg.norm(T) ** 2
            di = drone.N + (n * K1 + k) * drone.nv
            w0[di:di + drone.nz] = np.concatenate([zp[:3], r, vb, wb])
            w0[di + drone.nz:di + drone.nz + 4] = np.linalg.norm(T) / 4
            w0[di + drone.nz + 4:di + drone.nz + 8] = 0.0
    dcm = bool(getattr(veh, 'use_dcm', False))
    quat_flip = bool(veh.use_quat and not dcm and closed and np.linalg.norm(first_r - last_r) > 1)
    wraps = float(np.round((last_r - first_r)[0] / 2 / np.pi)) if (closed and not veh.use_quat and not dcm) else 0.0
    return w0, lbw, ubw, quat_flip, wraps


def drone_guess_batch(drone: ProblemSpec, point: ProblemSpec, XP: np.ndarray):
    '''
    drone_guess for B point-mass solutions XP [B, point.nw] at once (vectorised over the instances,
    node by node as drone_guess): (W [B, nw], LBW [B, nw], UBW [B, nw], quat_flip [B], euler_wraps [B]).
    Equal to drone_guess applied to every row (tests/test_corridor_cpu.py).
    '''
    if (drone.N, drone.K) != (point.N, point.K):
        raise ValueError('warm start needs the same discretisation')
    XP = np.atleast_2d(np.asarray(XP, float))
    B = XP.shape[0]
    veh: DroneConfig = drone.vehicle
    closed = bool(drone.config.closed)
    dcm = bool(getattr(veh, 'use_dcm', False))
    N, K1 = drone.N, drone.K1
    W = np.repeat(drone.w0[None], B, axis=0)
    LBW = np.repeat(drone.lbw[None], B, axis=0)
    UBW = np.repeat(drone.ubw[None], B, axis=0)
    h = XP[:, :N]
    W[:, :N], LBW[:, :N], UBW[:, :N] = h, h / 100, h * 10
    first_r = last_r = None
    ez = np.array([0., 0., 1.])
    for n in range(N):
        for k in range(K1):
            pi = point.N + (n * K1 + k) * point.nv
            zp, up, dup = XP[:, pi:pi + 6], XP[:, pi + 6:pi + 9], XP[:, pi + 9:pi + 12]
            Rw = _point_frame(point, n, k)
            T, vg, dT = up @ Rw.T, zp[:, 3:6] @ Rw.T, dup @ Rw.T
            Tn = np.linalg.norm(T, axis=1)
            if closed:
                e1 = vg / np.linalg.norm(vg, axis=1)[:, None]
                e3 = T / Tn[:, None]
                e1 = e1 - e3 * np.sum(e1 * e3, axis=1)[:, None]
                e1 = e1 / np.linalg.norm(e1, axis=1)[:, None]
                e2 = np.cross(e3, e1)
                R = np.stack([e1, e2, e3], axis=2)                     # columns e1 e2 e3
            else:
                t = T / Tn[:, None]
                v = -np.cross(t, ez)
                s = np.linalg.norm(v, axis=1)
                c = t @ ez
                hat = np.zeros((B, 3, 3))
                hat[:, 0, 1], hat[:, 0, 2], hat[:, 1, 2] = -v[:, 2], v[:, 1], -v[:, 0]
                hat[:, 1, 0], hat[:, 2, 0], hat[:, 2, 1] = v[:, 2], -v[:, 1], v[:, 0]
                R = np.eye(3)[None] + hat + (hat @ hat) * ((1 - c) / s ** 2)[:, None, None]
            if not veh.global_r:
                R = drone.line.p2Rp(drone.get_s(n, k)).T[None] @ R
            if dcm:
                r = R.reshape(B, 9)
            elif veh.use_quat:
                r = Rotation.from_matrix(R).as_quat()
                if last_r is not None:
                    flip = np.linalg.norm(r - last_r, axis=1) >= 1
                    r[flip] = -r[flip]
            else:
                r = np.flip(Rotation.from_matrix(R).as_euler('xyz', degrees=False), axis=1).copy()
                if last_r is not None:
                    far = np.linalg.norm(r - last_r, axis=1) > 1
                    d0 = r[:, 0] - last_r[:, 0]
                    r[far & (d0 > np.pi), 0] -= 2 * np.pi
                    r[far & ~(d0 > np.pi) & (d0 <= -np.pi), 0] += 2 * np.pi
                    if np.any(far & (np.linalg.norm(r - last_r, axis=1) > 1)):
                        raise NotImplementedError('Warmstart continuity failed for euler angles, try quaternion')
            if first_r is None:
                first_r = r
            last_r = r
            vb = np.einsum('bji,bj->bi', R, vg)
            wb = np.einsum('bji,bj->bi', R, np.cross(T, dT)) / (Tn ** 2)[:, None]
            di = drone.N + (n * K1 + k) * drone.nv
            W[:, di:di + drone.nz] = np.concatenate([zp[:, :3], r, vb, wb], axis=1)
            W[:, di + drone.nz:di + drone.nz + 4] = (Tn / 4)[:, None]
            W[:, di + drone.nz + 4:di + drone.nz + 8] = 0.0
    quat_flip = (np.zeros(B, bool) if (dcm or not veh.use_quat or not closed)
                 else np.linalg.norm(first_r - last_r, axis=1) > 1)
    wraps = (np.round((last_r - first_r)[:, 0] / 2 / np.pi) if (closed and not veh.use_quat and not dcm)
             else np.zeros(B))
    return W, LBW, UBW, quat_flip, wraps
