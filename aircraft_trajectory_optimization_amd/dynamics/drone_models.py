'''
Quadrotor models on the host (numpy): drone3d/dynamics/drone_models.py.

    DroneModel            global position, ESP or YPR attitude (drone_models.py:12-233)
    ParametricDroneModel  (s, y, n) position along the centreline, attitude global (global_r) or
                          relative to the Darboux frame (drone_models.py:236-328)

State z = [p (3), r (4 | 3), v_b (3), w_b (3)], input u = four rotor thrusts.
'''
import numpy as np

from aircraft_trajectory_optimization_amd.centerlines.base_centerline import BaseCenterline
from aircraft_trajectory_optimization_amd.dynamics.dynamics_model import DynamicsModel, ParametricDynamicsModel
from aircraft_trajectory_optimization_amd.dynamics.rotations import Parameterization, Reference, Rotation
from aircraft_trajectory_optimization_amd.pytypes import DroneConfig, DroneState


def _hat(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


class DroneModel(DynamicsModel):
    ''' inertial-frame drone model '''
    config: DroneConfig
    _last_q: np.ndarray = None

    def __init__(self, config: DroneConfig):
        self.config = config
        self.rot = Rotation(Reference.GLOBAL if config.global_r else Reference.PARAMETRIC,
                            Parameterization.DCM if getattr(config, 'use_dcm', False) else
                            Parameterization.ESP if config.use_quat else Parameterization.YPR)
        self.nr = self.rot.nr
        self.nz, self.nu = 9 + self.nr, 4     # p (3), r (nr), v_b (3), w_b (3)

    def _split(self, z):
        nr = self.nr
        return z[:3], z[3:3 + nr], z[3 + nr:6 + nr], z[6 + nr:9 + nr]

    def _pose(self, z, geo):
        ''' (p_dot, r_dot, R global, R relative to the frame the thrust is reported in) '''
        _, r, vb, wb = self._split(z)
        R = self.rot.R(r)
        return R @ vb, self.rot.rate(r, wb), R, R

    def _evaluate(self, z, u, geo):
        ''' drone_models.py:47-123 '''
        c = self.config
        _, _, vb, wb = self._split(z)
        p_dot, r_dot, R, R_rel = self._pose(z, geo)
        Fgb = -c.m * c.g * np.array([R[2, 0], R[2, 1], R[2, 2]])
        Fdb = -np.array([c.b1, c.b2, c.b3]) * vb
        Kdb = -np.array([c.bw1, c.bw2, c.bw3]) * wb
        Tb = np.array([0.0, 0.0, u[0] + u[1] + u[2] + u[3]])
        TKb = np.array([(u[0] + u[1] - u[2] - u[3]) * c.l, (-u[0] + u[1] + u[2] - u[3]) * c.l,
                        (u[0] - u[1] + u[2] - u[3]) * c.k])
        Fb = Fdb + Fgb + Tb
        Kb = Kdb + TKb
        Ib = np.array([c.I1, c.I2, c.I3])
        Wb = _hat(wb)
        vb_dot = Fb / c.m - Wb @ vb
        wb_dot = (Kb - Wb @ (Ib * wb)) / Ib
        return {'z_dot': np.concatenate([p_dot, r_dot, vb_dot, wb_dot]), 'R': R, 'Tg': R @ Tb, 'Fgb': Fgb,
                'vg': R @ vb, 'Tp': R_rel @ Tb}

    def get_empty_state(self) -> DroneState:
        return DroneState(r=self.rot.get_empty_state())

    def state2zu(self, state: DroneState):
        z = [*state.x.to_vec(), *state.r.to_vec(), *state.v.to_vec(), *state.w.to_vec()]
        return z, self.state2u(state)

    def _set_q(self, state, z, u):
        R = self.f_R(z, u)
        state.q.from_mat(R)
        if self._last_q is not None and np.linalg.norm(self._last_q - state.q.to_vec()) > 1.8:
            state.q.from_vec(-state.q.to_vec())
        self._last_q = state.q.to_vec()

    def zu2state(self, state: DroneState, z, u):
        ''' drone_models.py:162-183 '''
        z = np.asarray(z, float).reshape(-1)
        self.u2state(state, u)
        _, r, vb, wb = self._split(z)
        state.x.from_vec(z[:3])
        self._set_r(state, r)
        state.v.from_vec(vb)
        state.w.from_vec(wb)
        if self.config.use_quat and self.rot.param == Parameterization.ESP:
            state.q.from_vec(r)
        else:
            self._set_q(state, z, u)

    def _set_r(self, state, r):
        if self.rot.param == Parameterization.DCM:     # the quaternion of R (orthonormalised)
            U, _, Vt = np.linalg.svd(self.rot.R(r))
            state.r.from_mat(U @ Vt)
        else:
            state.r.from_vec(r)

    def _zu_base(self):
        c = self.config
        return [np.inf] * 3 + list(self.rot.ubr()) + [np.inf] * 3 + [c.w_max] * 3

    def _zl_base(self):
        c = self.config
        return [-np.inf] * 3 + list(self.rot.lbr()) + [-np.inf] * 3 + [c.w_min] * 3

    def zu(self):
        return self._zu_base()

    def zl(self):
        return self._zl_base()


class ParametricDroneModel(ParametricDynamicsModel, DroneModel):
    ''' drone model in the centreline's (s, y, n) coordinates '''

    def __init__(self, config: DroneConfig, line: BaseCenterline):
        self.line = line
        DroneModel.__init__(self, config)

    def _pose(self, z, geo):
        ''' drone_models.py:249-292 '''
        _, r, vb, wb = self._split(z)
        Rr = self.rot.R(r)
        Rp = geo['Rp']
        R_rel = Rp.T @ Rr if self.config.global_r else Rr
        p_dot, wp = self._parametric_rates(R_rel @ vb, z, geo)
        w_eff = wb if self.config.global_r else wb - Rr.T @ wp
        R = Rr if self.config.global_r else Rp @ Rr
        return p_dot, self.rot.rate(r, w_eff), R, R_rel

    def state2zu(self, state: DroneState):
        z = [*state.p.to_vec(), *state.r.to_vec(), *state.v.to_vec(), *state.w.to_vec()]
        return z, self.state2u(state)

    def zu2state(self, state: DroneState, z, u):
        ''' drone_models.py:306-328 '''
        z = np.asarray(z, float).reshape(-1)
        self.u2state(state, u)
        _, r, vb, wb = self._split(z)
        state.p.from_vec(z[:3])
        self._set_r(state, r)
        state.v.from_vec(vb)
        state.w.from_vec(wb)
        state.x.from_vec(self.line.p2x(*z[:3]))
        self._set_q(state, z, u)
