'''
Attitude parameterisations on the host (numpy): drone3d/dynamics/rotations.py.

    ESP (quaternion, scalar last: qi, qj, qk, qr)   R(q) = standard DCM / |q|^2,  r_dot = M(q) w
    YPR (a, b, c)                                    R = Rz(a) Ry(b) Rx(c),        r_dot = M(r) w
    DCM (R row-major; build-side, config 5)          R = r,                        r_dot = R [w]x

The same expressions as the device models (csrc/ato_models.hpp) and the reference's SX
graphs (rotations.py:44-102); bounds as rotations.py:130-161.
'''
from enum import Enum

import numpy as np

from aircraft_trajectory_optimization_amd.pytypes import GlobalEulerAngles, GlobalQuaternion, \
    RelativeEulerAngles, RelativeQuaternion


class Reference(Enum):
    ''' frame the orientation is expressed in '''
    GLOBAL = 0
    PARAMETRIC = 1


class Parameterization(Enum):
    ''' rotation parameterisation '''
    ESP = 0
    YPR = 1
    DCM = 2      # build-side (config 5): not in the reference's rotations.py:19-24


def esp_R(q) -> np.ndarray:
    qi, qj, qk, qr = (float(v) for v in q)
    R = np.array([[1 - 2 * qj ** 2 - 2 * qk ** 2, 2 * (qi * qj - qk * qr), 2 * (qi * qk + qj * qr)],
                  [2 * (qi * qj + qk * qr), 1 - 2 * qi ** 2 - 2 * qk ** 2, 2 * (qj * qk - qi * qr)],
                  [2 * (qi * qk - qj * qr), 2 * (qj * qk + qi * qr), 1 - 2 * qi ** 2 - 2 * qj ** 2]])
    return R / (qi ** 2 + qj ** 2 + qk ** 2 + qr ** 2)


def esp_M(q) -> np.ndarray:
    qi, qj, qk, qr = (float(v) for v in q)
    return 0.5 * np.array([[qr, -qk, qj], [qk, qr, -qi], [-qj, qi, qr], [-qi, -qj, -qk]])


def ypr_R(r) -> np.ndarray:
    a, b, c = (float(v) for v in r)
    Ra = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
    Rb = np.array([[np.cos(b), 0, np.sin(b)], [0, 1, 0], [-np.sin(b), 0, np.cos(b)]])
    Rc = np.array([[1, 0, 0], [0, np.cos(c), -np.sin(c)], [0, np.sin(c), np.cos(c)]])
    return Ra @ Rb @ Rc


def ypr_M(r) -> np.ndarray:
    _, b, c = (float(v) for v in r)
    return np.array([[0, np.sin(c) / np.cos(b), np.cos(c) / np.cos(b)],
                     [0, np.cos(c), -np.sin(c)],
                     [1, np.sin(c) * np.tan(b), np.cos(c) * np.tan(b)]])


class Rotation:
    ''' rotation handler (rotations.py:27-183) with numeric R(r) / M(r) '''

    def __init__(self, ref: Reference, param: Parameterization):
        self.ref, self.param = ref, param

    @property
    def nr(self) -> int:
        return {Parameterization.ESP: 4, Parameterization.YPR: 3, Parameterization.DCM: 9}[self.param]

    def R(self, r) -> np.ndarray:
        if self.param == Parameterization.DCM:
            return np.asarray(r, float).reshape(3, 3)
        return esp_R(r) if self.param == Parameterization.ESP else ypr_R(r)

    def M(self, r) -> np.ndarray:
        if self.param == Parameterization.DCM:
            raise ValueError('the DCM rate is R [w]x, not M(r) w: use rate()')
        return esp_M(r) if self.param == Parameterization.ESP else ypr_M(r)

    def rate(self, r, w) -> np.ndarray:
        ''' r_dot for the body rate w '''
        if self.param == Parameterization.DCM:
            w = np.asarray(w, float)
            W = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
            return (self.R(r) @ W).reshape(-1)
        return self.M(r) @ w

    def ubr(self):
        ''' rotations.py:130-145 '''
        if self.param == Parameterization.DCM:
            return [np.inf] * 9
        if self.param == Parameterization.ESP:
            return [np.inf] * 4
        if self.ref == Reference.GLOBAL:
            return [np.inf, np.pi / 2.1, np.pi / 2.1]
        return [np.pi / 2, np.pi / 2.1, np.pi / 2.1]

    def lbr(self):
        ''' rotations.py:147-161 '''
        if self.param == Parameterization.DCM:
            return [-np.inf] * 9
        if self.param == Parameterization.ESP:
            return [-np.inf] * 4
        if self.ref == Reference.GLOBAL:
            return [-np.inf, -np.pi / 2.1, -np.pi / 2.1]
        return [-np.pi / 2, -np.pi / 2.1, -np.pi / 2.1]

    def get_empty_state(self):
        ''' rotations.py:163-183 (DCM: the state's attitude field holds the quaternion of R) '''
        if self.param == Parameterization.DCM:
            return GlobalQuaternion() if self.ref == Reference.GLOBAL else RelativeQuaternion()
        if self.ref == Reference.GLOBAL:
            return GlobalQuaternion() if self.param == Parameterization.ESP else GlobalEulerAngles()
        return RelativeQuaternion() if self.param == Parameterization.ESP else RelativeEulerAngles()
