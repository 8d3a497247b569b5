'''
Message / config types shared by every layer.

Public surface mirrors drone3d/pytypes.py of the reference (class names, field
names, defaults and methods), so code written against the reference keeps
working:
  PythonMsg (new-field guard, copy, pprint)      pytypes.py:10-46
  vector types, quaternion / Euler math          pytypes.py:48-355
  RacerConfig / PointConfig / DroneConfig        pytypes.py:357-402
  actuation and state types                      pytypes.py:404-483
'''
from abc import ABC, abstractmethod
from dataclasses import dataclass, field, fields
import copy
import numpy as np
from scipy.spatial.transform import Rotation as _SciRot


@dataclass
class PythonMsg:
    ''' dataclass base that refuses attributes that are not declared fields '''

    def __setattr__(self, key, value):
        if not hasattr(self, key):
            raise TypeError(f'Not allowed to add new field "{key}" to class {self}')
        object.__setattr__(self, key, value)

    def copy(self):
        ''' deep copy of the message '''
        return copy.deepcopy(self)

    def pprint(self, indent: int = 0):
        ''' indented field dump '''
        pad = ' ' * max(indent, 0)
        print(pad + type(self).__name__)
        for key, val in vars(self).items():
            if isinstance(val, PythonMsg):
                val.pprint(indent=max(indent, 0) + 2)
            else:
                print(pad + '  ' + f'{key} : {val}')


@dataclass
class VectorizablePythonMsg(PythonMsg, ABC):
    ''' message convertible to and from a flat vector '''

    @abstractmethod
    def to_vec(self) -> np.ndarray:
        ''' flatten '''

    @abstractmethod
    def from_vec(self, vec) -> None:
        ''' fill from a flat vector '''


class _FieldVector:
    ''' to_vec / from_vec over the dataclass fields, in declaration order '''

    def to_vec(self):
        return np.array([getattr(self, f.name) for f in fields(self)])

    def from_vec(self, vec):
        names = [f.name for f in fields(self)]
        vals = list(vec)
        if len(vals) != len(names):
            raise ValueError(f'expected {len(names)} values, got {len(vals)}')
        for name, val in zip(names, vals):
            setattr(self, name, val)


def _quat_matrix(qi, qj, qk, qr, transpose=False):
    ''' rotation matrix of a (unit) quaternion in (qi, qj, qk, qr) order '''
    m = np.array([
        [1 - 2 * (qj * qj + qk * qk), 2 * (qi * qj - qk * qr), 2 * (qi * qk + qj * qr)],
        [2 * (qi * qj + qk * qr), 1 - 2 * (qi * qi + qk * qk), 2 * (qj * qk - qi * qr)],
        [2 * (qi * qk - qj * qr), 2 * (qj * qk + qi * qr), 1 - 2 * (qi * qi + qj * qj)],
    ])
    return m.T if transpose else m


@dataclass
class Position(_FieldVector, VectorizablePythonMsg):
    ''' global-frame position '''
    xi: float = field(default=0)
    xj: float = field(default=0)
    xk: float = field(default=0)

    def xdot(self, q: 'OrientationQuaternion', v: 'BodyLinearVelocity') -> 'Position':
        ''' global velocity from attitude and body velocity '''
        out = Position()
        out.from_vec(q.R() @ v.to_vec())
        return out


@dataclass
class BodyPosition(_FieldVector, VectorizablePythonMsg):
    ''' body-frame position (COM at origin) '''
    x1: float = field(default=0)
    x2: float = field(default=0)
    x3: float = field(default=0)


@dataclass
class BodyLinearVelocity(_FieldVector, VectorizablePythonMsg):
    ''' body-frame linear velocity '''
    v1: float = field(default=0)
    v2: float = field(default=0)
    v3: float = field(default=0)

    def mag(self):
        ''' speed '''
        return float(np.linalg.norm(self.to_vec()))

    def signed_mag(self):
        ''' speed, negative when moving backwards '''
        return self.mag() * np.sign(self.v1)


@dataclass
class BodyAngularVelocity(_FieldVector, VectorizablePythonMsg):
    ''' body-frame angular velocity '''
    w1: float = field(default=0)
    w2: float = field(default=0)
    w3: float = field(default=0)


@dataclass
class BodyLinearAcceleration(_FieldVector, VectorizablePythonMsg):
    ''' body-frame linear acceleration '''
    a1: float = field(default=0)
    a2: float = field(default=0)
    a3: float = field(default=0)


@dataclass
class BodyAngularAcceleration(_FieldVector, VectorizablePythonMsg):
    ''' body-frame angular acceleration '''
    a1: float = field(default=0)
    a2: float = field(default=0)
    a3: float = field(default=0)


@dataclass
class OrientationQuaternion(_FieldVector, VectorizablePythonMsg):
    ''' Euler symmetric parameters, scalar last '''
    qi: float = field(default=0)
    qj: float = field(default=0)
    qk: float = field(default=0)
    qr: float = field(default=1)

    def R(self):
        ''' body -> global rotation matrix '''
        return _quat_matrix(self.qi, self.qj, self.qk, self.qr)

    def Rinv(self):
        ''' global -> body rotation matrix '''
        return _quat_matrix(self.qi, self.qj, self.qk, self.qr, transpose=True)

    def e1(self):
        ''' longitudinal body axis '''
        return self.R()[:, 0]

    def e2(self):
        ''' lateral body axis (left) '''
        return self.R()[:, 1]

    def e3(self):
        ''' normal body axis (up) '''
        return self.R()[:, 2]

    def norm(self):
        ''' quaternion norm '''
        return float(np.sqrt(self.qr ** 2 + self.qi ** 2 + self.qj ** 2 + self.qk ** 2))

    def normalize(self):
        ''' scale to unit norm in place '''
        nrm = self.norm()
        self.from_vec(self.to_vec() / nrm)

    def from_yaw(self, yaw):
        ''' planar yaw -> quaternion '''
        self.from_vec([0, 0, np.sin(yaw / 2), np.cos(yaw / 2)])

    def to_yaw(self):
        ''' quaternion -> planar yaw '''
        return 2 * np.arctan2(self.qk, self.qr)

    def from_mat(self, R):
        ''' fill from a rotation matrix '''
        self.from_vec(_SciRot.from_matrix(R).as_quat())

    def qdot(self, w: BodyAngularVelocity) -> 'OrientationQuaternion':
        ''' quaternion rate for a body angular velocity '''
        qi, qj, qk, qr = self.to_vec()
        w1, w2, w3 = w.to_vec()
        out = OrientationQuaternion()
        out.from_vec([
            0.5 * (qr * w1 + qj * w3 - qk * w2),
            0.5 * (qr * w2 + qk * w1 - qi * w3),
            0.5 * (qr * w3 + qi * w2 - qj * w1),
            -0.5 * (qi * w1 + qj * w2 + qk * w3),
        ])
        return out


@dataclass
class ParametricPosition(_FieldVector, VectorizablePythonMsg):
    ''' centreline-relative position (s, y, n) '''
    s: float = field(default=0.)
    y: float = field(default=0.)
    n: float = field(default=0.)


@dataclass
class Orientation(VectorizablePythonMsg):
    ''' any 3D orientation '''

    @abstractmethod
    def R(self):
        ''' rotation matrix '''

    @abstractmethod
    def from_mat(self, R):
        ''' fill from rotation matrix '''


@dataclass
class GlobalOrientation(Orientation):
    ''' orientation relative to the global frame '''


@dataclass
class RelativeOrientation(Orientation):
    ''' orientation relative to the centreline (Darboux) frame '''


@dataclass
class EulerAngles(_FieldVector, VectorizablePythonMsg):
    ''' yaw (a), pitch (b), roll (c); R = Rz(a) Ry(b) Rx(c) '''
    a: float = field(default=0.)
    b: float = field(default=0.)
    c: float = field(default=0.)

    def R(self):
        ''' rotation matrix '''
        ca, sa = np.cos(self.a), np.sin(self.a)
        cb, sb = np.cos(self.b), np.sin(self.b)
        cc, sc = np.cos(self.c), np.sin(self.c)
        rz = np.array([[ca, -sa, 0], [sa, ca, 0], [0, 0, 1]])
        ry = np.array([[cb, 0, sb], [0, 1, 0], [-sb, 0, cb]])
        rx = np.array([[1, 0, 0], [0, cc, -sc], [0, sc, cc]])
        return rz @ ry @ rx

    def from_mat(self, R):
        ''' fill from rotation matrix '''
        cba = _SciRot.from_matrix(R).as_euler('xyz', degrees=False)
        self.from_vec(cba[::-1])


@dataclass
class GlobalEulerAngles(EulerAngles, GlobalOrientation):
    ''' global Euler angles '''


@dataclass
class RelativeEulerAngles(EulerAngles, RelativeOrientation):
    ''' centreline-relative Euler angles '''


@dataclass
class GlobalQuaternion(OrientationQuaternion, GlobalOrientation):
    ''' global quaternion '''


@dataclass
class RelativeQuaternion(OrientationQuaternion, RelativeOrientation):
    ''' centreline-relative quaternion '''


@dataclass
class RacerConfig(PythonMsg):
    ''' vehicle parameters common to every racer '''
    dt: float = field(default=0.1)
    m: float = field(default=1.0)
    g: float = field(default=9.81)
    b1: float = field(default=0)
    b2: float = field(default=0)
    b3: float = field(default=0)
    global_r: bool = field(default=False)
    collision_radius: float = field(default=0.3)


@dataclass
class PointConfig(RacerConfig):
    ''' point-mass limits '''
    T_max: float = field(default=32.4)
    T_min: float = field(default=-32.4)
    dT_max: float = field(default=350)
    dT_min: float = field(default=-350)


@dataclass
class DroneConfig(RacerConfig):
    ''' quadrotor parameters and limits '''
    I1: float = field(default=1.0e-3)
    I2: float = field(default=1.0e-3)
    I3: float = field(default=1.7e-3)
    l: float = field(default=0.15)
    k: float = field(default=0.05)
    T_max: float = field(default=8.1)
    T_min: float = field(default=0.2)
    dT_max: float = field(default=20)
    dT_min: float = field(default=-20)
    bw1: float = field(default=1e-4)
    bw2: float = field(default=1e-4)
    bw3: float = field(default=1e-4)
    w_max: float = field(default=10)
    w_min: float = field(default=-10)
    use_quat: bool = field(default=False)
    # build-side (config 5, not in the reference): direction-cosine-matrix attitude, the state
    # carries R row-major (nz = 18); takes precedence over use_quat
    use_dcm: bool = field(default=False)


@dataclass
class DroneActuation(_FieldVector, VectorizablePythonMsg):
    ''' four rotor thrusts '''
    u1: float = field(default=0.)
    u2: float = field(default=0.)
    u3: float = field(default=0.)
    u4: float = field(default=0.)


@dataclass
class PointActuation(_FieldVector, VectorizablePythonMsg):
    ''' point-mass thrust vector '''
    u1: float = field(default=0.)
    u2: float = field(default=0.)
    u3: float = field(default=0.)


@dataclass
class RacerState(PythonMsg):
    ''' state of any racer '''
    t: float = field(default=0.)
    x: Position = field(default=None)
    q: OrientationQuaternion = field(default=None)
    v: BodyLinearVelocity = field(default=None)
    w: BodyAngularVelocity = field(default=None)
    p: ParametricPosition = field(default=None)
    d: float = field(default=0)

    def __post_init__(self):
        defaults = {'x': Position, 'q': OrientationQuaternion, 'v': BodyLinearVelocity,
                    'w': BodyAngularVelocity, 'p': ParametricPosition}
        for name, ctor in defaults.items():
            if getattr(self, name) is None:
                setattr(self, name, ctor())


@dataclass
class DroneState(RacerState):
    ''' quadrotor state '''
    r: Orientation = field(default=None)
    u: DroneActuation = field(default=None)
    du: DroneActuation = field(default=None)

    def __post_init__(self):
        super().__post_init__()
        if self.r is None:
            self.r = RelativeQuaternion()
        if self.u is None:
            self.u = DroneActuation()
        if self.du is None:
            self.du = DroneActuation()


@dataclass
class PointState(RacerState):
    ''' point-mass state '''
    u: PointActuation = field(default=None)
    du: PointActuation = field(default=None)

    def __post_init__(self):
        super().__post_init__()
        if self.u is None:
            self.u = PointActuation()
        if self.du is None:
            self.du = PointActuation()
