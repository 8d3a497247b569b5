'''
The reference's own test (tests/test_kinematics.py:13-102) restated on the oracle's ODEs:
a parametric (s, y, n) model and the global model are integrated from matching initial
conditions (g = 1, zero input) for 100 steps of dt = 0.1; the global positions must agree
to DIST_TOL = 1e-4 m at every step. This pins the non-Euclidean kinematics the HIP kernels
evaluate (drone_models.py:249-292, point_model.py:149-213).

Differences: scipy solve_ivp (rtol 1e-11) instead of SUNDIALS IDAS; the oracle implements
the PLANAR lateral fit (the reference also sweeps TORSION_FREE, which needs IDAS).
'''
import numpy as np
import pytest
from scipy.integrate import solve_ivp

from oracle import ref_models
from oracle.ref_geometry import RefCenterline

DIST_TOL = 1e-4


def _line():
    x = np.array([[0, 10, 0], [0, 10, 20], [0, 5, 10]], dtype=float)
    return RefCenterline(x, closed=False)


def _integrate(rhs, z0):
    t = np.arange(1, 101) * 0.1
    sol = solve_ivp(rhs, (0, t[-1]), z0, t_eval=t, rtol=1e-11, atol=1e-12)
    assert sol.success
    return sol.y.T


@pytest.mark.parametrize('global_r', [True, False])
@pytest.mark.parametrize('use_esp', [True, False])
def test_drone_kinematics(global_r, use_esp):
    line = _line()
    veh = dict(m=1.0, g=1.0, b1=0, b2=0, b3=0, I1=1e-3, I2=1e-3, I3=1.7e-3, l=0.15, k=0.05,
               bw1=1e-4, bw2=1e-4, bw3=1e-4)
    u = np.zeros((4, 1))
    att0 = [0, 0, 0, 1] if use_esp else [0, 0, 0]
    es0 = line.frame(0.0)['es']
    zp = np.array([0, 0, 0, *att0, *(es0 if global_r else [1, 0, 0]), 0, 0, 0], float)
    zg = np.array([0, 0, 0, *att0, *es0, 0, 0, 0], float)

    def rhs_p(_, z):
        return ref_models.drone_zdot(z[:, None], u, veh, use_esp, 'parametric', global_r, line.frame(z[0]))[:, 0]

    def rhs_g(_, z):
        return ref_models.drone_zdot(z[:, None], u, veh, use_esp, 'global', True)[:, 0]

    P = _integrate(rhs_p, zp)
    G = _integrate(rhs_g, zg)
    for zp_k, zg_k in zip(P, G):
        f = line.frame(zp_k[0])
        x = f['xc'] + zp_k[1] * f['ey'] + zp_k[2] * f['en']
        assert np.linalg.norm(x - zg_k[:3]) < DIST_TOL


@pytest.mark.parametrize('global_r', [True, False])
def test_point_kinematics(global_r):
    line = _line()
    veh = dict(m=1.0, g=1.0, b1=0, b2=0, b3=0)
    u = np.zeros((3, 1))
    es0 = line.frame(0.0)['es']
    zp = np.array([0, 0, 0, *(es0 if global_r else [1, 0, 0])], float)
    zg = np.array([0, 0, 0, *es0], float)

    def rhs_p(_, z):
        return ref_models.point_zdot(z[:, None], u, veh, 'parametric', global_r, line.frame(z[0]))[:, 0]

    def rhs_g(_, z):
        return ref_models.point_zdot(z[:, None], u, veh, 'global', True)[:, 0]

    P = _integrate(rhs_p, zp)
    G = _integrate(rhs_g, zg)
    for zp_k, zg_k in zip(P, G):
        f = line.frame(zp_k[0])
        x = f['xc'] + zp_k[1] * f['ey'] + zp_k[2] * f['en']
        assert np.linalg.norm(x - zg_k[:3]) < DIST_TOL
