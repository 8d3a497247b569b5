'''
ORACLE (test infrastructure only): collocation coefficients.

Restates drone3d/utils/discretization_utils.py:8-51. tau_0 = 0 plus the K Gauss-Legendre
roots on (0, 1) (CasADi collocation_points(K, 'legendre'), tabulated in CasADi to 16
decimal places; here numpy's Gauss-Legendre rule rounded to 16 decimal places).
'''
import numpy as np

# the K = 4 table as printed from the reference's CasADi build
CASADI_LEGENDRE_K4 = [0.0694318442029737, 0.3300094782075719, 0.6699905217924281, 0.9305681557970262]


def legendre_roots(K):
    x, _ = np.polynomial.legendre.leggauss(K)
    return [float(f'{v:.16f}') for v in sorted((x + 1) / 2)]


def coefficients(K):
    ''' tau, B, C, D exactly as discretization_utils.py:14-34 builds them (np.poly1d) '''
    tau = np.append(0, legendre_roots(K))
    B = np.zeros(K + 1)
    C = np.zeros((K + 1, K + 1))
    D = np.zeros(K + 1)
    for j in range(K + 1):
        p = np.poly1d([1])
        for r in range(K + 1):
            if r != j:
                p *= np.poly1d([1, -tau[r]]) / (tau[j] - tau[r])
        B[j] = np.polyint(p)(1.0)
        tangent = np.polyder(p)
        for r in range(K + 1):
            C[j, r] = tangent(tau[r])
        D[j] = p(1.0)
    return tau, B, C, D


def intermediate(K, d):
    ''' discretization_utils.py:36-51 '''
    tau = np.append(0, legendre_roots(K))
    D = np.zeros(K + 1)
    for j in range(K + 1):
        p = np.poly1d([1])
        for r in range(K + 1):
            if r != j:
                p *= np.poly1d([1, -tau[r]]) / (tau[j] - tau[r])
        D[j] = p(d)
    return D
