'''
ORACLE (test infrastructure only): collocation coefficients.

Restates drone3d/utils/discretization_utils.py:8-51. tau_0 = 0 plus the K Gauss-Legendre
roots on (0, 1) (CasADi collocation_points(K, 'legendre'), tabulated in CasADi to 20 digits,
i.e. the nearest doubles of the roots; here the roots are found to 40 digits with mpmath and
rounded once).
'''
import numpy as np

# K = 4: (x + 1) / 2 for the roots x = +-sqrt(3/7 -+ 2/7 sqrt(6/5)) of P_4, rounded once
CASADI_LEGENDRE_K4 = [0.06943184420297371, 0.33000947820757187, 0.6699905217924281, 0.9305681557970263]


def legendre_roots(K):
    import mpmath
    with mpmath.workdps(40):
        guess, _ = np.polynomial.legendre.leggauss(K)
        roots = [mpmath.findroot(lambda z: mpmath.legendre(K, z), mpmath.mpf(float(g))) for g in guess]
        return [float((r + 1) / 2) for r in sorted(roots)]


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
