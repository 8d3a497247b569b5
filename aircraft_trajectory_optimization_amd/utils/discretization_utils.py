'''
Collocation coefficients and solution interpolants (host side, fp64).

Mirrors drone3d/utils/discretization_utils.py of the reference:
  get_collocation_coefficients            discretization_utils.py:8-34
  get_intermediate_collocation_coefficients  discretization_utils.py:36-51
  interpolate_collocation / interpolate_linear  discretization_utils.py:53-117

The roots are Gauss-Legendre (COLLOCATION_ROOT_METHOD = 'legendre',
discretization_utils.py:6) with tau_0 = 0 prepended. CasADi's
collocation_points() returns roots from 20-digit tables, i.e. the doubles
nearest to the true roots; _LEGENDRE holds those doubles for K <= 9
(Gauss-Legendre roots computed to 50 digits and rounded once), larger K use
numpy's rule. B, C, D use the same np.poly1d product construction as the
reference (it is numerically lossy), so the device sees the same
coefficients the reference's graph would. The reference's own transcription,
run against these roots, pins the result (tests/test_golden_transcription_cpu.py).
'''
from typing import Callable, Sequence, Tuple
import numpy as np

COLLOCATION_ROOT_METHOD = 'legendre'

# nearest doubles of the Gauss-Legendre roots on (0, 1)
_LEGENDRE = {
    1: [0.5],
    2: [0.2113248654051871, 0.7886751345948129],
    3: [0.11270166537925831, 0.5, 0.8872983346207417],
    4: [0.06943184420297371, 0.33000947820757187, 0.6699905217924281, 0.9305681557970263],
    5: [0.046910077030668004, 0.23076534494715845, 0.5, 0.7692346550528415, 0.953089922969332],
    6: [0.03376524289842399, 0.16939530676686773, 0.38069040695840156, 0.6193095930415985, 0.8306046932331322,
        0.966234757101576],
    7: [0.025446043828620736, 0.12923440720030277, 0.2970774243113014, 0.5, 0.7029225756886985,
        0.8707655927996972, 0.9745539561713793],
    8: [0.019855071751231884, 0.10166676129318664, 0.2372337950418355, 0.4082826787521751, 0.591717321247825,
        0.7627662049581645, 0.8983332387068134, 0.9801449282487681],
    9: [0.015919880246186954, 0.0819844463366821, 0.1933142836497048, 0.33787328829809554, 0.5,
        0.6621267117019045, 0.8066857163502952, 0.9180155536633179, 0.984080119753813],
}


def collocation_points(K: int, method: str = COLLOCATION_ROOT_METHOD) -> np.ndarray:
    ''' K collocation roots on (0, 1) '''
    if K <= 0:
        return np.zeros(0)
    if method == 'legendre':
        if K in _LEGENDRE:
            return np.array(_LEGENDRE[K])
        x, _ = np.polynomial.legendre.leggauss(K)
        return np.sort((x + 1.0) / 2.0)
    if method == 'radau':
        # Radau IIA: roots of P_K - P_{K-1} mapped to (0,1], right end included
        c = np.zeros(K + 1)
        c[K] = 1.0
        c[K - 1] = -1.0
        x = np.polynomial.legendre.legroots(c)
        return np.sort((1.0 - x) / 2.0)
    raise NotImplementedError(method)


def _lagrange_basis(tau: np.ndarray, j: int) -> np.poly1d:
    basis = np.poly1d([1.0])
    for r, tr in enumerate(tau):
        if r == j:
            continue
        basis = basis * (np.poly1d([1.0, -tr]) / (tau[j] - tr))
    return basis


def get_collocation_coefficients(K: int) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    '''
    tau (K+1,), B (K+1,) quadrature weights, C (K+1, K+1) with
    C[j, r] = l_j'(tau_r), D (K+1,) end values l_j(1).
    '''
    tau = np.concatenate([[0.0], collocation_points(K)])
    n = K + 1
    B = np.zeros(n)
    C = np.zeros((n, n))
    D = np.zeros(n)
    for j in range(n):
        lj = _lagrange_basis(tau, j)
        B[j] = np.polyint(lj)(1.0)
        dlj = np.polyder(lj)
        C[j, :] = [dlj(tr) for tr in tau]
        D[j] = lj(1.0)
    return tau, B, C, D


def get_intermediate_collocation_coefficients(K: int, d: float) -> np.ndarray:
    ''' Lagrange weights l_j(d) for a point at fraction d of an interval '''
    tau = np.concatenate([[0.0], collocation_points(K)])
    return np.array([_lagrange_basis(tau, j)(d) for j in range(K + 1)])


def interpolate_collocation(step_sizes: Sequence[float], X: np.ndarray, K: int) \
        -> Callable[[float], np.ndarray]:
    '''
    Piecewise Lagrange interpolant of a collocation solution.
    X has shape (N, K+1, n). Outside [0, sum(h)] the first / final
    (end-of-interval) values are held, as in the reference's pw_const
    construction.
    '''
    h = np.asarray(step_sizes, dtype=float)
    X = np.asarray(X, dtype=float)
    N = X.shape[0]
    tau, _, _, D = get_collocation_coefficients(K)
    t_start = np.concatenate([[0.0], np.cumsum(h)])
    x_end = np.einsum('k,kl->l', D, X[-1])
    bases = [_lagrange_basis(tau, j) for j in range(K + 1)]

    def interp(t: float) -> np.ndarray:
        t = float(t)
        if t < t_start[0]:
            return X[0, 0].copy()
        n = int(np.searchsorted(t_start, t, side='right')) - 1
        if n >= N:
            return x_end.copy()
        rel = (t - t_start[n]) / h[n]
        out = np.zeros(X.shape[2])
        for j in range(K + 1):
            out += X[n, j] * bases[j](rel)
        return out

    return interp


def interpolate_linear(step_sizes: Sequence[float], X: np.ndarray) -> Callable[[float], np.ndarray]:
    ''' piecewise-linear interpolant of interval start values X (N, n) '''
    h = np.asarray(step_sizes, dtype=float)
    X = np.asarray(X, dtype=float)
    t = np.concatenate([[0.0], np.cumsum(h)])[:-1]

    def interp(tq: float) -> np.ndarray:
        return np.array([np.interp(tq, t, X[:, l]) for l in range(X.shape[1])])

    return interp
