'''
Structure-exploiting factorisation of the raceline KKT system (replaces IPOPT's MUMPS / MA97
LDL^T, base_raceline.py:765-782).

    K = [ W + Sigma + delta_w I    J^T      ]
        [ J                       -D        ]

The transcription is a chain of intervals: every decision variable belongs to one interval
(stage), the Hessian is block diagonal by stage, and almost every constraint row touches one
stage or two neighbouring ones (continuity, joined to the later stage). Ordering each stage's
variables and rows together makes K block tridiagonal; the few rows that reach further (loop closure, equal step sizes of
the global frame) form a border eliminated last:

    S_0 = A_0,   S_n = A_n - B_n S_{n-1}^{-1} B_n^T
    C~_0 = C_0,  C~_n = C_n - C~_{n-1} S_{n-1}^{-1} B_n^T
    S_b = A_b - sum_n C~_n S_n^{-1} C~_n^T

Each S_n is factorised with Bunch-Kaufman LDL^T (LAPACK sytrf), so the inertia of K is the sum
of the inertias of the S_n and S_b (Haynsworth) -- exactly what IPOPT's inertia correction needs.
'''
from typing import Optional, Tuple

import numpy as np
import scipy.sparse as sp
from scipy.linalg import lapack


def _inertia_ldl(ldu, ipiv):
    ''' (n_pos, n_neg, n_zero) of a sytrf factor (lower storage): 1x1 pivots by sign, 2x2
    pivots [[a, b], [b, c]] (ipiv < 0 on both rows) by determinant and trace '''
    d = np.diag(ldu)
    two = ipiv < 0
    # rows of 2x2 blocks come in pairs: the first row of every pair
    idx2 = np.nonzero(two)[0][::2]
    one = ~two
    pos = int((d[one] > 0).sum())
    neg = int((d[one] < 0).sum())
    zero = int((d[one] == 0).sum())
    if len(idx2):
        a, c = d[idx2], d[idx2 + 1]
        b = ldu[idx2 + 1, idx2]
        det = a * c - b * b
        tr = a + c
        pos += int((det < 0).sum() + 2 * ((det > 0) & (tr > 0)).sum() + ((det == 0) & (tr > 0)).sum())
        neg += int((det < 0).sum() + 2 * ((det > 0) & (tr < 0)).sum() + ((det == 0) & (tr < 0)).sum())
        zero += int((det == 0).sum() + ((det == 0) & (tr == 0)).sum())
    return pos, neg, zero


class _Factor:
    ''' dense symmetric indefinite factor of one block '''

    def __init__(self, S: np.ndarray):
        self.n = S.shape[0]
        if self.n == 0:
            self.ldu, self.ipiv, self.info = S, np.zeros(0, np.int32), 0
            self.inertia = (0, 0, 0)
            return
        self.ldu, self.ipiv, self.info = lapack.dsytrf(S, lower=1, lwork=max(1, 64 * self.n))
        self.inertia = _inertia_ldl(self.ldu, self.ipiv) if self.info >= 0 else (0, 0, self.n)
        if self.info > 0:                      # exactly singular D block
            self.inertia = (self.inertia[0], self.inertia[1], max(1, self.inertia[2]))

    def solve(self, B: np.ndarray) -> np.ndarray:
        if self.n == 0:
            return B.copy()
        B2 = B.reshape(self.n, -1)
        x, info = lapack.dsytrs(self.ldu, self.ipiv, B2, lower=1)
        return x.reshape(B.shape)


class BlockKKT:
    '''
    Block structure of the KKT matrix for one problem: var_stage[j] (interval of variable j),
    Jacobian CSR pattern, lower-CSR Hessian pattern. Rows that touch one stage or two
    neighbouring stages join the later one; all other rows form the border.
    '''

    def __init__(self, n: int, m: int, var_stage: np.ndarray, j_row_ptr, j_col, h_row_ptr, h_col):
        self.n, self.m = n, m
        var_stage = np.asarray(var_stage)
        self.S = int(var_stage.max()) + 1
        jr = np.repeat(np.arange(m), np.diff(j_row_ptr))
        st = var_stage[np.asarray(j_col)]
        lo = np.full(m, np.iinfo(np.int64).max)
        hi = np.full(m, -1)
        np.minimum.at(lo, jr, st)
        np.maximum.at(hi, jr, st)
        # rows spanning two neighbouring stages join the LATER one: a continuity row then carries
        # its identity entry on the new interval's first node inside its own block (joined to the
        # earlier stage, a quaternion continuity block would keep only its rank-3 normalisation
        # Jacobian and leave that stage block singular)
        row_stage = np.where(hi - lo <= 1, hi, -1)
        row_stage[hi < 0] = 0                       # empty rows (none expected)
        self.row_stage = row_stage
        # global ordering: per stage [variables, rows], then border rows
        order, self.blocks = [], []
        for s in range(self.S):
            v = np.nonzero(var_stage == s)[0]
            r = n + np.nonzero(row_stage == s)[0]
            idx = np.concatenate([v, r])
            self.blocks.append(np.arange(len(order), len(order) + len(idx)))
            order.extend(idx.tolist())
        border = n + np.nonzero(row_stage < 0)[0]
        self.border = np.arange(len(order), len(order) + len(border))
        order.extend(border.tolist())
        self.perm = np.asarray(order)               # position -> original index
        self.n_border = len(border)
        # check the Hessian keeps to one stage
        hr = np.repeat(np.arange(n), np.diff(h_row_ptr))
        if len(hr) and np.any(var_stage[hr] != var_stage[np.asarray(h_col)]):
            raise ValueError('Hessian couples different stages; block ordering does not apply')
        self.bounds = [(b[0], b[-1] + 1) if len(b) else (0, 0) for b in self.blocks]

    def factor(self, K: sp.spmatrix) -> Tuple[Optional['BlockFactor'], Tuple[int, int, int]]:
        ''' K: full symmetric sparse matrix in the original ordering (n + m) '''
        Kp = K.tocsr()[self.perm][:, self.perm].tocsr()
        f = BlockFactor(self, Kp)
        return f, f.inertia


class BlockFactor:
    def __init__(self, st: BlockKKT, Kp: sp.csr_matrix):
        self.st = st
        b = st.bounds
        nb = st.border
        bsl = slice(nb[0], nb[-1] + 1) if len(nb) else slice(0, 0)
        self.bsl = bsl
        self.F, self.B, self.Ct = [], [], []
        pos = neg = zero = 0
        Sprev = None
        Ctil = None
        Sb = Kp[bsl, bsl].toarray() if len(nb) else np.zeros((0, 0))
        for s in range(st.S):
            sl = slice(*b[s])
            A = Kp[sl, sl].toarray()
            C = Kp[bsl, sl].toarray() if len(nb) else np.zeros((0, b[s][1] - b[s][0]))
            if s > 0:
                Bn = Kp[sl, slice(*b[s - 1])].toarray()        # coupling stage s <- s-1
                X = Sprev.solve(Bn.T)                           # S_{s-1}^{-1} B_s^T
                A = A - Bn @ X
                C = C - Ctil @ X
            else:
                Bn = None
            self.B.append(Bn)
            Fs = _Factor(A)
            self.F.append(Fs)
            p, q, z = Fs.inertia
            pos, neg, zero = pos + p, neg + q, zero + z
            if len(nb):
                Sb -= C @ Fs.solve(C.T)
            self.Ct.append(C)
            Sprev, Ctil = Fs, C
        self.Fb = _Factor(Sb)
        p, q, z = self.Fb.inertia
        self.inertia = (pos + p, neg + q, zero + z)

    def solve(self, rhs: np.ndarray) -> np.ndarray:
        st = self.st
        r = rhs[st.perm].astype(float)
        b = st.bounds
        y = [None] * st.S
        yb = r[self.bsl].copy()
        for s in range(st.S):
            ys = r[slice(*b[s])].copy()
            if s > 0:
                ys -= self.B[s] @ self.F[s - 1].solve(y[s - 1])
            y[s] = ys
            if len(yb):
                yb -= self.Ct[s] @ self.F[s].solve(ys)
        xb = self.Fb.solve(yb) if len(yb) else yb
        x = [None] * st.S
        for s in reversed(range(st.S)):
            t = y[s].copy()
            if s + 1 < st.S:
                t -= self.B[s + 1].T @ x[s + 1]
            if len(xb):
                t -= self.Ct[s].T @ xb
            x[s] = self.F[s].solve(t)
        out = np.empty_like(r)
        for s in range(st.S):
            out[slice(*b[s])] = x[s]
        out[self.bsl] = xb
        res = np.empty_like(out)
        res[st.perm] = out
        return res
