'''
The batched solver's sparse products (solver/batched_ipm.py: J x, J^T y, W x and the whole
augmented-system product K v used by iterative refinement) against scipy on random values.
The structure has empty Jacobian rows and columns and empty Hessian rows, so zero-length
segments of torch.segment_reduce (unsafe=True: no input validation) are exercised.
'''
import numpy as np
import scipy.sparse as sp
import torch

from aircraft_trajectory_optimization_amd.solver.batched_ipm import BatchedInteriorPoint


class _Structure:
    ''' duck-typed evaluator: only the sparsity and sizes the constructor reads '''

    def __init__(self, n, m, B, seed):
        rng = np.random.default_rng(seed)
        self.n, self.m, self.batch, self.device = n, m, B, torch.device('cpu')
        dense = rng.random((m, n)) < 0.25
        dense[:, [1, 4]] = False                 # empty Jacobian columns
        dense[[0, 3]] = False                    # empty Jacobian rows
        r, c = np.nonzero(dense)
        self.j_row_ptr = np.concatenate([[0], np.cumsum(dense.sum(1))]).astype(np.int64)
        self.j_col = c.astype(np.int64)
        low = np.tril(rng.random((n, n)) < 0.3)
        low[[2, 5]] = False                      # empty Hessian rows (lower triangle) ...
        low[:, 2] = False                        # ... and column 2 untouched entirely
        np.fill_diagonal(low, False)
        low[np.arange(0, n, 3), np.arange(0, n, 3)] = True   # some diagonal entries
        low[2, 2] = False
        hr, hc = np.nonzero(low)
        self.h_row_ptr = np.concatenate([[0], np.cumsum(low.sum(1))]).astype(np.int64)
        self.h_col = hc.astype(np.int64)
        self.lbg = np.zeros(m)
        self.ubg = np.where(np.arange(m) % 2 == 0, 0.0, 1.0)   # equalities and inequalities
        self.nnz_j, self.nnz_h = len(c), len(hc)
        self._jr, self._hr = r, hr


def test_sparse_products_match_scipy():
    n, m, B = 11, 9, 3
    st = _Structure(n, m, B, seed=4)
    ipm = BatchedInteriorPoint(st, None, np.full(n, -1.0), np.full(n, 1.0))
    rng = np.random.default_rng(9)
    Js = torch.as_tensor(rng.standard_normal((st.nnz_j, B)))
    H = torch.as_tensor(rng.standard_normal((st.nnz_h, B)))
    dx = torch.as_tensor(rng.standard_normal((n, B)))
    dr = torch.as_tensor(rng.standard_normal((m, B)))
    v = torch.as_tensor(rng.standard_normal((n + m, B)))
    for b in range(B):
        J = sp.csr_matrix((Js[:, b].numpy(), (st._jr, st.j_col)), shape=(m, n))
        L = sp.csr_matrix((H[:, b].numpy(), (st._hr, st.h_col)), shape=(n, n))
        W = L + sp.triu(L.T, k=1)
        vx, vy = v[:n, b].numpy(), v[n:, b].numpy()
        assert np.allclose(ipm._Jx(Js, v[:n])[:, b].numpy(), J @ vx, rtol=1e-14, atol=1e-14)
        assert np.allclose(ipm._JTy(Js, v[n:])[:, b].numpy(), J.T @ vy, rtol=1e-14, atol=1e-14)
        assert np.allclose(ipm._Wx(H, v[:n])[:, b].numpy(), W @ vx, rtol=1e-14, atol=1e-14)
        K = sp.bmat([[W + sp.diags(dx[:, b].numpy()), J.T], [J, sp.diags(dr[:, b].numpy())]], format='csr')
        assert np.allclose(ipm._Kmul(H, Js, dx, dr, v)[:, b].numpy(), K @ v[:, b].numpy(), rtol=1e-14, atol=1e-13)
        # no Hessian (least-squares multiplier system): K = [diag_x J^T; J diag_r]
        K0 = sp.bmat([[sp.diags(dx[:, b].numpy()), J.T], [J, sp.diags(dr[:, b].numpy())]], format='csr')
        assert np.allclose(ipm._Kmul(None, Js, dx, dr, v)[:, b].numpy(), K0 @ v[:, b].numpy(),
                           rtol=1e-14, atol=1e-13)
