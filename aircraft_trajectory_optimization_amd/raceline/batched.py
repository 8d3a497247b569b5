'''
Batched evaluation of a raceline NLP on one HIP device.

B independent instances share one ProblemSpec (same track, N, K, model). Decision
vectors, constraints, Jacobian values and gradients live in HBM as torch tensors in the
library's INTERLEAVED layout ([element][instance]); evaluation is a single libato call
(ato_eval) on the current torch stream. This is the drop-in for the reference's per-
iterate nlp_g / nlp_jac_g / nlp_f / nlp_grad_f calls (base_raceline.py:165, via IPOPT).
'''
from typing import Optional, Tuple

import numpy as np
import torch

from aircraft_trajectory_optimization_amd import native
from aircraft_trajectory_optimization_amd.raceline.problem import ProblemSpec


class BatchedNLP:
    ''' device-resident batch of NLP instances '''

    def __init__(self, spec: ProblemSpec, batch: int, dtype: torch.dtype = torch.float64,
                 layout: int = native.ATO_LAYOUT_INTERLEAVED, device: Optional[torch.device] = None,
                 buffers: bool = True):
        if not torch.cuda.is_available():
            raise RuntimeError('BatchedNLP needs a HIP device (torch.cuda.is_available() is False)')
        self.device = device or torch.device('cuda', torch.cuda.current_device())
        with torch.cuda.device(self.device):
            self.problem = native.NativeProblem(spec.native_spec())
        self.spec = spec
        self.batch = int(batch)
        self.dtype = dtype
        self.layout = layout
        self.fp32 = dtype == torch.float32
        nw, ng, nnz, B = self.problem.nw, self.problem.ng, self.problem.nnz, self.batch
        shape = (lambda n: (n, B)) if layout == native.ATO_LAYOUT_INTERLEAVED else (lambda n: (B, n))
        opts = {'device': self.device, 'dtype': dtype}
        # resident input / output buffers of evaluate(); buffers=False: the caller passes its own
        # (the solver's evaluator, whose outputs are fresh tensors: at B = 8192 J alone is GBs)
        self.w = torch.zeros(shape(nw), **opts) if buffers else None
        self.g = torch.zeros(shape(ng), **opts) if buffers else None
        self.jac = torch.zeros(shape(nnz), **opts) if buffers else None
        self.grad_f = torch.zeros(shape(nw), **opts) if buffers else None
        self.f = torch.zeros(B, **opts) if buffers else None
        self.problem.reserve(B)
        # evaluations write only the structural nonzeros of grad f (its other entries stay the zeros of
        # the buffers above; the solver's fresh output tensors are zero-filled, solver/batched_ipm.py)
        self.problem.gradf_mode(True)
        self.row_ptr, self.col = self.problem.sparsity()
        self.lbg, self.ubg = self.problem.bounds()
        self.isph = None          # per-instance sphere centres [2 P][B] (set_instance_spheres)

    def set_instance_spheres(self, tables: Optional[np.ndarray]):
        '''
        Per-instance obstacle tubes (config 4): tables (B, P, 3) of (dy, dn, available radius) per
        node, one ObstacleFreeTube.sphere_table per instance (mesh_obstacle.py:219-237). The centres go
        to the device ([2 P][B], read by the sphere rows); lbg / ubg become per-instance (ng, B) arrays
        with each instance's radius^2 in its sphere rows. None returns to the spec's shared table.
        '''
        if tables is None:
            self.isph = None
            self.lbg, self.ubg = self.problem.bounds()
            return
        if self.spec.sphere_table is None:
            raise ValueError('per-instance spheres need a problem with sphere rows (spec.sphere_table)')
        P = self.spec.P
        T = np.asarray(tables, np.float64).reshape(self.batch, P, 3)
        cen = np.ascontiguousarray(T[:, :, :2].reshape(self.batch, 2 * P).T)
        self.isph = torch.as_tensor(cen, device=self.device)
        rows = self.problem.sphere_rows(P)
        lb, ub = self.problem.bounds()
        self.lbg = np.repeat(lb[:, None], self.batch, axis=1)
        self.ubg = np.repeat(ub[:, None], self.batch, axis=1)
        has = rows >= 0
        self.ubg[rows[has], :] = (T[:, has, 2] ** 2).T
        self.sphere_rows = rows

    def _bind_spheres(self):
        ''' the handle may be shared (subset evaluators): point it at this batch's centres '''
        if self.spec.sphere_table is not None:
            self.problem.set_instance_spheres(self.isph.data_ptr() if self.isph is not None else 0, self.batch)

    @property
    def sizes(self) -> Tuple[int, int, int]:
        ''' nw, ng, nnz '''
        return self.problem.nw, self.problem.ng, self.problem.nnz

    def set_w(self, W: np.ndarray):
        ''' W: (B, nw) host array of decision vectors '''
        W = np.asarray(W, dtype=np.float64).reshape(self.batch, -1)
        t = torch.as_tensor(W, dtype=self.dtype)
        if self.layout == native.ATO_LAYOUT_INTERLEAVED:
            t = t.T.contiguous()
        self.w.copy_(t.to(self.device))

    def evaluate(self, g: bool = True, jac: bool = True, cost: bool = True, stream=None):
        ''' launch the evaluation (asynchronous on `stream`, default the current torch stream) '''
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        self._bind_spheres()
        self.problem.eval_ptrs(
            self.batch, self.w.data_ptr(),
            g=self.g.data_ptr() if g else 0,
            jac=self.jac.data_ptr() if jac else 0,
            f=self.f.data_ptr() if cost else 0,
            grad_f=self.grad_f.data_ptr() if cost else 0,
            layout=self.layout, stream=st.cuda_stream, fp32=self.fp32)

    def hessian(self, lam: torch.Tensor, sigma: torch.Tensor, stream=None) -> torch.Tensor:
        '''
        Hessian of the Lagrangian (lower triangle, values in hess_sparsity() order) for multipliers
        lam (same layout as g) and objective factors sigma [B]; fp64 only.
        '''
        if self.fp32:
            raise TypeError('the Hessian is evaluated in fp64')
        if not hasattr(self, 'hess_row_ptr'):
            self.hess_row_ptr, self.hess_col, self.hess_colors = self.problem.hess_sparsity()
            shape = (len(self.hess_col), self.batch) if self.layout == native.ATO_LAYOUT_INTERLEAVED \
                else (self.batch, len(self.hess_col))
            self.hess = torch.zeros(shape, device=self.device, dtype=torch.float64)
            self.problem.reserve(self.batch)
        lam = lam.contiguous()
        sigma = sigma.contiguous()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        self._bind_spheres()
        self.problem.hess_eval_ptrs(self.batch, self.w.data_ptr(), lam.data_ptr(), sigma.data_ptr(),
                                    self.hess.data_ptr(), layout=self.layout, stream=st.cuda_stream)
        return self.hess

    def _host(self, t: torch.Tensor) -> np.ndarray:
        a = t.detach().to('cpu', torch.float64).numpy()
        return a.T.copy() if self.layout == native.ATO_LAYOUT_INTERLEAVED else a

    def results(self):
        ''' (g (B, ng), jac values (B, nnz), f (B,), grad_f (B, nw)) on the host '''
        torch.cuda.synchronize(self.device)
        return self._host(self.g), self._host(self.jac), self.f.detach().cpu().double().numpy(), \
            self._host(self.grad_f)
