'''
Shared test fixtures: tracks, product / oracle problem construction, host-check loader.
'''
import ctypes
import os
import subprocess

import numpy as np

from aircraft_trajectory_optimization_amd import native

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

from aircraft_trajectory_optimization_amd.tracks import TRACKS, make_line as product_line, \
    make_spec as product_spec  # noqa: F401


def oracle_line(track, closed=True):
    from oracle.ref_geometry import RefCenterline
    x, shape = TRACKS[track]
    return RefCenterline(np.array(x, float), closed, gate_shape=shape)


def oracle_nlp(track='race', model='drone', frame='parametric', N=50, K=4, use_quat=True, global_r=True,
               fix_gate_center=False, quat_flip=False, spheres=None, v0=1.0, h0=1, rk4=False, closed=True,
               euler_wraps=0.0, use_dcm=False, cpc=None):
    from oracle.ref_transcription import RefNLP
    line = oracle_line(track, closed)
    veh = {'use_quat': use_quat, 'global_r': global_r, 'use_dcm': use_dcm} if model == 'drone' else \
        {'global_r': global_r}
    fixed = (line.s[:-1] if closed else line.s) if frame == 'parametric' else None
    return RefNLP(line, model, frame, N, K, veh=veh, fix_gate_center=fix_gate_center, fixed_gates=fixed,
                  quat_flip=quat_flip, spheres=spheres, v0=v0, h0=h0, rk4=rk4, closed=closed,
                  euler_wraps=euler_wraps, cpc=cpc)


def random_w(spec_or_nlp, rng, scale=0.05):
    ''' a seeded point near w0, strictly inside the box, with unit-ish quaternions '''
    w0 = np.array(spec_or_nlp.w0, float)
    w = w0 + scale * rng.standard_normal(w0.shape)
    N = spec_or_nlp.N
    w[:N] = np.abs(w0[:N]) * (1 + 0.2 * rng.random(N))
    return w


def sym_dense(row_ptr, col, vals, n):
    ''' symmetric dense matrix from a lower-triangle CSR '''
    H = np.zeros((n, n))
    for r in range(n):
        c = col[row_ptr[r]:row_ptr[r + 1]]
        H[r, c] = vals[row_ptr[r]:row_ptr[r + 1]]
    return H + np.tril(H, -1).T


def csr_dense(row_ptr, col, vals, ng, nw):
    J = np.zeros((ng, nw))
    for r in range(ng):
        J[r, col[row_ptr[r]:row_ptr[r + 1]]] = vals[row_ptr[r]:row_ptr[r + 1]]
    return J


# ------------------------------------------------------------------ test-only CPU build of the programs
HOSTCHECK_SRC = os.path.join(REPO, 'tests', 'native', 'hostcheck.cpp')
HOSTCHECK_LIB = os.path.join(REPO, 'tests', 'native', 'libato_hostcheck.so')


def build_hostcheck(force=False):
    srcs = [HOSTCHECK_SRC] + [os.path.join(REPO, 'aircraft_trajectory_optimization_amd', 'csrc', f)
                              for f in ('ato_models.hpp', 'ato_dual.hpp', 'ato_program.hpp', 'ato_layout.hpp',
                                        'ato_hessian.hpp')]
    if not force and os.path.exists(HOSTCHECK_LIB) and \
            os.path.getmtime(HOSTCHECK_LIB) >= max(os.path.getmtime(s) for s in srcs):
        return HOSTCHECK_LIB
    # x86-64-v3 (AVX2), not -march=native: the library is built here and also runs on the GPU box's host
    subprocess.check_call(['g++', '-std=c++20', '-O3', '-march=x86-64-v3', '-fopenmp', '-fPIC', '-shared', '-o',
                           HOSTCHECK_LIB, HOSTCHECK_SRC])
    return HOSTCHECK_LIB


class HostCheck:
    ''' the segment programs compiled for the CPU (test harness only) '''

    def __init__(self, spec_dict):
        lib = ctypes.CDLL(build_hostcheck())
        vp = ctypes.c_void_p
        lib.atoh_create.argtypes = [ctypes.POINTER(native.AtoProblemDesc), ctypes.POINTER(vp)]
        lib.atoh_last_error.restype = ctypes.c_char_p
        lib.atoh_eval.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, vp]
        lib.atoh_eval_threads.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, vp, ctypes.c_int]
        lib.atoh_destroy.argtypes = [vp]
        lib.atoh_sizes.argtypes = [vp] + [ctypes.POINTER(ctypes.c_int32)] * 3
        lib.atoh_sparsity.argtypes = [vp, vp, vp]
        lib.atoh_bounds.argtypes = [vp, vp, vp]
        lib.atoh_hess_sparsity.argtypes = [vp, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]
        lib.atoh_hess_pattern.argtypes = [vp, vp, vp]
        lib.atoh_hess_eval.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp]
        lib.atoh_set_instance_spheres.argtypes = [vp, vp, ctypes.c_long]
        lib.atoh_sphere_rows.argtypes = [vp, vp]
        self.lib = lib
        self.holder = native.DescHolder(spec_dict)
        h = vp()
        if lib.atoh_create(ctypes.byref(self.holder.desc), ctypes.byref(h)) != 0:
            raise RuntimeError(lib.atoh_last_error().decode())
        self.h = h
        a, b, c = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        lib.atoh_sizes(h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        self.nw, self.ng, self.nnz = a.value, b.value, c.value
        self.row_ptr = np.zeros(self.ng + 1, np.int32)
        self.col = np.zeros(self.nnz, np.int32)
        lib.atoh_sparsity(h, self.row_ptr.ctypes.data, self.col.ctypes.data)
        self.lbg = np.zeros(self.ng)
        self.ubg = np.zeros(self.ng)
        lib.atoh_bounds(h, self.lbg.ctypes.data, self.ubg.ctypes.data)

    def set_instance_spheres(self, centres):
        ''' per-instance sphere centres: host [2 P][B] array (kept alive here) or None '''
        self._isph = None if centres is None else np.ascontiguousarray(centres, np.float64)
        ptr = self._isph.ctypes.data if self._isph is not None else None
        stride = self._isph.shape[1] if self._isph is not None else 0
        if self.lib.atoh_set_instance_spheres(self.h, ptr, stride) != 0:
            raise RuntimeError(self.lib.atoh_last_error().decode())

    def sphere_rows(self, P):
        rows = np.zeros(P, np.int32)
        self.lib.atoh_sphere_rows(self.h, rows.ctypes.data)
        return rows

    def eval(self, W):
        ''' W: (B, nw) -> g (B, ng), J (B, nnz), f (B,), grad_f (B, nw) '''
        W = np.ascontiguousarray(np.atleast_2d(W), dtype=np.float64)
        B = W.shape[0]
        g = np.zeros((B, self.ng))
        J = np.zeros((B, self.nnz))
        f = np.zeros(B)
        gf = np.zeros((B, self.nw))
        rc = self.lib.atoh_eval(self.h, B, W.ctypes.data, g.ctypes.data, J.ctypes.data, f.ctypes.data,
                                gf.ctypes.data)
        if rc != 0:
            raise RuntimeError(self.lib.atoh_last_error().decode())
        return g, J, f, gf

    def eval_threads(self, W, nthreads, out=None):
        ''' W (B, nw) -> the same outputs as eval, instances over nthreads OpenMP threads '''
        W = np.ascontiguousarray(np.atleast_2d(W), dtype=np.float64)
        B = W.shape[0]
        if out is None:
            out = (np.zeros((B, self.ng)), np.zeros((B, self.nnz)), np.zeros(B), np.zeros((B, self.nw)))
        g, J, f, gf = out
        rc = self.lib.atoh_eval_threads(self.h, B, W.ctypes.data, g.ctypes.data, J.ctypes.data, f.ctypes.data,
                                        gf.ctypes.data, int(nthreads))
        if rc != 0:
            raise RuntimeError(self.lib.atoh_last_error().decode())
        return out

    def hess_pattern(self):
        nnz, nc = ctypes.c_int32(), ctypes.c_int32()
        if self.lib.atoh_hess_sparsity(self.h, ctypes.byref(nnz), ctypes.byref(nc)) != 0:
            raise RuntimeError(self.lib.atoh_last_error().decode())
        rp = np.zeros(self.nw + 1, np.int32)
        col = np.zeros(nnz.value, np.int32)
        self.lib.atoh_hess_pattern(self.h, rp.ctypes.data, col.ctypes.data)
        return rp, col, nc.value

    def hess(self, W, LAM, sigma):
        ''' W (B, nw), LAM (B, ng), sigma (B,) -> lower-triangle values (B, nnz_h) '''
        rp, col, _ = self.hess_pattern()
        W = np.ascontiguousarray(np.atleast_2d(W), dtype=np.float64)
        LAM = np.ascontiguousarray(np.atleast_2d(LAM), dtype=np.float64)
        sig = np.ascontiguousarray(np.atleast_1d(sigma), dtype=np.float64)
        H = np.zeros((W.shape[0], len(col)))
        if self.lib.atoh_hess_eval(self.h, W.shape[0], W.ctypes.data, LAM.ctypes.data, sig.ctypes.data,
                                   H.ctypes.data) != 0:
            raise RuntimeError(self.lib.atoh_last_error().decode())
        return H

    def __del__(self):
        try:
            self.lib.atoh_destroy(self.h)
        except Exception:  # pylint: disable=broad-except
            pass


class HostEvaluator:
    ''' evaluator interface of solver.ipm over the CPU build of the programs (tests only) '''

    def __init__(self, spec):
        self.hc = HostCheck(spec.native_spec())
        self.nw, self.ng = self.hc.nw, self.hc.ng
        self.j_row_ptr, self.j_col = self.hc.row_ptr, self.hc.col
        self.h_row_ptr, self.h_col, _ = self.hc.hess_pattern()
        self.lbg, self.ubg = self.hc.lbg, self.hc.ubg
        self.var_stage = var_stages(spec)

    def eval(self, x):
        g, J, f, gf = self.hc.eval(x)
        return f[0], g[0], gf[0], J[0]

    def hess(self, x, lam, sigma):
        return self.hc.hess(x, lam, sigma)[0]


def var_stages(spec):
    ''' interval of every decision variable: h_n -> n, node (n, k) -> n (CPC progress of node q: q's) '''
    from aircraft_trajectory_optimization_amd.raceline.evaluator import variable_stages
    return variable_stages(spec)


# ------------------------------------------------------------------ golden fixtures of the reference's own transcription
GOLDEN_DIR = os.path.join(REPO, 'tests', 'golden', 'transcription')
DIRECTIONAL_DIR = os.path.join(REPO, 'tests', 'golden', 'directional')


def golden_names(directory=GOLDEN_DIR):
    return sorted(f[:-4] for f in os.listdir(directory) if f.endswith('.npz'))


def directional_names():
    ''' the bench-size fixtures: g, f, J V and grad f . V along seeded directions V '''
    return golden_names(DIRECTIONAL_DIR)


def golden_case(name, directory=GOLDEN_DIR):
    ''' (fixture dict, keyword arguments for product_spec / oracle_nlp) of one golden case
    (tests/golden/make_transcription_golden.py). Warm-started cases carry the closure sign /
    Euler wraps the reference derives from its first and last guessed attitude
    (drone_raceline.py:81-95). '''
    import json
    d = dict(np.load(os.path.join(directory, f'{name}.npz')))
    cfg = json.loads(str(d['cfg']))
    kw = {k: v for k, v in cfg.items() if k not in ('spheres', 'warm')}
    if 'spheres' in d:
        kw['spheres'] = d['spheres']
    if 'ws_first_r' in d:
        first, last = d['ws_first_r'], d['ws_last_r']
        if kw.get('use_quat', True):
            kw['quat_flip'] = bool(np.linalg.norm(first - last) > 1)
        else:
            kw['euler_wraps'] = float(np.round((last - first)[0] / 2 / np.pi))
    return d, kw


def csr_matvec(row_ptr, col, vals, V):
    ''' (CSR values) @ V for a dense V (n, k) '''
    import scipy.sparse as sp
    n = len(row_ptr) - 1
    return sp.csr_matrix((vals, col, row_ptr), shape=(n, V.shape[0])) @ V


def golden_jacobian(d, i):
    J = np.zeros((int(d['ng']), int(d['nw'])))
    J[d['J_row'], d['J_col']] = d['J_val'][i]
    return J


# ------------------------------------------------------------------ KKT certificate against the oracle
def kkt_certificate(nlp, x, lam_g, lam_x, lbw, ubw):
    '''
    First-order optimality of x for the reference NLP as the ORACLE states it (not the product's
    evaluator): {primal, dual, compl} in unscaled quantities.
      primal  max violation of lbg <= g(x) <= ubg and lbw <= x <= ubw
      dual    |grad f + J^T lam_g + lam_x|_inf            (IPOPT's sign convention)
      compl   max over active-multiplier constraints of |multiplier| * distance to its bound
    '''
    x = np.asarray(x, float)
    lam_g, lam_x = np.asarray(lam_g, float), np.asarray(lam_x, float)
    g = nlp.g(x)
    lbg, ubg = np.asarray(nlp.lbg, float), np.asarray(nlp.ubg, float)
    lbw, ubw = np.asarray(lbw, float), np.asarray(ubw, float)
    primal = max(np.max(np.maximum(lbg - g, 0), initial=0), np.max(np.maximum(g - ubg, 0), initial=0),
                 np.max(np.maximum(lbw - x, 0), initial=0), np.max(np.maximum(x - ubw, 0), initial=0))
    dual = np.abs(nlp.grad_lagrangian(x, lam_g, 1.0) + lam_x).max()

    def comp(v, lam, lo, hi):
        eq = lo == hi
        with np.errstate(invalid='ignore'):
            up = np.where((lam > 0) & np.isfinite(hi) & ~eq, lam * np.maximum(hi - v, 0), 0)
            dn = np.where((lam < 0) & np.isfinite(lo) & ~eq, -lam * np.maximum(v - lo, 0), 0)
        return max(np.max(up, initial=0), np.max(dn, initial=0))
    compl = max(comp(g, lam_g, lbg, ubg), comp(x, lam_x, lbw, ubw))
    return {'primal': float(primal), 'dual': float(dual), 'compl': float(compl)}
