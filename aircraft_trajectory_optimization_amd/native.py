'''
ctypes binding of libato.so (include/ato.h).

This is the only way the package evaluates the NLP: there is no CPU fallback. If the
HIP library is missing or cannot be loaded, `load()` raises.
'''
import ctypes
import os
from typing import Optional, Tuple

import numpy as np

KMAX = 9
GEOM_WIDTH = 16

ATO_MODEL_DRONE, ATO_MODEL_POINT = 0, 1
ATO_ATT_ESP, ATO_ATT_YPR, ATO_ATT_DCM = 0, 1, 2
ATO_FRAME_GLOBAL, ATO_FRAME_PARAMETRIC = 0, 1
ATO_TRANS_COLLOCATION, ATO_TRANS_RK4 = 0, 1
ATO_GATE_CIRCLE, ATO_GATE_SQUARE = 0, 1
ATO_LAYOUT_INTERLEAVED, ATO_LAYOUT_INSTANCE_MAJOR = 0, 1
ABI_VERSION = 3
CPC_MAX = 16                 # ATO_CPC_MAX

_c_double_p = ctypes.POINTER(ctypes.c_double)


class AtoGate(ctypes.Structure):
    ''' mirror of ato_gate '''
    _fields_ = [
        ('interval', ctypes.c_int32),
        ('shape', ctypes.c_int32),
        ('fix_center', ctypes.c_int32),
        ('axial', ctypes.c_int32),
        ('at_end', ctypes.c_int32),
        ('n_coef', ctypes.c_int32),
        ('coef', ctypes.c_double * (KMAX + 1)),
        ('gate_x', ctypes.c_double * 3),
        ('R', ctypes.c_double * 9),
        ('xc', ctypes.c_double * 3),
        ('ey', ctypes.c_double * 3),
        ('en', ctypes.c_double * 3),
        ('d_max', ctypes.c_double),
    ]


class AtoProblemDesc(ctypes.Structure):
    ''' mirror of ato_problem_desc '''
    _fields_ = [
        ('abi_version', ctypes.c_int32),
        ('model', ctypes.c_int32),
        ('attitude', ctypes.c_int32),
        ('frame', ctypes.c_int32),
        ('global_r', ctypes.c_int32),
        ('transcription', ctypes.c_int32),
        ('N', ctypes.c_int32),
        ('K', ctypes.c_int32),
        ('closed', ctypes.c_int32),
        ('cleanly_closed', ctypes.c_int32),
        ('quat_flip', ctypes.c_int32),
        ('force_regularity', ctypes.c_int32),
        ('n_gates', ctypes.c_int32),
        ('phase_len', ctypes.c_int32),
        ('has_spheres', ctypes.c_int32),
        ('pad0', ctypes.c_int32),
        ('euler_wraps', ctypes.c_double),
        ('gamma', ctypes.c_double),
        ('m', ctypes.c_double),
        ('g', ctypes.c_double),
        ('b', ctypes.c_double * 3),
        ('I', ctypes.c_double * 3),
        ('bw', ctypes.c_double * 3),
        ('l', ctypes.c_double),
        ('kt', ctypes.c_double),
        ('T_max', ctypes.c_double),
        ('Rcost', ctypes.c_double * 16),
        ('dRcost', ctypes.c_double * 16),
        ('tau', ctypes.c_double * (KMAX + 1)),
        ('Bq', ctypes.c_double * (KMAX + 1)),
        ('C', ctypes.c_double * ((KMAX + 1) * (KMAX + 1))),
        ('D', ctypes.c_double * (KMAX + 1)),
        ('A_skew', ctypes.c_double * 4),
        ('node_geom', _c_double_p),
        ('node_s', _c_double_p),
        ('interval_s', _c_double_p),
        ('gates', ctypes.POINTER(AtoGate)),
        ('spheres', _c_double_p),
        ('cpc_m', ctypes.c_int32),
        ('pad1', ctypes.c_int32),
        ('cpc_wp', ctypes.c_double * (CPC_MAX * 3)),
    ]


class AtoIpmDims(ctypes.Structure):
    ''' include/ato_ipm.h ato_ipm_dims '''
    _fields_ = [('n', ctypes.c_int32), ('m', ctypes.c_int32), ('mi', ctypes.c_int32), ('meq', ctypes.c_int32),
                ('iin', ctypes.c_void_p), ('ieq', ctypes.c_void_p), ('W', ctypes.c_int32)]


class AtoIpmBounds(ctypes.Structure):
    ''' include/ato_ipm.h ato_ipm_bounds '''
    _fields_ = [('xL', ctypes.c_void_p), ('xU', ctypes.c_void_p), ('dL', ctypes.c_void_p), ('dU', ctypes.c_void_p)]


IPM_SYMBOLS = ('ato_ipm_work_size', 'ato_ipm_errors', 'ato_ipm_rhs', 'ato_ipm_direction', 'ato_ipm_measures',
               'ato_ipm_multipliers', 'ato_ipm_filter_accept', 'ato_ipm_kkt_diag', 'ato_ipm_perturb',
               'ato_ipm_status', 'ato_ipm_barrier', 'ato_ipm_filter_multi', 'ato_ipm_refine_work',
               'ato_ipm_refine_pass', 'ato_ipm_refine_decide', 'ato_ipm_resto_rows', 'ato_ipm_js_jty')

EXPORTED_SYMBOLS = ('ato_create', 'ato_destroy', 'ato_sizes', 'ato_sparsity', 'ato_bounds',
                    'ato_reserve', 'ato_eval', 'ato_eval_f32', 'ato_hess_sparsity', 'ato_hess_eval',
                    'ato_mesh_create', 'ato_mesh_destroy', 'ato_mesh_signed_distance',
                    'ato_timing', 'ato_timing_read', 'ato_timing_stride', 'ato_last_error', 'ato_version',
                    'ato_kkt_create', 'ato_kkt_destroy', 'ato_kkt_reserve', 'ato_kkt_factor', 'ato_kkt_solve',
                    'ato_kkt_residual', 'ato_kkt_residual_list', 'ato_set_instance_spheres',
                    'ato_sphere_rows', 'ato_gradf_mode', 'ato_gradf_sparsity') + IPM_SYMBOLS


def library_path() -> str:
    ''' in-tree location of the HIP library (ATO_LIB_PATH overrides it: diagnostic kernel variants) '''
    return os.environ.get('ATO_LIB_PATH') or os.path.join(os.path.dirname(os.path.abspath(__file__)), '_lib',
                                                          'libato.so')


def declare(lib: ctypes.CDLL, prefix: str = 'ato') -> ctypes.CDLL:
    ''' attach argtypes / restypes '''
    vp = ctypes.c_void_p
    i32p = ctypes.POINTER(ctypes.c_int32)
    getattr(lib, f'{prefix}_last_error').restype = ctypes.c_char_p
    if prefix == 'ato':
        lib.ato_version.restype = ctypes.c_char_p
        lib.ato_create.argtypes = [ctypes.POINTER(AtoProblemDesc), ctypes.POINTER(vp)]
        lib.ato_destroy.argtypes = [vp]
        lib.ato_sizes.argtypes = [vp, i32p, i32p, i32p]
        lib.ato_sparsity.argtypes = [vp, ctypes.POINTER(i32p), ctypes.POINTER(i32p)]
        lib.ato_bounds.argtypes = [vp, _c_double_p, _c_double_p]
        lib.ato_reserve.argtypes = [vp, ctypes.c_int32]
        lib.ato_eval.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, vp, vp]
        lib.ato_eval_f32.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, vp, vp]
        lib.ato_hess_sparsity.argtypes = [vp, i32p, ctypes.POINTER(i32p), ctypes.POINTER(i32p), i32p]
        lib.ato_hess_eval.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, vp]
        lib.ato_mesh_create.argtypes = [vp, ctypes.c_int32, vp, ctypes.c_int32, ctypes.POINTER(vp)]
        lib.ato_mesh_destroy.argtypes = [vp]
        lib.ato_mesh_signed_distance.argtypes = [vp, ctypes.c_int32, vp, vp, vp, vp]
        lib.ato_timing.argtypes = [vp, ctypes.c_int32]
        lib.ato_timing_read.argtypes = [vp, _c_double_p, _c_double_p, i32p]
        lib.ato_timing_stride.argtypes = [vp, ctypes.c_int32]
        lib.ato_set_instance_spheres.argtypes = [vp, vp, ctypes.c_int64]
        lib.ato_sphere_rows.argtypes = [vp, i32p]
        lib.ato_gradf_mode.argtypes = [vp, ctypes.c_int32]
        lib.ato_gradf_sparsity.argtypes = [vp, i32p, i32p]
        lib.ato_kkt_create.argtypes = [vp, ctypes.POINTER(vp)]
        lib.ato_kkt_destroy.argtypes = [vp]
        lib.ato_kkt_reserve.argtypes = [vp, ctypes.c_int32]
        lib.ato_kkt_factor.argtypes = [vp, ctypes.c_int32, vp, ctypes.c_int64, ctypes.c_int64, vp, vp, vp, vp, vp, vp]
        lib.ato_kkt_solve.argtypes = [vp, ctypes.c_int32, vp, ctypes.c_int64, ctypes.c_int64, vp, vp]
        lib.ato_kkt_residual.argtypes = [vp, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, vp, vp, vp, vp, vp, vp,
                                         vp, vp]
        lib.ato_kkt_residual_list.argtypes = [vp, ctypes.c_int32, vp, ctypes.c_int64, ctypes.c_int64, vp, vp, vp,
                                              vp, vp, vp, vp, vp]
        for fn in ('ato_kkt_create', 'ato_kkt_destroy', 'ato_kkt_reserve', 'ato_kkt_factor', 'ato_kkt_solve',
                   'ato_kkt_residual', 'ato_kkt_residual_list'):
            getattr(lib, fn).restype = ctypes.c_int
        dp, bp, d = ctypes.POINTER(AtoIpmDims), ctypes.POINTER(AtoIpmBounds), ctypes.c_double
        lib.ato_ipm_work_size.argtypes = [dp]
        lib.ato_ipm_work_size.restype = ctypes.c_size_t
        lib.ato_ipm_errors.argtypes = [dp, bp] + [vp] * 12 + [vp, d, vp, vp, vp]
        lib.ato_ipm_rhs.argtypes = [dp, bp] + [vp] * 12 + [d] + [vp] * 7 + [vp]
        lib.ato_ipm_direction.argtypes = [dp, bp] + [vp] * 12 + [vp] * 4 + [vp, vp, vp]
        lib.ato_ipm_measures.argtypes = [dp, bp] + [vp] * 6 + [d, vp, vp, vp]
        lib.ato_ipm_multipliers.argtypes = [dp, bp, vp, vp, vp, vp, d] + [vp] * 8 + [vp]
        lib.ato_ipm_filter_accept.argtypes = [ctypes.c_int32, ctypes.c_int32] + [vp] * 19 + [vp]
        lib.ato_ipm_kkt_diag.argtypes = [dp] + [vp] * 7 + [vp]
        lib.ato_ipm_filter_multi.argtypes = [ctypes.c_int32] * 3 + [vp] * 18 + [vp]
        lib.ato_ipm_perturb.argtypes = [ctypes.c_int32] * 3 + [vp] * 16 + [vp]
        lib.ato_ipm_status.argtypes = [ctypes.c_int32] + [vp] * 11 + [vp]
        lib.ato_ipm_barrier.argtypes = [ctypes.c_int32] + [vp] * 10 + [vp]
        lib.ato_ipm_refine_work.argtypes = [ctypes.c_int32, ctypes.c_int32]
        lib.ato_ipm_refine_pass.argtypes = [ctypes.c_int32, ctypes.c_int32] + [vp] * 7 + [vp]
        lib.ato_ipm_refine_decide.argtypes = [ctypes.c_int32] * 4 + [vp] * 12 + [vp]
        lib.ato_ipm_resto_rows.argtypes = [ctypes.c_int32, ctypes.c_int32] + [vp] * 5 + [vp]
        lib.ato_ipm_js_jty.argtypes = [ctypes.c_int32] * 3 + [vp] * 8 + [vp]
        for fn in IPM_SYMBOLS[1:]:
            getattr(lib, fn).restype = ctypes.c_int
        for fn in ('ato_create', 'ato_destroy', 'ato_sizes', 'ato_sparsity', 'ato_bounds', 'ato_reserve',
                   'ato_eval', 'ato_eval_f32', 'ato_hess_sparsity', 'ato_hess_eval', 'ato_timing',
                   'ato_timing_read', 'ato_timing_stride', 'ato_mesh_create', 'ato_mesh_destroy', 'ato_mesh_signed_distance',
                   'ato_set_instance_spheres', 'ato_sphere_rows', 'ato_gradf_mode', 'ato_gradf_sparsity'):
            getattr(lib, fn).restype = ctypes.c_int
    return lib


_LIB: Optional[ctypes.CDLL] = None


def load(path: Optional[str] = None) -> ctypes.CDLL:
    ''' load libato.so; raises if it is missing (no CPU fallback exists) '''
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or library_path()
    if not os.path.exists(p):
        raise RuntimeError(f'HIP library not built: {p} (run __graft_entry__.build())')
    lib = declare(ctypes.CDLL(p))
    if path is None:
        _LIB = lib
    return lib


def _carr(ctype, values, length):
    arr = (ctype * length)()
    vals = np.asarray(values, dtype=float).reshape(-1)
    for i, v in enumerate(vals[:length]):
        arr[i] = v
    return arr


class DescHolder:
    '''
    Builds an AtoProblemDesc from numpy data and keeps every referenced array alive.
    '''

    def __init__(self, spec: 'dict'):
        self.spec = spec
        d = AtoProblemDesc()
        d.abi_version = ABI_VERSION
        for key in ('model', 'attitude', 'frame', 'global_r', 'transcription', 'N', 'K', 'closed',
                    'cleanly_closed', 'quat_flip', 'force_regularity', 'phase_len'):
            setattr(d, key, int(spec[key]))
        d.euler_wraps = float(spec.get('euler_wraps', 0.0))
        d.gamma = float(spec['gamma'])
        veh = spec['vehicle']
        d.m, d.g = veh['m'], veh['g']
        d.b = _carr(ctypes.c_double, veh['b'], 3)
        d.I = _carr(ctypes.c_double, veh.get('I', [1, 1, 1]), 3)
        d.bw = _carr(ctypes.c_double, veh.get('bw', [0, 0, 0]), 3)
        d.l, d.kt, d.T_max = veh.get('l', 0.0), veh.get('k', 0.0), veh['T_max']
        nu = int(spec['nu'])
        Rm = np.zeros(16)
        dRm = np.zeros(16)
        Rm[:nu * nu] = np.asarray(spec['Rcost'], float).reshape(nu, nu).reshape(-1)
        dRm[:nu * nu] = np.asarray(spec['dRcost'], float).reshape(nu, nu).reshape(-1)
        d.Rcost = _carr(ctypes.c_double, Rm, 16)
        d.dRcost = _carr(ctypes.c_double, dRm, 16)
        K1 = int(spec['K']) + 1
        d.tau = _carr(ctypes.c_double, spec['tau'], KMAX + 1)
        d.Bq = _carr(ctypes.c_double, spec['B'], KMAX + 1)
        Cf = np.zeros((KMAX + 1) * (KMAX + 1))
        Cf[:K1 * K1] = np.asarray(spec['C'], float).reshape(K1, K1).reshape(-1)
        d.C = _carr(ctypes.c_double, Cf, (KMAX + 1) ** 2)
        d.D = _carr(ctypes.c_double, spec['D'], KMAX + 1)
        d.A_skew = _carr(ctypes.c_double, spec.get('A_skew', np.zeros(4)), 4)

        self._keep = []

        def ptr(arr):
            if arr is None:
                return None
            a = np.ascontiguousarray(arr, dtype=np.float64)
            self._keep.append(a)
            return a.ctypes.data_as(_c_double_p)

        d.node_geom = ptr(spec.get('node_geom'))
        d.node_s = ptr(spec.get('node_s'))
        d.interval_s = ptr(spec.get('interval_s'))
        gates = spec.get('gates', [])
        d.n_gates = len(gates)
        garr = (AtoGate * max(len(gates), 1))()
        for i, gspec in enumerate(gates):
            g = garr[i]
            for key in ('interval', 'shape', 'fix_center', 'axial', 'at_end', 'n_coef'):
                setattr(g, key, int(gspec[key]))
            g.coef = _carr(ctypes.c_double, gspec['coef'], KMAX + 1)
            g.gate_x = _carr(ctypes.c_double, gspec['gate_x'], 3)
            g.R = _carr(ctypes.c_double, np.asarray(gspec['R']).reshape(-1), 9)
            g.xc = _carr(ctypes.c_double, gspec['xc'], 3)
            g.ey = _carr(ctypes.c_double, gspec['ey'], 3)
            g.en = _carr(ctypes.c_double, gspec['en'], 3)
            g.d_max = float(gspec['d_max'])
        self._keep.append(garr)
        d.gates = ctypes.cast(garr, ctypes.POINTER(AtoGate))
        spheres = spec.get('spheres')
        d.has_spheres = 1 if spheres is not None else 0
        d.spheres = ptr(spheres)
        wp = spec.get('cpc_waypoints')
        if wp is not None:
            wp = np.asarray(wp, float).reshape(-1, 3)
            if len(wp) > CPC_MAX:
                raise ValueError(f'at most {CPC_MAX} CPC waypoints')
            d.cpc_m = len(wp)
            d.cpc_wp = _carr(ctypes.c_double, wp.reshape(-1), CPC_MAX * 3)
        self.desc = d


class NativeProblem:
    '''
    One ato_handle: problem structure on the current HIP device.
    Evaluation takes raw device pointers (integers), e.g. torch tensor.data_ptr().
    '''

    def __init__(self, spec: dict, lib: Optional[ctypes.CDLL] = None):
        self.lib = lib or load()
        self.holder = DescHolder(spec)
        h = ctypes.c_void_p()
        rc = self.lib.ato_create(ctypes.byref(self.holder.desc), ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(f'ato_create failed ({rc}): {self.lib.ato_last_error().decode()}')
        self.handle = h
        nw, ng, nnz = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        self._check(self.lib.ato_sizes(h, ctypes.byref(nw), ctypes.byref(ng), ctypes.byref(nnz)))
        self.nw, self.ng, self.nnz = nw.value, ng.value, nnz.value

    def _check(self, rc):
        if rc != 0:
            raise RuntimeError(f'libato error {rc}: {self.lib.ato_last_error().decode()}')

    def sparsity(self) -> Tuple[np.ndarray, np.ndarray]:
        ''' CSR (row_ptr[ng+1], col[nnz]) '''
        rp = ctypes.POINTER(ctypes.c_int32)()
        cp = ctypes.POINTER(ctypes.c_int32)()
        self._check(self.lib.ato_sparsity(self.handle, ctypes.byref(rp), ctypes.byref(cp)))
        row_ptr = np.ctypeslib.as_array(rp, shape=(self.ng + 1,)).copy()
        col = np.ctypeslib.as_array(cp, shape=(self.nnz,)).copy()
        return row_ptr, col

    def bounds(self) -> Tuple[np.ndarray, np.ndarray]:
        ''' lbg, ubg '''
        lb = np.zeros(self.ng)
        ub = np.zeros(self.ng)
        self._check(self.lib.ato_bounds(self.handle, lb.ctypes.data_as(_c_double_p),
                                        ub.ctypes.data_as(_c_double_p)))
        return lb, ub

    def gradf_mode(self, sparse: bool):
        ''' sparse: evaluations write only the structural nonzeros of grad f (gradf_sparsity); the
        other entries of the caller's buffer are left as they are (zero-fill it once) '''
        self._check(self.lib.ato_gradf_mode(self.handle, 1 if sparse else 0))

    def gradf_sparsity(self) -> np.ndarray:
        ''' indices of the structural nonzeros of grad f (ascending) '''
        n = ctypes.c_int32()
        self._check(self.lib.ato_gradf_sparsity(self.handle, ctypes.byref(n), None))
        idx = np.zeros(n.value, np.int32)
        self._check(self.lib.ato_gradf_sparsity(self.handle, ctypes.byref(n),
                                                idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return idx

    def gradf_nnz(self) -> int:
        return int(len(self.gradf_sparsity()))

    def set_instance_spheres(self, centres: int, stride: int):
        ''' per-instance sphere centres: device pointer to [P][2][stride] doubles (0 clears) '''
        self._check(self.lib.ato_set_instance_spheres(self.handle, centres or None, int(stride)))

    def sphere_rows(self, P: int) -> np.ndarray:
        ''' row index of every node's sphere row (-1: none) '''
        rows = np.zeros(P, np.int32)
        self._check(self.lib.ato_sphere_rows(self.handle, rows.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return rows

    def reserve(self, max_batch: int):
        ''' allocate scratch for f reductions up to max_batch '''
        self._check(self.lib.ato_reserve(self.handle, int(max_batch)))

    def eval_ptrs(self, batch: int, w: int, g: int = 0, jac: int = 0, f: int = 0, grad_f: int = 0,
                  layout: int = ATO_LAYOUT_INTERLEAVED, stream: int = 0, fp32: bool = False):
        ''' launch the evaluation on device pointers (asynchronous on `stream`) '''
        fn = self.lib.ato_eval_f32 if fp32 else self.lib.ato_eval
        self._check(fn(self.handle, int(batch), int(layout), w or None, g or None, jac or None,
                       f or None, grad_f or None, stream or None))

    def hess_sparsity(self) -> Tuple[np.ndarray, np.ndarray, int]:
        ''' lower-triangle CSR (row_ptr[nw+1], col[nnz_h]) of the Lagrangian Hessian, colour count '''
        nnz, nc = ctypes.c_int32(), ctypes.c_int32()
        rp = ctypes.POINTER(ctypes.c_int32)()
        cp = ctypes.POINTER(ctypes.c_int32)()
        self._check(self.lib.ato_hess_sparsity(self.handle, ctypes.byref(nnz), ctypes.byref(rp), ctypes.byref(cp),
                                               ctypes.byref(nc)))
        row_ptr = np.ctypeslib.as_array(rp, shape=(self.nw + 1,)).copy()
        col = np.ctypeslib.as_array(cp, shape=(nnz.value,)).copy() if nnz.value else np.zeros(0, np.int32)
        return row_ptr, col, nc.value

    def hess_eval_ptrs(self, batch: int, w: int, lam: int, sigma: int, hess: int,
                       layout: int = ATO_LAYOUT_INTERLEAVED, stream: int = 0):
        ''' Hessian of the Lagrangian on device pointers (fp64, asynchronous on `stream`) '''
        self._check(self.lib.ato_hess_eval(self.handle, int(batch), int(layout), w, lam, sigma, hess,
                                           stream or None))

    def timing_start(self, max_calls: int):
        ''' record HIP events around the kernels of the next max_calls evaluations '''
        self._check(self.lib.ato_timing(self.handle, int(max_calls)))

    def timing_stride(self, stride: int):
        ''' events on every stride-th evaluation only (ato_timing_stride) '''
        self._check(self.lib.ato_timing_stride(self.handle, int(stride)))

    def timing_read(self):
        ''' (sum of Jacobian-kernel ms, sum of cost-reduce ms, calls) since timing_start '''
        a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_int32()
        self._check(self.lib.ato_timing_read(self.handle, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    def close(self):
        ''' release the handle '''
        if getattr(self, 'handle', None):
            self.lib.ato_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pylint: disable=broad-except
            pass
