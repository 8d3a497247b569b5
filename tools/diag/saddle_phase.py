'''
DIAGNOSTIC (GPU): shader-clock split of k_front_saddle (csrc/ato_kkt.hip) on the racetrack 50 x 4
KKT with saddle fronts, recorded by the workgroup of front ATO_KKT_STAMP_FRONT (50: the first saddle
front) of instance 0 in a stamps build, plus the number of (front, instance) pairs sent to the
Bunch-Kaufman fallback (all factorisations of the run). ATO_PHASE_B sets the batch (default 512).

    python tools/diag/kkt_variants.py stamps -DATO_KKT_STAMPS -DATO_KKT_STAMP_FRONT=50     (CPU)
    ATO_LIB_PATH=tools/diag/_lib/libato_stamps.so python tools/diag/saddle_phase.py        (GPU)
'''
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    from aircraft_trajectory_optimization_amd import native
    from aircraft_trajectory_optimization_amd.raceline.batched import BatchedNLP
    from aircraft_trajectory_optimization_amd.raceline.evaluator import variable_stages
    from aircraft_trajectory_optimization_amd.raceline.instances import seeded_instances
    from aircraft_trajectory_optimization_amd.solver.kkt_device import DeviceKKT
    from aircraft_trajectory_optimization_amd.solver.kkt_plan import build_plan, collocation_saddle
    from aircraft_trajectory_optimization_amd.tracks import make_spec
    spec = make_spec(track='race', frame='parametric', N=50, K=4)
    B = int(os.environ.get('ATO_PHASE_B', '512'))
    bn = BatchedNLP(spec, B)
    W, _, _ = seeded_instances(spec, np.arange(B))
    bn.set_w(W)
    bn.evaluate()
    hrp, hcol, _ = bn.problem.hess_sparsity()
    sad = collocation_saddle(spec.N, spec.K1, spec.nv, spec.nz, bn.sizes[1], bn.row_ptr, bn.col)
    plan = build_plan(bn.sizes[0], bn.sizes[1], variable_stages(spec), bn.row_ptr, bn.col, hrp, hcol, saddle=sad)
    g = torch.Generator(device='cuda').manual_seed(0)
    lam = torch.randn((bn.sizes[1], B), dtype=torch.float64, device='cuda', generator=g)
    H = bn.hessian(lam, torch.ones(B, dtype=torch.float64, device='cuda'))
    dx = torch.rand((plan.n, B), dtype=torch.float64, device='cuda', generator=g) + 0.1
    dr = -(torch.rand((plan.m, B), dtype=torch.float64, device='cuda', generator=g) * 1e-2 + 1e-6)
    dr[torch.as_tensor(np.asarray(bn.lbg) == np.asarray(bn.ubg), device='cuda')] = 0.0
    kkt = DeviceKKT(plan, B)
    reps = 3
    for _ in range(reps):
        kkt.factor(H, bn.jac, dx, dr)
    torch.cuda.synchronize()
    lib = native.load()
    lib.ato_kkt_diag_stamps.argtypes = [ctypes.c_void_p]
    out = (ctypes.c_ulonglong * 16)()
    assert lib.ato_kkt_diag_stamps(out) == 0
    v = list(out)
    names = ['assembly', 'Gauss-Jordan', 'unscramble', 'HE, G', 'W', 'S', 'stores']
    res = {n: int(v[i]) for i, n in enumerate(names)}
    res['total_cycles'] = int(sum(v[:10]))
    res['gauss_jordan_split'] = {'owner search (wave 0: every 8th step)': int(v[7]), 'barrier + pivot read': int(v[8]),
                                 'update': int(v[9])}
    res['fallback_pairs_per_factorisation'] = v[14] / reps
    res['saddle_pairs_per_factorisation'] = int((plan.n_sad > 0).sum()) * B
    print(json.dumps(res))


if __name__ == '__main__':
    main()
