'''
DIAGNOSTIC (GPU): shader-clock split of the pivot steps of the KKT factorisation, recorded by
the workgroup of front ATO_KKT_STAMP_FRONT (default 0; the first interval leaf is front 50 since the
pre-front split) of instance 0 in a stamps build (tools/diag/kkt_variants.py stamps -DATO_KKT_STAMPS
-DATO_KKT_STAMP_FRONT=50); ATO_PHASE_B sets the batch (default 1).

    ATO_LIB_PATH=tools/diag/_lib/libato_stamps.so python tools/diag/kkt_phase.py
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
    from aircraft_trajectory_optimization_amd.solver.kkt_plan import build_plan
    from aircraft_trajectory_optimization_amd.tracks import make_spec
    spec = make_spec(track='race', frame='parametric', N=50, K=4)
    B = int(os.environ.get('ATO_PHASE_B', '1'))
    bn = BatchedNLP(spec, B)
    W, _, _ = seeded_instances(spec, np.arange(B))
    bn.set_w(W)
    bn.evaluate()
    hrp, hcol, _ = bn.problem.hess_sparsity()
    plan = build_plan(bn.sizes[0], bn.sizes[1], variable_stages(spec), bn.row_ptr, bn.col, hrp, hcol)
    g = torch.Generator(device='cuda').manual_seed(0)
    lam = torch.randn((bn.sizes[1], B), dtype=torch.float64, device='cuda', generator=g)
    H = bn.hessian(lam, torch.ones(B, dtype=torch.float64, device='cuda'))
    dx = torch.rand((plan.n, B), dtype=torch.float64, device='cuda', generator=g) + 0.1
    dr = -(torch.rand((plan.m, B), dtype=torch.float64, device='cuda', generator=g) * 1e-2 + 1e-6)
    kkt = DeviceKKT(plan, B)
    for _ in range(3):
        kkt.factor(H, bn.jac, dx, dr)
    torch.cuda.synchronize()
    lib = native.load()
    lib.ato_kkt_diag_stamps.argtypes = [ctypes.c_void_p]
    out = (ctypes.c_ulonglong * 16)()
    assert lib.ato_kkt_diag_stamps(out) == 0
    v = list(out)
    steps = max(int(v[15]), 1)
    names = {0: 'assembly', 1: 'extract+barrier', 5: 'column read+keys+DPP max', 2: 'pivot picks+decision',
             6: 'inverse+inertia', 7: 'live bookkeeping', 8: 'record+row factors', 3: 'factor-column store',
             4: 'update'}
    res = {n: v[i] for i, n in names.items()}
    res['steps'] = steps
    res['per_step_cycles'] = {n: v[i] / steps for i, n in names.items() if i != 0}
    print(json.dumps(res))


if __name__ == '__main__':
    main()
