'''
DIAGNOSTIC ONLY: run the device evaluation, Hessian, KKT factorisation and KKT solve several
times on identical inputs and report whether the outputs are bitwise identical.

    python tools/diag/det_kernels.py [--N 5 --K 2 --batch 2]   (GPU)
'''
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--N', type=int, default=5)
    ap.add_argument('--K', type=int, default=2)
    ap.add_argument('--batch', type=int, default=2)
    ap.add_argument('--reps', type=int, default=5)
    a = ap.parse_args()
    from aircraft_trajectory_optimization_amd.raceline.batched import BatchedNLP
    from aircraft_trajectory_optimization_amd.raceline.evaluator import variable_stages
    from aircraft_trajectory_optimization_amd.raceline.instances import seeded_instances
    from aircraft_trajectory_optimization_amd.solver.kkt_device import DeviceKKT
    from aircraft_trajectory_optimization_amd.solver.kkt_plan import build_plan
    from aircraft_trajectory_optimization_amd.tracks import make_spec
    spec = make_spec(track='race', N=a.N, K=a.K)
    B = a.batch
    bn = BatchedNLP(spec, B)
    W, _, _ = seeded_instances(spec, np.arange(B))
    hrp, hcol, _ = bn.problem.hess_sparsity()
    plan = build_plan(bn.sizes[0], bn.sizes[1], variable_stages(spec), bn.row_ptr, bn.col, hrp, hcol)
    kkt = DeviceKKT(plan, B)
    g = torch.Generator(device='cuda').manual_seed(0)
    lam = torch.randn((bn.sizes[1], B), dtype=torch.float64, device='cuda', generator=g)
    sig = torch.ones(B, dtype=torch.float64, device='cuda')
    dx = torch.rand((plan.n, B), dtype=torch.float64, device='cuda', generator=g) + 0.1
    dr = -(torch.rand((plan.m, B), dtype=torch.float64, device='cuda', generator=g) * 1e-2 + 1e-6)
    rhs = torch.randn((plan.dim, B), dtype=torch.float64, device='cuda', generator=g)
    outs = []
    for _ in range(a.reps):
        bn.set_w(W)
        bn.evaluate()
        H = bn.hessian(lam, sig).clone()
        J = bn.jac.clone()
        gv = bn.g.clone() if hasattr(bn, 'g') else None
        kkt.factor(H, J, dx, dr)
        x = rhs.clone()
        kkt.solve(x)
        torch.cuda.synchronize()
        outs.append((J, H, x, kkt.inertia.clone(), gv))
    names = ['jac', 'hess', 'kkt_x', 'inertia', 'g']
    for i, nm in enumerate(names):
        if outs[0][i] is None:
            continue
        same = all(torch.equal(outs[0][i], o[i]) for o in outs[1:])
        dmax = max(float((outs[0][i].double() - o[i].double()).abs().max()) for o in outs[1:])
        print(f'{nm:8s} bitwise identical over {a.reps} runs: {same}  max diff {dmax:.3e}', flush=True)


if __name__ == '__main__':
    main()
