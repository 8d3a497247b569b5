'''
DIAGNOSTIC ONLY: time the factor kernel built with experiment switches (-DATO_KKT_EXP_NOUPD: no
Schur update; -DATO_KKT_EXP_NOSTORE: no factor-column stores). Results are wrong by design; the
times say which part of a pivot step costs what.
    python tools/diag/kkt_exp.py --build-only  |  python tools/diag/kkt_exp.py
'''
import ctypes
import glob
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
EXPS = {'base': [], 'noupd': ['-DATO_KKT_EXP_NOUPD'], 'nostore': ['-DATO_KKT_EXP_NOSTORE'],
        'none': ['-DATO_KKT_EXP_NOUPD', '-DATO_KKT_EXP_NOSTORE']}


def build():
    from aircraft_trajectory_optimization_amd import build_native
    build_native.build(verbose=False)
    objs = [o for o in sorted(glob.glob(os.path.join(build_native.OBJ, '*.o'))) if not o.endswith('ato_kkt.o')]
    src = os.path.join(build_native.CSRC, 'ato_kkt.hip')
    for name, flags in EXPS.items():
        obj = os.path.join(HERE, f'kkt_{name}.o')
        subprocess.check_call(['hipcc', *build_native.FLAGS, *flags, '-c', src, '-o', obj])
        subprocess.check_call(['hipcc', '-shared', '-fPIC', f'--offload-arch={build_native.ARCH}', '-o',
                               os.path.join(HERE, f'libkkt_{name}.so'), *objs, obj])


def main():
    if '--build-only' in sys.argv:
        build()
        return
    import torch
    from aircraft_trajectory_optimization_amd import native
    from aircraft_trajectory_optimization_amd.raceline.batched import BatchedNLP
    from aircraft_trajectory_optimization_amd.raceline.evaluator import variable_stages
    from aircraft_trajectory_optimization_amd.raceline.instances import seeded_instances
    from aircraft_trajectory_optimization_amd.solver.kkt_plan import build_plan
    from aircraft_trajectory_optimization_amd.tracks import make_spec
    B = 64
    spec = make_spec(track='race', N=50, K=4)
    bn = BatchedNLP(spec, B)
    bn.set_w(seeded_instances(spec, np.arange(B))[0])
    bn.evaluate()
    hrp, hcol, _ = bn.problem.hess_sparsity()
    plan = build_plan(bn.sizes[0], bn.sizes[1], variable_stages(spec), bn.row_ptr, bn.col, hrp, hcol)
    g = torch.Generator(device='cuda').manual_seed(0)
    H = bn.hessian(torch.randn((bn.sizes[1], B), dtype=torch.float64, device='cuda', generator=g),
                   torch.ones(B, dtype=torch.float64, device='cuda'))
    dx = torch.rand((plan.n, B), dtype=torch.float64, device='cuda', generator=g) + 0.1
    dr = -(torch.rand((plan.m, B), dtype=torch.float64, device='cuda', generator=g) * 1e-2 + 1e-6)
    from aircraft_trajectory_optimization_amd.solver import kkt_device
    for name in EXPS:
        lib = native.declare(ctypes.CDLL(os.path.join(HERE, f'libkkt_{name}.so')))
        native._LIB = lib
        kkt = kkt_device.DeviceKKT(plan, B)
        kkt.factor(H, bn.jac, dx, dr)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            kkt.factor(H, bn.jac, dx, dr)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 3
        print(f'{name:8s} factor {ms:7.2f} ms  {ms * 1e3 / plan.dim:5.2f} us per pivot step', flush=True)
        kkt.close()


if __name__ == '__main__':
    main()
