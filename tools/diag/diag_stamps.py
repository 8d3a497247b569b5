'''
DIAGNOSTIC ONLY: build tools/diag/libato_diag.so (library objects + diag_stamps.hip) and
report where ODE-unit waves spend their time (s_memtime stamps, shader clock cycles).

    python tools/diag/diag_stamps.py [--build-only]
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
LIB = os.path.join(HERE, 'libato_diag.so')


def build():
    from aircraft_trajectory_optimization_amd import build_native
    build_native.build(verbose=False)
    objs = sorted(glob.glob(os.path.join(build_native.OBJ, '*.o')))
    src = os.path.join(HERE, 'diag_stamps.hip')
    obj = os.path.join(HERE, 'diag_stamps.o')
    subprocess.check_call(['hipcc', *build_native.FLAGS, '-c', src, '-o', obj])
    subprocess.check_call(['hipcc', '-shared', '-fPIC', f'--offload-arch={build_native.ARCH}', '-o', LIB,
                           *objs, obj])


def main():
    if '--build-only' in sys.argv:
        build()
        return
    import torch
    from aircraft_trajectory_optimization_amd import native
    from aircraft_trajectory_optimization_amd.raceline.batched import BatchedNLP
    from aircraft_trajectory_optimization_amd.raceline.instances import seeded_instances
    from aircraft_trajectory_optimization_amd.tracks import make_spec
    lib = native.declare(ctypes.CDLL(LIB))
    lib.atodiag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 5
    spec = make_spec()
    B = 512
    W, _, _ = seeded_instances(spec, range(B))
    prob = native.NativeProblem(spec.native_spec(), lib=lib)
    bn = BatchedNLP.__new__(BatchedNLP)
    w = torch.as_tensor(W.T.copy(), device='cuda')
    g = torch.zeros((prob.ng, B), device='cuda', dtype=torch.float64)
    J = torch.zeros((prob.nnz, B), device='cuda', dtype=torch.float64)
    n_units = len(prob.holder.spec) and None
    for kind, name in ((1, 'ODE_A'), (2, 'ODE_B')):
        st = torch.zeros((4096 * 8, 4), device='cuda', dtype=torch.int64)
        for _ in range(3):
            rc = lib.atodiag_stamps(prob.handle, B, kind, w.data_ptr(), g.data_ptr(), J.data_ptr(), st.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream)
            assert rc == 0
        torch.cuda.synchronize()
        s = st.cpu().numpy().astype(np.int64)
        s = s[s[:, 3] > 0]
        t0 = s[:, 0].min()
        load = s[:, 1] - s[:, 0]
        comp = s[:, 2] - s[:, 1]
        drain = s[:, 3] - s[:, 2]
        start = s[:, 0] - t0
        end = s[:, 3] - t0
        pct = lambda a: f'median {np.median(a):8.0f}  p90 {np.percentile(a, 90):8.0f}  max {a.max():8.0f}'  # noqa
        print(f'{name}: {len(s)} waves (cycles)')
        print('  loads      ', pct(load))
        print('  model+store', pct(comp))
        print('  drain      ', pct(drain))
        print('  start      ', pct(start))
        print('  end        ', pct(end))


if __name__ == '__main__':
    main()
