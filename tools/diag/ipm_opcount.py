'''
DIAGNOSTIC (CPU): torch operator count of the batched interior-point solver per lap section
(solver/batched_ipm.py, ATO_IPM_PROFILE laps), on the CPU stand-ins of the tests. Every
operator is one kernel launch on the device, so this is the launch budget of a lockstep
iteration.

    python tools/diag/ipm_opcount.py
'''
import collections
import os
import sys

os.environ['ATO_IPM_PROFILE'] = '1'
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

from aircraft_trajectory_optimization_amd.solver import batched_ipm  # noqa: E402
from aircraft_trajectory_optimization_amd.solver.ipm import IPMOptions  # noqa: E402
from tests.batched_backends import HostBatchEvaluator, HostBlockKKT  # noqa: E402
from tests.helpers import product_spec  # noqa: E402

COUNT = collections.Counter()
OPS = collections.defaultdict(collections.Counter)
STATE = {'n': 0}
PENDING = collections.Counter()


class Count(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        STATE['n'] += 1
        PENDING[str(func)] += 1
        return func(*args, **(kwargs or {}))


_lap = batched_ipm._Laps.lap


def lap(self, name=None):
    if name is not None:
        COUNT[name] += STATE['n']
        OPS[name].update(PENDING)
    STATE['n'] = 0
    PENDING.clear()
    _lap(self, name)


batched_ipm._Laps.lap = lap

spec = product_spec(track='race', model='point', use_quat=False, N=8, K=3)
B = 3
rng = np.random.default_rng(0)
W = np.repeat(spec.w0[None], B, axis=0)
for b in range(1, B):
    W[b, :spec.N] *= 1 + 0.1 * rng.uniform(-1, 1, spec.N)
if '--device' in sys.argv:             # the device solver (fused kernels, ctypes calls not counted)
    solver = batched_ipm.device_solver(spec, B, spec.lbw, spec.ubw, IPMOptions(max_iter=200))
else:
    ev = HostBatchEvaluator(spec, B)
    solver = batched_ipm.BatchedInteriorPoint(ev, HostBlockKKT(ev), spec.lbw, spec.ubw, IPMOptions(max_iter=200))
with Count():
    res = solver.solve(W)
it = int(max(res.iters))
tot = sum(COUNT.values())
print(f'lockstep iterations ~{it}, operators {tot} ({tot / max(it, 1):.0f} per iteration)')
for k, v in COUNT.most_common():
    print(f'  {k:16s} {v:7d}  {v / max(it, 1):7.1f} / it')
if '-v' in sys.argv:
    for sec in ('direction', 'check', 'kkt_other', 'ls_logic', 'barrier', 'kkt_refine', 'rhs', 'accept'):
        print(sec, OPS[sec].most_common(12))
