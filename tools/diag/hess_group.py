'''
DIAGNOSTIC (GPU): time of one device Hessian (ato_hess_eval) at several batch widths, the racetrack 50 x 4
drone at seeded cold starts; ATO_HESS_GROUP_BYTES sets how many colours share a launch (1: one colour per
launch, the round-5 schedule). Prints one JSON line.
    ATO_HESS_GROUP_BYTES=1 python tools/diag/hess_group.py
'''
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from aircraft_trajectory_optimization_amd.raceline.instances import seeded_instances  # noqa: E402
from aircraft_trajectory_optimization_amd.solver.batched_ipm import BatchedDeviceEvaluator  # noqa: E402
from aircraft_trajectory_optimization_amd.tracks import make_spec  # noqa: E402

spec = make_spec(track='race', N=50, K=4)
out = {'group_bytes': os.environ.get('ATO_HESS_GROUP_BYTES', 'default')}
rng = np.random.default_rng(0)
for B in (32, 64, 128, 512):
    W, _, _ = seeded_instances(spec, range(B))
    X = torch.as_tensor(np.ascontiguousarray(W.T), device='cuda')
    ev = BatchedDeviceEvaluator(spec, B)
    f, g, gf, jv = ev.eval(X)
    lam = torch.as_tensor(rng.standard_normal((g.shape[0], B)), device='cuda')
    sig = torch.ones(B, dtype=torch.float64, device='cuda')
    H = ev.hess(X, lam, sig)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        H2 = ev.hess(X, lam, sig)
    e1.record()
    torch.cuda.synchronize()
    out[f'B{B}_ms'] = e0.elapsed_time(e1) / 20
    out[f'B{B}_checksum'] = float(H2.abs().sum())
    assert torch.equal(H, H2)
print(json.dumps(out), flush=True)
