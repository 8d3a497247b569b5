'''
DIAGNOSTIC: where the bench step's time goes besides the evaluation kernel. Times K evaluations
of the bench workload (racetrack 50x4x13, B = 512) (a) with the library's per-call timing events,
(b) without them, (c) the host-side cost of one evaluate() call (no synchronisation).
'''
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from aircraft_trajectory_optimization_amd.raceline.batched import BatchedNLP  # noqa: E402
from aircraft_trajectory_optimization_amd.raceline.instances import seeded_instances  # noqa: E402
from aircraft_trajectory_optimization_amd.tracks import make_spec  # noqa: E402

K = 200
spec = make_spec(track='race', model='drone', frame='parametric', N=50, K=4, use_quat=True, global_r=True)
B = 512
W, _, _ = seeded_instances(spec, list(range(B)))
bn = BatchedNLP(spec, B)
bn.set_w(W)
for _ in range(20):
    bn.evaluate()
torch.cuda.synchronize()
for events in (True, False, True, False):
    if events:
        bn.problem.timing_start(K)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        bn.evaluate()
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t1 = time.perf_counter() - t0
    msg = ''
    if events:
        k_ms, r_ms, calls = bn.problem.timing_read()
        bn.problem.timing_start(0)
        msg = f' kernel {k_ms / calls * 1e3:.1f} us reduce {r_ms / calls * 1e3:.1f} us'
    print(f'events={events}: step {t1 / K * 1e6:.1f} us, host issue {t_host / K * 1e6:.1f} us/call{msg}', flush=True)
# graph capture of one evaluation
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    bn.evaluate()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
try:
    with torch.cuda.graph(g):
        bn.evaluate()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        g.replay()
    torch.cuda.synchronize()
    print(f'graph replay: step {(time.perf_counter() - t0) / K * 1e6:.1f} us', flush=True)
except Exception as e:  # noqa: BLE001
    print('graph capture failed:', e)
