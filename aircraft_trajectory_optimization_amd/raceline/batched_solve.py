'''
Sharded batched solve (north star): every rank (one process per GPU) solves its
own contiguous block of seeded problem instances with the device interior-point solver -- no
communication while solving -- and the per-instance results are then all-gathered over RCCL
(xGMI) as fixed 32-byte records:

    [lap time (f64), final KKT error E0 (f64, IPOPT's scaled optimality error), iterations, status]

(the last two stored as f64 so the record is one [B, 4] float64 tensor, 32 bytes per instance;
8192 instances = 256 KB, latency-bound). Instances are independent, so the sharded result equals
the single-process result over all seeds instance for instance (the gloo test checks this on CPU
stand-ins). The reference solves one problem at a time (base_raceline.py:157-191) and has no
parallelism of any kind: this layer is build-side.
'''
from typing import Callable, Dict, Optional, Sequence, Tuple

import numpy as np
import torch

from aircraft_trajectory_optimization_amd.raceline.instances import seeded_instances
from aircraft_trajectory_optimization_amd.raceline.problem import ProblemSpec
from aircraft_trajectory_optimization_amd.raceline.shard import gather_direct, gather_records, max_over_ranks

RECORD_FIELDS = ('lap_time', 'kkt_error', 'iterations', 'status')
RECORD_BYTES = 8 * len(RECORD_FIELDS)


def solve_shard(spec: ProblemSpec, seeds: Sequence[int], options, on_iteration: Optional[Callable] = None,
                solver_factory=None, progress: int = 0):
    ''' solve the seeded cold-start instances `seeds` (SURVEY 8(d) config 3 generator) as one batch:
    (result, solver, W) '''
    from aircraft_trajectory_optimization_amd.solver.batched_ipm import device_solver
    W, LBW, UBW = seeded_instances(spec, seeds)
    factory = solver_factory or device_solver
    solver = factory(spec, len(W), LBW, UBW, options)
    res = solver.solve(W, progress=progress, on_iteration=on_iteration)
    return res, solver, W


def solve_records(spec: ProblemSpec, res, solver) -> torch.Tensor:
    ''' [B, 4] float64 records of a finished batched solve (on the solve's device) '''
    from aircraft_trajectory_optimization_amd.solver.batched_ipm import STATUS_NAMES
    code = {v: k for k, v in STATUS_NAMES.items()}
    x = res.x
    lap = x[:spec.N].sum(0)
    fe0 = getattr(solver, 'final_e0', None)
    hist = getattr(solver, 'history', None)
    if fe0 is not None:
        e0 = torch.as_tensor(np.asarray(fe0, np.float64), device=x.device)
    elif hist is not None and len(hist):
        e0 = torch.as_tensor(hist[-1][4], dtype=torch.float64, device=x.device)
    else:
        e0 = torch.full_like(lap, float('nan'))
    iters = torch.as_tensor(np.asarray(res.iters, np.float64), device=x.device)
    status = torch.as_tensor([float(code[s]) for s in res.status], dtype=torch.float64, device=x.device)
    return torch.stack([lap, e0, iters, status], dim=1).contiguous()


def gather_solve_records(records: torch.Tensor) -> torch.Tensor:
    ''' all ranks' records, rank-major (row i = seed i) '''
    if records.dtype != torch.float64 or records.dim() != 2 or records.shape[1] != len(RECORD_FIELDS):
        raise ValueError('solve records are [B, 4] float64')
    return gather_records(records)


def summarize_records(rec) -> Dict:
    ''' converged counts, statuses and lap-time statistics of gathered records '''
    from aircraft_trajectory_optimization_amd.solver.batched_ipm import STATUS_NAMES
    rec = rec.cpu().numpy() if torch.is_tensor(rec) else np.asarray(rec)
    status = rec[:, 3].astype(int)
    names = [STATUS_NAMES[s] for s in status]
    ok = np.isin(names, ['optimal', 'acceptable'])
    lap = rec[:, 0]
    out = {'instances': int(len(rec)), 'converged': int(ok.sum()),
           'statuses': {s: names.count(s) for s in sorted(set(names))},
           'instance_iterations': int(rec[:, 2].sum()),
           'iterations': {'min': int(rec[:, 2].min()), 'median': float(np.median(rec[:, 2])),
                          'max': int(rec[:, 2].max())},
           'kkt_error_converged_max': float(rec[ok, 1].max()) if ok.any() else None}
    if ok.any():
        out['lap_time_converged'] = {'min': float(lap[ok].min()), 'median': float(np.median(lap[ok])),
                                     'max': float(lap[ok].max())}
    return out


def window_timer(warmup: int, steps: int, sync: Callable[[], None]) -> Tuple[Callable, Dict]:
    '''
    on_iteration hook that times lockstep iterations [warmup, warmup + steps) of a solve: the
    device is synchronised at both ends. Instance-iterations in the window ('count') are those of
    the solve's StepCounter between the two ends: the instances that took a step in each of the
    window's lockstep iterations ('count_main') plus the iterations of the restoration phases that ran
    meanwhile ('count_resto'; IPOPT's iteration counter runs through the restoration phase, and so do
    max_iter and sqp_full's instance_iterations)
    '''
    import time
    st: Dict = {'t0': None, 't1': None, 'count': 0, 'count_main': 0, 'count_resto': 0, 'timed': 0}
    base = {}

    def hook(it, n_step, counter=None):
        if n_step >= 0 and it == warmup and st['t0'] is None:
            sync()
            st['t0'] = time.perf_counter()
            if counter is not None:       # this iteration's own steps are already in the counter
                base['v'], base['r'] = counter.value - n_step, counter.resto
        if st['t0'] is not None and st['t1'] is None:
            if n_step < 0 or it == warmup + steps:
                sync()
                st['t1'] = time.perf_counter()
                if counter is not None:
                    end = counter.value - max(n_step, 0)
                    st['count'] = end - base['v']
                    st['count_resto'] = counter.resto - base['r']
                else:
                    st['count'] = st['count_main']
            else:
                st['count_main'] += n_step
                st['timed'] += 1
    return hook, st


def time_solution_gathers(xs: torch.Tensor, sync: Callable[[], None], device=None) -> Dict:
    '''
    The audit gather of the converged decision vectors xs [B_local, nw], timed both
    ways (max over ranks): the direct point-to-point all-gather and the collective all_gather.
    Every rank must call it. Returns bytes and milliseconds, and whether both gave the same result.
    '''
    import time
    import torch.distributed as dist
    out = {'bytes_per_rank': int(xs.numel() * xs.element_size())}
    results = []
    for name, fn in (('direct_p2p', gather_direct), ('all_gather', gather_records)):
        sync()
        if dist.is_available() and dist.is_initialized():
            dist.barrier()
        t0 = time.perf_counter()
        r = fn(xs)
        sync()
        out[f'{name}_ms'] = max_over_ranks(time.perf_counter() - t0, device) * 1e3
        results.append(r)
    out['bytes_total'] = int(results[0].numel() * results[0].element_size())
    out['identical'] = bool(torch.equal(results[0], results[1]))
    return out
