#!/usr/bin/env python
'''
Benchmark of the hot path: batched evaluation of the collocation NLP's g(w), dg/dw (all
structural entries), f(w) and grad f(w) -- what IPOPT asks CasADi for on every iterate of
the reference (base_raceline.py:165, :182-189).

Workload (BASELINE.json configs[2]): racetrack of scripts/race.py, parametric frame,
quaternion drone (13 states, 4 inputs), global attitude, square gates, closed loop,
N = 50 intervals, K = 4 Legendre collocation, fp64, B = 512 seeded instances per GPU
(SURVEY 8(d) config 3 generator). One step = one ato_eval over the whole batch, inputs
resident in HBM. Multi-GPU: one process per GPU, instances sharded (weak scaling), no
collective inside the timed region; per-instance summaries are all-gathered over RCCL
afterwards.

    python bench.py [--gpus N --steps K --warmup W --batch B]
'''
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = 'SQP iters/sec (batched) + lap-time err vs CasADi, 50×4 collocation'
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
TIMING_STRIDE = 10         # kernel-timing events on every 10th timed step


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--batch', type=int, default=512, help='instances per GPU')
    ap.add_argument('--dtype', choices=['f64', 'f32'], default='f64')
    ap.add_argument('--layout', choices=['interleaved', 'instance'], default='interleaved')
    ap.add_argument('--cpu-seconds', type=float, default=15.0, help='budget of the oracle CPU baseline')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-solve', action='store_true', help='skip the interior-point solves (batched and single)')
    ap.add_argument('--solve-batch', type=int, default=512, help='instances of the batched interior-point solve')
    ap.add_argument('--solve-max-iter', type=int, default=200)
    ap.add_argument('--traffic-json', default=os.path.join(ROOT, 'profiles', 'traffic_latest.json'))
    return ap.parse_args()


def cpu_baseline(spec_kwargs, W, budget_s):
    '''
    SURVEY 8(d): the build's C++ CPU twin of ato_eval -- the same segment programs compiled with
    g++ -O3 (tests/native/hostcheck.cpp, OpenMP over instances) -- timed on the host cores of the
    same box on the same instances: one thread and all threads of this process' share
    (OMP_NUM_THREADS). The numpy restatement (oracle, complex-step Jacobian) is reported beside it.
    The reference's CasADi/IPOPT path cannot run anywhere in this pipeline.
    '''
    from tests.helpers import HostCheck, oracle_nlp
    from aircraft_trajectory_optimization_amd.tracks import make_spec
    hc = HostCheck(make_spec(**spec_kwargs).native_spec())
    threads = max(1, int(os.environ.get('OMP_NUM_THREADS', os.cpu_count() or 1)))

    def rate(nthreads, budget):
        out = None
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget:
            out = hc.eval_threads(W, nthreads, out)
            n += W.shape[0]
        return n / (time.perf_counter() - t0), n

    r1, n1 = rate(1, budget_s / 3)
    rT, nT = rate(threads, budget_s / 3)
    nlp = oracle_nlp(**spec_kwargs)
    t0, k = time.perf_counter(), 0
    while k < 3:
        w = W[k]
        nlp.g(w)
        nlp.jac_dense(w)
        nlp.f(w)
        nlp.grad_f(w)
        k += 1
    r_np = k / (time.perf_counter() - t0)
    return {'value': rT, 'unit': 'evals/s', 'cores': threads, 'kind': 'port',
            'single_thread_value': r1, 'numpy_oracle_value': r_np,
            'sample': f'C++ twin of ato_eval (g++ -O3 -march=x86-64-v3, OpenMP): {nT} evaluations on '
                      f'{threads} threads and {n1} on 1 thread of the same {W.shape[0]} seeded 50x4x13 '
                      f'racetrack instances (g, dg/dw, f, grad f), about {budget_s / 3:.0f} s each; numpy oracle '
                      f'(complex-step dense J) {k} instances'}


def batched_solve(B, max_iter):
    '''
    The SQP (interior-point) iteration itself, batched: BASELINE config 3 shape (racetrack 50 x 4
    drone, B instances on one GPU, fp64). Instance 0 is race.py's use_ws start (point-mass warm
    start); the others are seeded perturbations of it (raceline/batch_instances.py). Every
    evaluation, Hessian, KKT factorisation (ato_kkt_factor) and solve runs on the device; the
    lockstep iteration logic is torch on the device. Instance 0 is also solved by the
    single-instance host-KKT solver: lap_time_err_instance0_vs_host_s compares the two (the
    CasADi/IPOPT lap time itself is unpinned: IPOPT is not reachable here).
    '''
    from tools.solve_batched import run
    out = run(B, max_iter, host_ref=True)
    out['lap_time_vs_casadi'] = 'unpinned (no IPOPT reachable here); vs the single-instance solver: see ' \
                                'lap_time_err_instance0_vs_host_s'
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from aircraft_trajectory_optimization_amd import native
    from aircraft_trajectory_optimization_amd.raceline.batched import BatchedNLP
    from aircraft_trajectory_optimization_amd.raceline.instances import seeded_instances
    from aircraft_trajectory_optimization_amd.raceline.shard import gather_records, max_over_ranks, shard_seeds
    from aircraft_trajectory_optimization_amd.tracks import make_spec

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        dist.init_process_group('nccl')
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)

    spec_kwargs = dict(track='race', model='drone', frame='parametric', N=50, K=4, use_quat=True, global_r=True)
    spec = make_spec(**spec_kwargs)
    B = args.batch
    W, _, _ = seeded_instances(spec, shard_seeds(rank, world, B))
    dtype = torch.float64 if args.dtype == 'f64' else torch.float32
    layout = native.ATO_LAYOUT_INTERLEAVED if args.layout == 'interleaved' else native.ATO_LAYOUT_INSTANCE_MAJOR
    bn = BatchedNLP(spec, B, dtype=dtype, layout=layout, device=dev)
    bn.set_w(W)
    nw, ng, nnz = bn.sizes

    for _ in range(args.warmup):
        bn.evaluate()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    # kernel durations from HIP events on the evaluation stream, recorded on every TIMING_STRIDE-th
    # step of the timed loop: each recorded step adds three event packets (about 10 us of gaps at
    # B = 512, tools/diag/step_gaps.py), which would otherwise be part of every measured step
    bn.problem.timing_stride(TIMING_STRIDE)
    bn.problem.timing_start((args.steps + TIMING_STRIDE - 1) // TIMING_STRIDE)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        bn.evaluate()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(t1 - t0, dev)
    k_ms, r_ms, calls = bn.problem.timing_read()
    bn.problem.timing_start(0)
    bn.problem.timing_stride(1)

    # per-instance summary {lap-time guess sum(h), cost f, max equality residual}, all-gathered (RCCL)
    g, _, f, _ = bn.results()
    eq = bn.lbg == bn.ubg
    summary = np.stack([W[:, :spec.N].sum(axis=1), f, np.abs(g[:, eq]).max(axis=1)], axis=1)
    gathered = gather_records(torch.as_tensor(summary, device=dev))
    assert bool(torch.isfinite(gathered).all()), 'non-finite evaluation results'

    if rank == 0:
        elem = 8 if args.dtype == 'f64' else 4
        bytes_per_eval = elem * (nw + ng + nnz + nw + 1)   # read w; write g, J, grad f, f
        kernel_s = (k_ms / max(calls, 1)) / 1e3
        achieved = B * bytes_per_eval / kernel_s / 1e9
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                tj = json.load(open(args.traffic_json, encoding='utf-8'))
                if tj.get('batch') == B and tj.get('dtype') == args.dtype and tj.get('layout') == args.layout:
                    traffic = tj.get('hbm_bytes_per_launch')
            except (OSError, ValueError):
                traffic = None
        value = world * B * args.steps / elapsed
        out = {
            'metric': METRIC,
            'value': value,
            'unit': 'constraint+Jacobian evals/s (g, dg/dw, f, grad f per instance)',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': elapsed / args.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': args.dtype,
            'data': 'synthetic: seeded cold-start instances (SURVEY 8(d) config 3 generator)',
            'config': {'workload': 'racetrack_parametric_esp_drone_colloc_N50_K4', 'N': 50, 'K': 4, 'nz': 13,
                       'nu': 4, 'batch_per_gpu': B, 'global_batch': world * B, 'layout': args.layout,
                       'nw': nw, 'ng': ng, 'nnz': nnz, 'parallelism': f'instances sharded x{world}'},
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'kernel': 'k_eval', 'kernel_avg_us': kernel_s * 1e6,
                         'reduce_avg_us': r_ms / max(calls, 1) * 1e3,
                         'timed_launches': calls, 'timing_stride': TIMING_STRIDE,
                         'algorithmic_bytes_per_launch': B * bytes_per_eval},
            'cpu_baseline': None,
        }
        if world == 1 and not args.no_cpu_baseline:
            out['cpu_baseline'] = cpu_baseline(spec_kwargs, W, args.cpu_seconds)
        if world == 1 and not args.no_solve:
            out['sqp'] = batched_solve(args.solve_batch, args.solve_max_iter)
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
