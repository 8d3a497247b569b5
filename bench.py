#!/usr/bin/env python
'''
Benchmark of BASELINE.json's metric: "SQP iters/sec (batched) + lap-time err vs CasADi, 50x4
collocation" -- the batched interior-point (SQP-type) solve of the racetrack 50 x 4 drone NLP
whose every iteration evaluates g(w), dg/dw, f, grad f and the Hessian on the GPU (the hot path:
what IPOPT asks CasADi for on every iterate of the reference, base_raceline.py:165, :182-189),
factorises and solves the KKT systems on the GPU, and runs the line search.

Workload (BASELINE.json configs[2]): racetrack of scripts/race.py,
parametric frame, quaternion drone (13 states, 4 inputs), global attitude, square gates, closed
loop, N = 50, K = 4 Legendre collocation, fp64, B = 512 seeded COLD starts per GPU
(raceline/instances.py), IPOPT's max_iter = 1000 (base_raceline.py:54).

One step = one lockstep iteration of the batched solver over its batch. The solve starts from the
cold starts; lockstep iterations [W, W + K) are timed (device synchronised at both ends; the
first W are the warmup); value = instance-iterations in the window of all ranks / slowest rank's
window time. The solve then runs to completion (every instance optimal / acceptable / max_iter /
failed), and the full solve is reported beside it (sqp_full: it/s over the whole solve,
converged solves/s, statuses, lap times, KKT errors). Multi-GPU: one process per GPU, instances
sharded (weak scaling), no communication while solving; per-instance 32-byte records
{lap, KKT error, iterations, status} are all-gathered over RCCL afterwards.

Also measured: the evaluation kernel alone (ato_eval over the same batch, `evals`, with the
k_eval HBM roofline from >= 10 sampled launches) and the CPU baselines (rank 0, N = 1).

    python bench.py [--gpus N --steps K --warmup W --batch B --max-iter 1000]
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
SPEC_KW = dict(track='race', model='drone', frame='parametric', N=50, K=4, use_quat=True, global_r=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20, help='timed lockstep SQP iterations (the driver runs 20)')
    ap.add_argument('--warmup', type=int, default=5, help='untimed lockstep iterations before the window (driver: 5)')
    ap.add_argument('--batch', type=int, default=512, help='instances per GPU')
    ap.add_argument('--max-iter', type=int, default=1000, help="IPOPT's max_iter (base_raceline.py:54)")
    ap.add_argument('--eval-steps', type=int, default=200)
    ap.add_argument('--eval-warmup', type=int, default=20)
    ap.add_argument('--dtype', choices=['f64', 'f32'], default='f64', help='evaluation-kernel bench dtype')
    ap.add_argument('--layout', choices=['interleaved', 'instance'], default='interleaved')
    ap.add_argument('--track', choices=['race', 'fig8', 'obstacles'], default='race',
                    help='fig8: the config-5 evaluation workload (scripts/fig_8.py, N = 50, K = 4), with --dtype f32 '
                         '--batch 8192 --no-solve; obstacles: config 4 (obstacles.py pipeline over perturbed '
                         'tubes, raceline/obstacle_batch.py)')
    ap.add_argument('--pose', choices=['esp', 'dcm'], default='esp',
                    help='attitude: esp (quaternion, the reference\'s) or dcm (config 5\'s direction-cosine-matrix '
                         'pose, build-side): --track fig8 --pose dcm --dtype f32 --batch 8192 --no-solve')
    ap.add_argument('--cpc', action='store_true',
                    help='config 5\'s CPC gate-progress formulation (build-side, global frame, the gates as '
                         'waypoints; N rounds up to the gate phases): --track fig8 --pose dcm --cpc --dtype f32 '
                         '--batch 8192 --no-solve')
    ap.add_argument('--jac32', action='store_true',
                    help='config 5 solve (--track fig8): the Jacobian of every iterate from the fp32 evaluation kernel '
                         '(g, f, grad f, the Hessian and the KKT stay fp64); use with --tol 1e-6')
    ap.add_argument('--tol', type=float, default=1e-8, help="IPOPT's tol (1e-8, base_raceline.py defaults)")
    ap.add_argument('--cpu-seconds', type=float, default=15.0, help='budget of the CPU baselines')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-solve', action='store_true', help='evaluation kernel only')
    ap.add_argument('--no-single', action='store_true', help='skip the B = 1 re-solve of instance 0')
    ap.add_argument('--progress', type=int, default=0, help='solver progress line every N lockstep iterations')
    ap.add_argument('--traffic-json', default=os.path.join(ROOT, 'profiles', 'traffic_latest.json'))
    return ap.parse_args()


def eval_bench(spec, W, args, dev, world):
    '''
    ato_eval over the batch (inputs resident in HBM): evals/s and the k_eval roofline. Kernel
    durations come from HIP events recorded inside the library on the evaluation stream, on
    every stride-th step so that >= 40 launches are sampled (each recorded step adds ~10 us of
    event gaps, tools/diag/step_gaps.py, which the other steps do not pay; with 10 samples the
    average wandered by +-2 us against the rocprof average of the same run, r06final).
    '''
    import torch
    import torch.distributed as dist
    from aircraft_trajectory_optimization_amd import native
    from aircraft_trajectory_optimization_amd.raceline.batched import BatchedNLP
    from aircraft_trajectory_optimization_amd.raceline.shard import max_over_ranks
    B = W.shape[0]
    dtype = torch.float64 if args.dtype == 'f64' else torch.float32
    layout = native.ATO_LAYOUT_INTERLEAVED if args.layout == 'interleaved' else native.ATO_LAYOUT_INSTANCE_MAJOR
    bn = BatchedNLP(spec, B, dtype=dtype, layout=layout, device=dev)
    bn.set_w(W)
    nw, ng, nnz = bn.sizes
    for _ in range(args.eval_warmup):
        bn.evaluate()
    stride = max(1, args.eval_steps // 40)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    bn.problem.timing_stride(stride)
    bn.problem.timing_start((args.eval_steps + stride - 1) // stride)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.eval_steps):
        bn.evaluate()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(t1 - t0, dev)
    k_ms, r_ms, calls = bn.problem.timing_read()
    bn.problem.timing_start(0)
    bn.problem.timing_stride(1)
    g, _, f, _ = bn.results()
    assert np.isfinite(g).all() and np.isfinite(f).all(), 'non-finite evaluation results'
    elem = 8 if args.dtype == 'f64' else 4
    # read w; write g, J, the structural nonzeros of grad f (h and the inputs: the states
    # never enter the cost) and f
    nnz_gf = bn.problem.gradf_nnz()
    bytes_per_eval = elem * (nw + ng + nnz + nnz_gf + 1)
    kernel_s = (k_ms / max(calls, 1)) / 1e3
    achieved = B * bytes_per_eval / kernel_s / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json, encoding='utf-8'))
            if (tj.get('batch'), tj.get('dtype'), tj.get('layout'), tj.get('track', 'race'), tj.get('pose', 'esp'),
                    tj.get('cpc', False)) == (B, args.dtype, args.layout, args.track, args.pose, args.cpc):
                traffic = tj.get('hbm_bytes_per_launch')
        except (OSError, ValueError):
            traffic = None
    evals = {'value': world * B * args.eval_steps / elapsed, 'unit': 'constraint+Jacobian evals/s (g, dg/dw, f, '
             'grad f per instance, all GPUs)', 'steps': args.eval_steps, 'warmup': args.eval_warmup,
             'ms_per_step': elapsed / args.eval_steps * 1e3, 'dtype': args.dtype, 'layout': args.layout,
             'nw': nw, 'ng': ng, 'nnz': nnz, 'nnz_grad_f': nnz_gf}
    roofline = {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic, 'kernel': 'k_eval',
                'kernel_avg_us': kernel_s * 1e6, 'reduce_avg_us': r_ms / max(calls, 1) * 1e3,
                'timed_launches': calls, 'timing_stride': stride,
                'algorithmic_bytes_per_launch': B * bytes_per_eval,
                'note': 'the evaluation kernel of every SQP iteration, timed on its own (evals)'}
    return evals, roofline


def cpu_baseline(W, budget_s, spec_kw):
    '''
    Rank 0, N = 1, on the GPU box's host cores:
      * value: the single-instance interior-point solve on the CPU -- the same algorithm
        (solver/ipm.py) with every evaluation by the C++ CPU twin of the programs
        (tests/native/hostcheck.cpp, g++ -O3, 1 thread) and the host block LDL^T KKT -- on
        instance 0 of the same cold starts, capped so it runs about budget_s / 2: SQP it/s;
      * the C++ twin's evaluation rate (g, dg/dw, f, grad f) on 1 thread and on all threads,
        and the numpy oracle's (complex-step Jacobian), as sub-keys.
    The reference's CasADi/IPOPT path cannot run anywhere in this pipeline.
    '''
    from aircraft_trajectory_optimization_amd.solver.ipm import InteriorPointSolver, IPMOptions
    from aircraft_trajectory_optimization_amd.tracks import make_spec
    from tests.helpers import HostCheck, HostEvaluator, oracle_nlp
    spec = make_spec(**spec_kw)
    ev = HostEvaluator(spec)
    # calibrate the iteration cap on a short solve, then time the capped solve
    t0 = time.perf_counter()
    InteriorPointSolver(ev, spec.lbw, spec.ubw, ev.lbg, ev.ubg, IPMOptions(max_iter=3)).solve(W[0])
    per_it = (time.perf_counter() - t0) / 3
    cap = int(max(5, min(1000, budget_s / 2 / max(per_it, 1e-3))))
    t0 = time.perf_counter()
    r = InteriorPointSolver(ev, spec.lbw, spec.ubw, ev.lbg, ev.ubg, IPMOptions(max_iter=cap)).solve(W[0])
    t_solve = time.perf_counter() - t0
    hc = HostCheck(spec.native_spec())
    threads = max(1, int(os.environ.get('OMP_NUM_THREADS', os.cpu_count() or 1)))

    def rate(nthreads, budget):
        out = None
        n, t0_ = 0, time.perf_counter()
        while time.perf_counter() - t0_ < budget:
            out = hc.eval_threads(W, nthreads, out)
            n += W.shape[0]
        return n / (time.perf_counter() - t0_), n

    r1, n1 = rate(1, budget_s / 4)
    rT, nT = rate(threads, budget_s / 4)
    # the same SQP on every core: one cold start per worker process (tools/cpu_baseline.py, a child
    # process that never touches the GPU), same wall-time budget as the 1-core solve
    import subprocess
    allc = None
    try:
        cp = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'cpu_baseline.py'), '--workers', str(threads),
                             '--budget', str(budget_s / 2), '--spec', json.dumps(spec_kw)],
                            capture_output=True, text=True, timeout=budget_s * 4 + 120, check=False)
        allc = json.loads(cp.stdout.strip().splitlines()[-1]) if cp.returncode == 0 else {'error': cp.stderr[-400:]}
    except (subprocess.TimeoutExpired, ValueError, IndexError) as exc:
        allc = {'error': repr(exc)}
    nlp = oracle_nlp(**spec_kw)
    t0 = time.perf_counter()
    for k in range(2):
        nlp.g(W[k])
        nlp.jac_dense(W[k])
    r_np = 2 / (time.perf_counter() - t0)
    return {'value': r.iters / t_solve, 'unit': 'SQP iterations/s (one instance)', 'cores': 1, 'kind': 'port',
            'sample': f'instance 0 of the config-3 cold starts, the interior-point solver (solver/ipm.py) with the '
                      f'C++ CPU twin of the programs (1 thread) and the host block LDL^T KKT: {r.iters} iterations '
                      f'(cap {cap}) in {t_solve:.1f} s; twin evaluations: {nT} on {threads} threads, {n1} on 1 '
                      f'thread; numpy oracle 2 instances',
            'evals_per_s_1_thread': r1, 'evals_per_s_all_threads': rT, 'eval_threads': threads,
            'numpy_oracle_evals_per_s': r_np,
            'sqp_all_cores': None if allc is None or 'error' in allc else
            {'cores': allc['workers'], 'iterations_per_s': allc['iterations_per_s'], 'budget_s': allc['budget_s'],
             'per_worker_iterations_per_s': allc.get('per_worker_iterations_per_s'), 'pinned': allc.get('pinned'),
             'sample': f"{allc['workers']} worker processes, one config-3 cold start each (seeds 0..), the same "
                       f"solver on the C++ twin + host block LDL^T, {allc['budget_s']:.0f} s each: "
                       f"{allc['iterations']} iterations"},
            'sqp_all_cores_error': allc.get('error') if allc else None}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from aircraft_trajectory_optimization_amd.raceline.batched_solve import gather_solve_records, solve_records, \
        solve_shard, summarize_records, time_solution_gathers, window_timer, RECORD_BYTES
    from aircraft_trajectory_optimization_amd.raceline.instances import seeded_instances
    from aircraft_trajectory_optimization_amd.raceline.shard import max_over_ranks, shard_seeds
    from aircraft_trajectory_optimization_amd.solver.ipm import IPMOptions
    from aircraft_trajectory_optimization_amd.tracks import make_spec

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)                 # before the process group: RCCL binds this rank's device
    dev = torch.device('cuda', local)
    if world > 1:
        dist.init_process_group('nccl', device_id=dev)

    if args.track == 'obstacles':
        return obstacles_main(args, dev, world, rank)
    spec_kw = dict(SPEC_KW, track=args.track, use_dcm=args.pose == 'dcm')
    if args.cpc:
        if not args.no_solve:
            raise SystemExit('--cpc is an evaluation workload: add --no-solve')
        spec_kw.update(frame='global', cpc={'waypoints': None, 'tol': 0.3})
    spec = make_spec(**spec_kw)
    B = args.batch
    track = 'racetrack' if args.track == 'race' else 'fig8'
    seeds = shard_seeds(rank, world, B)
    W, _, _ = seeded_instances(spec, seeds)

    # ---- 1. the evaluation kernel alone (k_eval roofline)
    evals, roofline = eval_bench(spec, W, args, dev, world)

    out = None
    if not args.no_solve:
        # ---- 2. the batched SQP solve: lockstep iterations [W, W + K) timed, then to completion
        sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731
        hook, win = window_timer(args.warmup, args.steps, sync)
        sync()
        if world > 1:
            dist.barrier()
        if args.track == 'fig8':
            # config 5 as a solve: the fig-8 drone (DCM or ESP pose) over per-instance corridors, each
            # warm-started from its own point-mass raceline (raceline/batch_instances.py corridor_batch:
            # one batched point-mass solve, before the timed solve), fp64 evaluation and KKT
            from aircraft_trajectory_optimization_amd.raceline.batch_instances import corridor_batch
            from aircraft_trajectory_optimization_amd.solver.batched_ipm import device_solver
            wkw = {k: v for k, v in spec_kw.items() if k not in ('model',)}
            spec, Wws, LBW, UBW, _, _ = corridor_batch(len(seeds), device=dev, seeds=seeds,
                                                        progress=args.progress, **wkw)
            sync()
            t0 = time.perf_counter()
            solver = device_solver(spec, len(seeds), LBW, UBW, IPMOptions(max_iter=args.max_iter, tol=args.tol),
                                   device=dev, jac32=args.jac32)
            res = solver.solve(Wws, on_iteration=hook, progress=args.progress)
        else:
            t0 = time.perf_counter()
            if args.jac32:
                raise SystemExit('--jac32 is the config-5 solve leg: --track fig8')
            res, solver, _ = solve_shard(spec, seeds, IPMOptions(max_iter=args.max_iter, tol=args.tol), on_iteration=hook,
                                         progress=args.progress)
        sync()
        t_solve = time.perf_counter() - t0
        if win['t0'] is None or win['t1'] is None:
            raise RuntimeError('the solve ended before the timed window began')
        window_s = max_over_ranks(win['t1'] - win['t0'], dev)
        counts = torch.tensor([float(win['count']), float(win['timed']), float(win['count_main']),
                               float(win['count_resto'])], dtype=torch.float64, device=dev)
        timed_min = torch.tensor([float(win['timed'])], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(counts, op=dist.ReduceOp.SUM)
            dist.all_reduce(timed_min, op=dist.ReduceOp.MIN)
        solve_s = max_over_ranks(t_solve, dev)
        rec = solve_records(spec, res, solver)
        allrec = gather_solve_records(rec)            # RCCL all-gather of the 32-byte records
        # the optional audit gather of the converged decision vectors, after the window
        sol_gather = time_solution_gathers(res.x.T.contiguous(), sync, dev) if world > 1 else None
        lockstep = int(len(solver.history))
        if rank == 0:
            summ = summarize_records(allrec)
            steps_timed = int(timed_min.item())
            value = float(counts[0].item()) / window_s
            sqp_full = {'window': {'instance_iterations': int(counts[0].item()),
                                   'main_loop': int(counts[2].item()), 'restoration_phases': int(counts[3].item()),
                                   'note': 'value counts both, as IPOPT\'s iteration counter (and max_iter, and '
                                           'instance_iterations below) does'},
                        'solve_s': solve_s, 'lockstep_iterations': lockstep,
                        'iterations_per_s': summ['instance_iterations'] / solve_s,
                        'converged_solves_per_s': summ['converged'] / solve_s, 'max_iter': args.max_iter,
                        'records_all_gathered': {'bytes_per_instance': RECORD_BYTES, 'instances': len(allrec),
                                                 'collective': 'all_gather' + (' (RCCL)' if world > 1 else ' (1 rank)')},
                        **summ, 'solver_stats': {k: v for k, v in res.stats.items() if k not in ('resto_phases',)}}
            if sol_gather is not None:
                sqp_full['solutions_all_gathered'] = sol_gather
            lap_err = None
            if not args.no_single:
                # the first OPTIMAL instance re-solved alone (B = 1) from the same start: batched vs
                # single-instance lap time (an unconverged instance would compare two stopped iterates)
                from aircraft_trajectory_optimization_amd.raceline.batched_solve import solve_shard as one
                opt = [i for i, st in enumerate(res.status) if st == 'optimal']
                i0 = opt[0] if opt else 0
                if args.track == 'fig8':
                    s1 = device_solver(spec, 1, LBW[i0:i0 + 1], UBW[i0:i0 + 1],
                                       IPMOptions(max_iter=args.max_iter, tol=args.tol), device=dev, jac32=args.jac32)
                    r1 = s1.solve(Wws[i0:i0 + 1])
                else:
                    r1, s1, _ = one(spec, [seeds[i0]], IPMOptions(max_iter=args.max_iter, tol=args.tol))
                lap1 = float(r1.x[:spec.N].sum())
                lap_err = abs(float(allrec[i0, 0]) - lap1)
                sqp_full['lap_check_instance'] = {'seed': int(seeds[i0]), 'batched_lap_s': float(allrec[i0, 0]),
                                                  'single_lap_s': lap1, 'batched_status': res.status[i0],
                                                  'single_status': r1.status[0], 'batched_iters': int(res.iters[i0]),
                                                  'single_iters': int(r1.iters[0])}
            out = {
                'metric': METRIC,
                'value': value,
                'unit': 'SQP iterations/s (instance-iterations of the batched interior-point solve, all GPUs)',
                'n_gpus': world,
                'steps': steps_timed,
                'warmup': args.warmup,
                'ms_per_step': window_s / max(steps_timed, 1) * 1e3,
                'higher_is_better': True,
                'scaling': 'weak',
                'vs_baseline': None,
                'dtype': 'f64',
                'precision': ('fp32 Jacobian (ato_eval_f32, widened), fp64 g / f / grad f / Hessian / KKT' if args.jac32
                              else 'fp64 throughout'),
                'data': ('synthetic: seeded per-instance corridors, each warm-started from its own point-mass raceline '
                         '(raceline/batch_instances.py corridor_batch)' if args.track == 'fig8'
                         else 'synthetic: seeded cold-start instances (SURVEY 8(d) config 3 generator, '
                              'raceline/instances.py)'),
                'config': {'workload': f'{track}_parametric_{args.pose}_drone_colloc_N50_K4_'
                                       f'{"warm" if args.track == "fig8" else "cold"}_start_batched_sqp',
                           'N': 50, 'K': 4, 'nz': spec.nz, 'nu': 4, 'batch_per_gpu': B, 'global_batch': world * B,
                           'max_iter': args.max_iter, 'tol': args.tol, 'layout': args.layout,
                           'parallelism': f'instances sharded x{world}, records all-gathered'},
                'lap_time_err_vs_casadi': None,
                'lap_time_err_note': 'CasADi/IPOPT cannot run in this pipeline (SURVEY F8): lap-time parity with it '
                                     'is unpinned; the transcription is pinned to the reference\'s own code '
                                     '(tests/golden), solutions by oracle KKT + second-order certificates; '
                                     'lap_time_err_batched_vs_single_s compares the first optimal instance '
                                     'batched vs alone (sqp_full.lap_check_instance)',
                'lap_time_err_batched_vs_single_s': lap_err,
                'roofline': roofline,
                'cpu_baseline': None,
                'evals': evals,
                'sqp_full': sqp_full,
            }
            if world == 1 and not args.no_cpu_baseline:
                cb = cpu_baseline(W, args.cpu_seconds, spec_kw)
                # a CPU cold solve needs hundreds of iterations (the GPU run's median for a converged
                # instance), far beyond the bounded sample: converged solves/s on the host cores is the
                # measured it/s over that median (an estimate, labelled as such)
                med = summ.get('iterations', {}).get('median')
                if med:
                    cb['converged_solves_per_s_1_core_est'] = cb['value'] / med
                    if cb.get('sqp_all_cores'):
                        cb['sqp_all_cores']['converged_solves_per_s_est'] = \
                            cb['sqp_all_cores']['iterations_per_s'] / med
                    cb['converged_est_note'] = (f'CPU iterations/s divided by the median iterations per instance of '
                                                f'the GPU solve ({med:.0f}); GPU converged solves/s: '
                                                f'sqp_full.converged_solves_per_s')
                out['cpu_baseline'] = cb
    elif rank == 0:
        out = {'metric': METRIC, 'value': evals['value'], 'unit': evals['unit'], 'n_gpus': world,
               'steps': args.eval_steps, 'warmup': args.eval_warmup, 'ms_per_step': evals['ms_per_step'],
               'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': args.dtype,
               'data': 'synthetic: seeded cold-start instances (evaluation kernel only, --no-solve)',
               'config': {'workload': (f'{track}_global_{args.pose}_cpc_drone_colloc_N{spec.N}_K4_eval' if args.cpc else
                                       f'{track}_parametric_{args.pose}_drone_colloc_N50_K4_eval'), 'batch_per_gpu': B,
                          'nz': spec.nz,
                          'global_batch': world * B, 'layout': args.layout},
               'roofline': roofline, 'cpu_baseline': None, 'evals': evals}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def obstacles_main(args, dev, world, rank):
    '''
    Config 4: obstacles.py's pipeline over perturbed planning tubes, this rank's shard of
    the seeds (raceline/obstacle_batch.py): point-mass racelines on every tube in one batched solve,
    drone guesses, drone solves batched per quaternion closure sign. The timed window is lockstep
    iterations [W, W + K) of the largest drone batch; the whole pipeline is reported beside it.
    '''
    import torch
    import torch.distributed as dist
    from aircraft_trajectory_optimization_amd.raceline.batched_solve import window_timer
    from aircraft_trajectory_optimization_amd.raceline.obstacle_batch import config4_problem, solve_config4_shard
    from aircraft_trajectory_optimization_amd.raceline.problem import ProblemSpec
    from aircraft_trajectory_optimization_amd.raceline.shard import max_over_ranks, shard_seeds
    from aircraft_trajectory_optimization_amd.solver.ipm import IPMOptions
    B = args.batch
    seeds = shard_seeds(rank, world, B)
    prob = config4_problem()
    dspec = ProblemSpec(prob['line'], prob['cfg'].copy(), prob['dveh'], 'parametric', sphere_table=prob['table'])
    evals, roofline = eval_bench(dspec, np.repeat(dspec.w0[None], B, axis=0), args, dev, world)
    sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731
    hook, win = window_timer(args.warmup, args.steps, sync)
    sync()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    r = solve_config4_shard(seeds, IPMOptions(max_iter=args.max_iter), prob, on_iteration=hook)
    sync()
    t_all = max_over_ranks(time.perf_counter() - t0, dev)
    if win['t0'] is None or win['t1'] is None:
        raise RuntimeError('the drone solve ended before the timed window began')
    window_s = max_over_ranks(win['t1'] - win['t0'], dev)
    counts = torch.tensor([float(win['count']), float(win['timed'])], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(counts, op=dist.ReduceOp.SUM)
    st = r['status']
    ok = np.array([x in ('optimal', 'acceptable') for x in st])
    if rank == 0:
        steps_timed = int(win['timed'])
        out = {'metric': METRIC, 'value': float(counts[0].item()) / window_s,
               'unit': 'SQP iterations/s (instance-iterations of the batched drone solve, all GPUs)',
               'n_gpus': world, 'steps': steps_timed, 'warmup': args.warmup,
               'ms_per_step': window_s / max(steps_timed, 1) * 1e3, 'higher_is_better': True, 'scaling': 'weak',
               'vs_baseline': None, 'dtype': 'f64',
               'data': 'synthetic: seeded perturbed planning tubes (SURVEY 8(d) config 4 generator, '
                       'ObstacleFreeTube.perturbed_tables)',
               'config': {'workload': 'obstacles_parametric_esp_drone_colloc_N50_K4_perturbed_tubes_batched_sqp',
                          'N': 50, 'K': 4, 'batch_per_gpu': B, 'global_batch': world * B, 'max_iter': args.max_iter,
                          'drone_batches_by_closure_sign': r['groups'],
                          'parallelism': f'instances sharded x{world}'},
               'lap_time_err_vs_casadi': None,
               'roofline': roofline, 'cpu_baseline': None, 'evals': evals,
               'pipeline': {'wall_s': t_all, 'point_mass_solve_s': r['point_solve_s'],
                            'drone_solve_s': r['drone_solve_s'],
                            'point_mass_optimal': int(sum(x == 'optimal' for x in r['point_status'])),
                            'statuses': {k: st.count(k) for k in sorted(set(st))},
                            'converged_per_s': float(ok.sum()) / t_all,
                            'drone_iterations': {'median': float(np.median(r['iters'])), 'sum': int(r['iters'].sum())},
                            'lap_converged': {'min': float(r['lap'][ok].min()), 'median': float(np.median(r['lap'][ok])),
                                              'max': float(r['lap'][ok].max())} if ok.any() else None}}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
