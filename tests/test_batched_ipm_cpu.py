'''
The lockstep batched interior-point solver (solver/batched_ipm.py) on CPU stand-ins of its
device pieces: every instance must follow the single-instance solver (solver/ipm.py, the
IPOPT algorithm) -- same status, same iteration count, same solution -- and instances that
converge early must stay frozen while the others iterate.
'''
import numpy as np
import pytest
import torch

from aircraft_trajectory_optimization_amd.solver.batched_ipm import BatchedInteriorPoint
from aircraft_trajectory_optimization_amd.solver.ipm import InteriorPointSolver, IPMOptions
from tests.batched_backends import HostBatchEvaluator, HostBlockKKT
from tests.helpers import HostEvaluator, product_spec


def _instances(spec, B, seed=0):
    rng = np.random.default_rng(seed)
    W = np.repeat(spec.w0[None], B, axis=0)
    for b in range(1, B):
        W[b, :spec.N] *= 1 + 0.1 * rng.uniform(-1, 1, spec.N)
    return W


@pytest.mark.parametrize('cfg', [dict(track='race', model='point', use_quat=False, N=8, K=3),
                                 dict(track='fig8', model='point', use_quat=False, frame='global', N=7, K=2)],
                         ids=['point-param', 'point-global'])
def test_batched_matches_single_instance(cfg):
    spec = product_spec(**cfg)
    B = 3
    W = _instances(spec, B)
    ev = HostBatchEvaluator(spec, B)
    opts = IPMOptions(max_iter=200)
    res = BatchedInteriorPoint(ev, HostBlockKKT(ev), spec.lbw, spec.ubw, opts).solve(W)
    x = res.x.numpy()
    for b in range(B):
        hev = HostEvaluator(spec)
        ref = InteriorPointSolver(hev, spec.lbw, spec.ubw, hev.lbg, hev.ubg, opts).solve(W[b])
        assert res.status[b] == ref.status
        assert res.iters[b] == ref.iters
        assert np.abs(x[:, b] - ref.x).max() <= 1e-6 * max(1.0, np.abs(ref.x).max())
        assert abs(x[:spec.N, b].sum() - ref.x[:spec.N].sum()) <= 1e-8


@pytest.mark.parametrize('cfg', [dict(track='race', model='point', use_quat=False, N=8, K=3),
                                 dict(track='fig8', model='point', use_quat=False, frame='global', N=7, K=2)],
                         ids=['point-param', 'point-global'])
def test_nested_dissection_order_follows_single_instance(cfg):
    ''' the device's nested-dissection elimination order (tests/kkt_emulation.py on the 'nd' plan)
    on real iterates: same statuses and iteration counts (+-5) as the host block LDL^T of the
    single-instance solver, solutions to rounding-level agreement '''
    from tests.batched_backends import EmulatedPlanKKT
    spec = product_spec(**cfg)
    B = 2
    W = _instances(spec, B)
    ev = HostBatchEvaluator(spec, B)
    opts = IPMOptions(max_iter=300)
    res = BatchedInteriorPoint(ev, EmulatedPlanKKT(ev, 'nd'), spec.lbw, spec.ubw, opts).solve(W)
    x = res.x.numpy()
    for b in range(B):
        hev = HostEvaluator(spec)
        ref = InteriorPointSolver(hev, spec.lbw, spec.ubw, hev.lbg, hev.ubg, opts).solve(W[b])
        assert res.status[b] == ref.status
        assert abs(int(res.iters[b]) - ref.iters) <= 5
        # the fig-8 point mass has weakly determined directions (input rates the cost barely
        # sees): another pivot order stops the barrier a couple of iterations later at a point
        # whose objective agrees to 1e-11 and whose inputs agree to ~1e-6 of the largest entry
        assert abs(hev.eval(x[:, b])[0] - hev.eval(ref.x)[0]) <= 1e-9 * max(1.0, abs(hev.eval(ref.x)[0]))
        assert abs(x[:spec.N, b].sum() - ref.x[:spec.N].sum()) <= 1e-8
        assert np.abs(x[:, b] - ref.x).max() <= 1e-5 * max(1.0, np.abs(ref.x).max())



def test_compaction_follows_full_width_solve():
    ''' once at most half of the columns still iterate, the solver carries only those (evaluator
    subset, KKT view, gathered state): every instance's status, iteration count, solution,
    multipliers and per-iteration history equal the full-width solve's '''
    spec = product_spec(track='fig8', model='point', use_quat=False, frame='global', N=7, K=2)
    B = 4
    W = _instances(spec, B, seed=3)
    W[3, :spec.N] *= 0.4                          # a slower instance: the others finish first
    runs = []
    for compact in (False, True):
        ev = HostBatchEvaluator(spec, B)
        solver = BatchedInteriorPoint(ev, HostBlockKKT(ev), spec.lbw, spec.ubw, IPMOptions(max_iter=200))
        solver.compact = compact
        runs.append((solver.solve(W), solver.history))
    (r0, h0), (r1, h1) = runs
    assert r0.stats['compactions'] == 0 and r1.stats['compactions'] >= 1
    assert r0.status == r1.status
    assert [int(i) for i in r0.iters] == [int(i) for i in r1.iters]
    for a, b in ((r0.x, r1.x), (r0.lam_g, r1.lam_g), (r0.lam_x, r1.lam_x), (r0.f, r1.f)):
        assert torch.allclose(a, b, rtol=1e-12, atol=1e-12)
    assert h0.shape == h1.shape and np.allclose(h0, h1, rtol=1e-12, atol=1e-12)


def test_kkt_failure_falls_back_to_restoration():
    ''' IPOPT's fallback mechanism: when no search direction can be computed (delta_w beyond its
    maximum) the instance enters the feasibility restoration phase instead of stopping
    (IpoptAlgorithm::Optimize -> BacktrackingLineSearch::ActivateFallbackMechanism). The KKT step
    of instance 1 is made to fail at its third iteration in both solvers: both restore, neither
    reports 'kkt_failure', and the batched instance follows the single-instance solve. '''
    spec = product_spec(track='race', model='point', use_quat=False, N=8, K=3)
    B = 2
    W = _instances(spec, B)
    ev = HostBatchEvaluator(spec, B)
    opts = IPMOptions(max_iter=200)
    bs = BatchedInteriorPoint(ev, HostBlockKKT(ev), spec.lbw, spec.ubw, opts)
    calls = {'n': 0}
    orig_step = bs._kkt_step

    def failing_step(*args, **kw):
        out = orig_step(*args, **kw)
        calls['n'] += 1
        if calls['n'] == 3:
            ok = out[3].clone()
            ok[1] = False
            out = out[:3] + (ok,) + out[4:]
        return out

    bs._kkt_step = failing_step
    res = bs.solve(W)
    hev = HostEvaluator(spec)
    hs = InteriorPointSolver(hev, spec.lbw, spec.ubw, hev.lbg, hev.ubg, opts)
    hcalls = {'n': 0}
    orig_kkt = hs._kkt

    def failing_kkt(*args, **kw):
        hcalls['n'] += 1
        return None if hcalls['n'] == 3 else orig_kkt(*args, **kw)

    hs._kkt = failing_kkt
    ref = hs.solve(W[1])
    assert ref.stats['restorations'] >= 1 and ref.status != 'kkt_failure'
    assert res.status[1] == ref.status and res.status[0] != 'kkt_failure'
    assert res.iters[1] == ref.iters
    x = res.x.numpy()
    assert np.abs(x[:, 1] - ref.x).max() <= 1e-6 * max(1.0, np.abs(ref.x).max())


def test_batched_backtracking_rounds_match_trial_by_trial():
    ''' the line search's batched backtracking rounds (_multi_round: the next K trials of the searching
    columns evaluated together and tested in order, filter reset heuristic included) against the
    trial-by-trial lockstep loop (LS_MULTI_K = 0): identical statuses, iteration counts, solutions and
    per-iteration histories on drone cold starts that backtrack (K = 8 and K = 2: rounds that leave columns
    searching) '''
    spec = product_spec(track='race', N=4, K=2)
    B = 2
    W = _instances(spec, B, seed=5)
    runs = []
    for k in (0, 8, 2):
        ev = HostBatchEvaluator(spec, B)
        solver = BatchedInteriorPoint(ev, HostBlockKKT(ev), spec.lbw, spec.ubw, IPMOptions(max_iter=25))
        solver.LS_MULTI_K = k
        runs.append((solver.solve(W), solver.history))
    (r0, h0) = runs[0]
    assert r0.stats.get('ls_multi') is None
    for r, h in runs[1:]:
        assert r.stats['ls_multi'][0] > 0
        assert r.status == r0.status
        assert [int(i) for i in r.iters] == [int(i) for i in r0.iters]
        assert torch.equal(r.x, r0.x)
        assert h.shape == h0.shape and np.array_equal(h, h0)
