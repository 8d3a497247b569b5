'''
Seeded batches of warm-started drone instances for the batched solver (build-defined; the
reference solves one problem at a time and has no RNG).

Instance 0 is the point-mass warm start of the drone NLP itself (race.py's use_ws path,
drone_raceline.py:158-274); instance b > 0 draws from numpy.random.default_rng(b):
    step sizes h_n * U[0.95, 1.05], lateral offsets y, n + N(0, 0.05^2) (parametric frame),
    body velocity * U[0.95, 1.05]; bounds as the warm start's (h in [h/100, 10 h]).
'''
import numpy as np

from aircraft_trajectory_optimization_amd.raceline.problem import ProblemSpec


def perturbed_warm_starts(spec: ProblemSpec, B: int, seeds=None, scale: float = 1.0):
    ''' (W [B, nw], LBW [B, nw], UBW [B, nw]) around spec.w0; seeds (default 0..B-1): instance i draws
    from default_rng(seeds[i]), seed 0 is the unperturbed warm start; scale multiplies every
    perturbation amplitude (0.05 relative / 0.05 m at scale 1) '''
    seeds = list(range(B)) if seeds is None else list(seeds)
    N, P, nv = spec.N, spec.P, spec.nv
    node = N + np.arange(P) * nv
    # body velocity: after (s, y, n) and the attitude (quaternion 4, Euler 3, DCM 9)
    iv = {13: 7, 12: 6, 18: 12}[spec.nz] if spec.is_drone else 3
    W = np.repeat(spec.w0[None], B, axis=0)
    LBW = np.repeat(spec.lbw[None], B, axis=0)
    UBW = np.repeat(spec.ubw[None], B, axis=0)
    for b in range(B):
        if seeds[b] == 0:
            continue
        rng = np.random.default_rng(seeds[b])
        W[b, :N] *= (1 + scale * rng.uniform(-0.05, 0.05, N))
        if spec.param:
            W[b, node + 1] += scale * rng.normal(0.0, 0.05, P)
            W[b, node + 2] += scale * rng.normal(0.0, 0.05, P)
        W[b, (node[:, None] + iv + np.arange(3)).reshape(-1)] *= np.repeat(1 + scale * rng.uniform(-0.05, 0.05, P), 3)
        W[b] = np.clip(W[b], LBW[b], UBW[b])
    return W, LBW, UBW


def warm_started_batch(B: int, device=None, seeds=None, **kw):
    '''
    B perturbed warm starts of a drone scenario (make_spec keywords, e.g. track='fig8', use_dcm=True:
    config 5's fig-8 batch with the DCM pose) from ONE point-mass solve on the device (the reference's
    use_ws path, drone_raceline.py:158-274): (drone spec, W, LBW, UBW, point-mass lap time)
    '''
    from aircraft_trajectory_optimization_amd.solver.batched_ipm import device_solver
    from aircraft_trajectory_optimization_amd.solver.ipm import IPMOptions
    from aircraft_trajectory_optimization_amd.tracks import make_spec, make_warm_spec
    pspec = make_spec(**{**kw, 'model': 'point', 'use_quat': False, 'use_dcm': False})
    pres = device_solver(pspec, 1, pspec.lbw[None], pspec.ubw[None], IPMOptions(max_iter=1000),
                         device=device).solve(pspec.w0[None])
    if pres.status[0] != 'optimal':
        raise RuntimeError(f'point-mass warm start: {pres.status[0]}')
    x = pres.x[:, 0].cpu().numpy()
    spec = make_warm_spec(x, **{**kw, 'model': 'drone'})
    W, LBW, UBW = perturbed_warm_starts(spec, B, seeds)
    return spec, W, LBW, UBW, float(x[:pspec.N].sum())



def corridor_bounds(spec: ProblemSpec, seeds, lbw=None, ubw=None):
    '''
    Per-instance corridors (build-defined; config 5's batch): seed 0 keeps the track's tube, seed b > 0
    bounds the lateral offset y of every node (parametric frame) by +-w_b(s), a half-width
    w_b = U[0.8, 1.3] m modulated along the lap by 0.1 m * sin(2 pi k_b s / L + phi_b), k_b in {1, 2, 3}.
    Returns (LBW [B, nw], UBW [B, nw]) from spec's (or the given) bounds.
    '''
    if not spec.param:
        raise ValueError('corridor instances need the parametric frame (lateral offset y)')
    seeds = list(seeds)
    B = len(seeds)
    lbw = spec.lbw if lbw is None else lbw
    ubw = spec.ubw if ubw is None else ubw
    LBW = np.repeat(np.asarray(lbw, float)[None], B, axis=0) if np.ndim(lbw) == 1 else np.array(lbw, float)
    UBW = np.repeat(np.asarray(ubw, float)[None], B, axis=0) if np.ndim(ubw) == 1 else np.array(ubw, float)
    node = spec.N + np.arange(spec.P) * spec.nv
    s = np.array([spec.get_s(n, k) for n in range(spec.N) for k in range(spec.K1)])
    L = spec.line.s_max() - spec.line.s_min()
    for b, sd in enumerate(seeds):
        if sd == 0:
            continue
        rng = np.random.default_rng(sd)
        w0, k, ph = rng.uniform(0.8, 1.3), rng.integers(1, 4), rng.uniform(0, 2 * np.pi)
        w = w0 + 0.1 * np.sin(2 * np.pi * k * (s - spec.line.s_min()) / L + ph)
        LBW[b, node + 1] = np.maximum(LBW[b, node + 1], -w)
        UBW[b, node + 1] = np.minimum(UBW[b, node + 1], w)
    return LBW, UBW


def corridor_batch(B: int, device=None, seeds=None, progress: int = 0, **kw):
    '''
    B drone instances over per-instance corridors (corridor_bounds) of a parametric scenario (make_spec
    keywords, e.g. track='fig8', use_dcm=True: config 5's batch), each warm-started the reference's way
    (use_ws, drone_raceline.py:158-274) from ITS OWN point-mass raceline: one batched point-mass solve on
    the device over the B corridors, then the drone guesses of all of them (drone_guess_batch).
    Returns (drone spec, W, LBW, UBW, point-mass statuses, point-mass lap times [B]); the drone bounds
    carry the instance's corridor and the guess's step-size bounds. Instances whose point-mass solve did
    not converge keep that guess anyway (their status is returned).
    '''
    from aircraft_trajectory_optimization_amd.raceline.warmstart import drone_guess_batch
    from aircraft_trajectory_optimization_amd.solver.batched_ipm import device_solver
    from aircraft_trajectory_optimization_amd.solver.ipm import IPMOptions
    from aircraft_trajectory_optimization_amd.tracks import make_spec
    seeds = list(range(B)) if seeds is None else list(seeds)
    pspec = make_spec(**{**kw, 'model': 'point', 'use_quat': False, 'use_dcm': False})
    PL, PU = corridor_bounds(pspec, seeds)
    psolver = device_solver(pspec, B, PL, PU, IPMOptions(max_iter=1000), device=device)
    pres = psolver.solve(np.repeat(pspec.w0[None], B, axis=0), progress=progress)
    XP = pres.x.T.cpu().numpy()
    if hasattr(psolver.kkt, 'close'):
        psolver.kkt.close()
    del psolver
    spec = make_spec(**{**kw, 'model': 'drone'})
    W, LBW, UBW, flips, wraps = drone_guess_batch(spec, pspec, XP)
    if np.any(flips != flips[0]) or np.any(wraps != wraps[0]):
        # the closure sign / Euler wraps are structural constants of the NLP: one per batch
        raise NotImplementedError('corridor_batch: closure signs or Euler wraps differ between instances')
    if flips[0] or wraps[0]:
        spec = make_spec(**{**kw, 'model': 'drone', 'quat_flip': bool(flips[0]), 'euler_wraps': float(wraps[0])})
    LBW, UBW = corridor_bounds(spec, seeds, LBW, UBW)
    W = np.clip(W, LBW, UBW)
    return spec, W, LBW, UBW, list(pres.status), XP[:, :pspec.N].sum(1)


def cpc_warm_batch(B: int, device=None, seeds=None, use_dcm: bool = True, N: int = 56, K: int = 4,
                   tol: float = 0.3, track: str = 'fig8'):
    '''
    Config 5's CPC instances (build-side gate-progress formulation, global frame; parity unpinned), warm
    started the reference's way (use_ws, drone_raceline.py:158-274) from a point-mass raceline of the SAME
    formulation: one point-mass CPC solve on the device (waypoints, one total time; from its own progress
    guess), then the drone guess from its trajectory (attitude from thrust and velocity, body rates,
    thrusts) with the point mass's progress variables (the node layout of both is the same). Instance
    b > 0 perturbs that start as perturbed_warm_starts does. Returns (spec, W, LBW, UBW, point-mass lap).
    (A drone raceline through the gates re-sampled on a uniform time grid is a worse start: the gate
    rows let the path pass the waypoints by up to the gate opening, the complementarity rows do not.)
    '''
    from aircraft_trajectory_optimization_amd.raceline.warmstart import drone_guess
    from aircraft_trajectory_optimization_amd.solver.batched_ipm import device_solver
    from aircraft_trajectory_optimization_amd.solver.ipm import IPMOptions
    from aircraft_trajectory_optimization_amd.tracks import make_spec
    cpc = {'waypoints': None, 'tol': tol}
    kw = dict(track=track, frame='global', N=N, K=K, use_quat=True, global_r=True, use_dcm=use_dcm)
    pspec = make_spec(**{**kw, 'model': 'point', 'use_quat': False, 'use_dcm': False, 'cpc': cpc})
    # a small batch of perturbed point-mass starts (the complementarity rows make single starts fragile):
    # the converged one with the shortest lap is the warm start
    PW, PL, PU = perturbed_warm_starts(pspec, 16)
    psolver = device_solver(pspec, 16, PL, PU, IPMOptions(max_iter=3000), device=device)
    pres = psolver.solve(PW)
    ok = [b for b, st in enumerate(pres.status) if st in ('optimal', 'acceptable')]
    if not ok:
        raise RuntimeError(f'CPC warm start: no point-mass solve converged ({set(pres.status)})')
    laps = pres.x[:pspec.N].sum(0).cpu().numpy()
    x = pres.x[:, min(ok, key=lambda b: laps[b])].cpu().numpy()
    cpc_warm_batch.point_statuses = list(pres.status)
    p0 = make_spec(**{**kw, 'model': 'point', 'use_quat': False, 'use_dcm': False})
    d0 = make_spec(**{**kw, 'model': 'drone'})
    nx = p0.nw
    w0, lbw, ubw, flip, wraps = drone_guess(d0, p0, x[:nx])
    spec = make_spec(**{**kw, 'model': 'drone', 'quat_flip': flip, 'euler_wraps': wraps, 'cpc': cpc})
    spec.w0 = np.concatenate([np.asarray(w0, float), x[nx:]])
    spec.lbw = np.concatenate([np.asarray(lbw, float), pspec.lbw[nx:]])
    spec.ubw = np.concatenate([np.asarray(ubw, float), pspec.ubw[nx:]])
    W, LBW, UBW = perturbed_warm_starts(spec, B, seeds)
    return spec, W, LBW, UBW, float(x[:pspec.N].sum())


def resample_uniform_time(spec: ProblemSpec, w) -> np.ndarray:
    '''
    A collocation solution w of `spec` (global frame) re-sampled on a uniform time grid of the same N, K:
    every step size becomes T / N (T = sum h, the lap time), and every node variable is interpolated in time
    (linear between the old nodes, the lap closed periodically); quaternions are renormalised, DCM
    attitudes projected back onto SO(3) (polar factor). The CPC formulation has one total time (all h
    equal): a solution with phase-wise steps would violate its dynamics by O(h differences).
    '''
    w = np.asarray(w, float)
    N, K1, nv, nz = spec.N, spec.K1, spec.nv, spec.nz
    h = w[:N]
    T = float(h.sum())
    t0 = np.concatenate([[0.0], np.cumsum(h)[:-1]])
    told = (t0[:, None] + spec.tau[None, :] * h[:, None]).reshape(-1)       # node times
    Z = w[N:N + spec.P * nv].reshape(spec.P, nv)
    hn = T / N
    tnew = (np.arange(N)[:, None] * hn + spec.tau[None, :] * hn).reshape(-1)
    # periodic extension: the closed lap's first node follows the last one at time T
    tx = np.concatenate([told, [T]])
    Zx = np.vstack([Z, Z[:1]])
    Zn = np.stack([np.interp(tnew, tx, Zx[:, c]) for c in range(nv)], axis=1)
    if spec.is_drone:
        if nz == 18:                                   # DCM: rows 3..12, project on SO(3)
            for q in range(spec.P):
                U_, _, Vt = np.linalg.svd(Zn[q, 3:12].reshape(3, 3))
                Zn[q, 3:12] = (U_ @ Vt).reshape(-1)
        elif nz == 13:                                 # quaternion 3..7
            Zn[:, 3:7] /= np.linalg.norm(Zn[:, 3:7], axis=1, keepdims=True)
    out = w.copy()
    out[:N] = hn
    out[N:N + spec.P * nv] = Zn.reshape(-1)
    return out
