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


def perturbed_warm_starts(spec: ProblemSpec, B: int, seeds=None):
    ''' (W [B, nw], LBW [B, nw], UBW [B, nw]) around spec.w0; seeds (default 0..B-1): instance i draws
    from default_rng(seeds[i]), seed 0 is the unperturbed warm start '''
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
        W[b, :N] *= rng.uniform(0.95, 1.05, N)
        if spec.param:
            W[b, node + 1] += rng.normal(0.0, 0.05, P)
            W[b, node + 2] += rng.normal(0.0, 0.05, P)
        W[b, (node[:, None] + iv + np.arange(3)).reshape(-1)] *= np.repeat(rng.uniform(0.95, 1.05, P), 3)
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

