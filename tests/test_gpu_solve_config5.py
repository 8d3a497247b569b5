'''
Config 5 as a solve: the fig-8 drone raceline (scripts/fig_8.py, parametric, global_r,
N = 50, K = 4) with the build-side DCM pose over B = 8192 perturbed point-mass warm starts on one GPU.
Its own file, run last: the batch holds ~150 GB of device memory (factor storage 12.4 MB per instance).
'''
import numpy as np
import pytest

from tests.helpers import oracle_nlp

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')

B = 8192
CFG = dict(track='fig8', model='drone', frame='parametric', N=50, K=4, use_quat=True, global_r=True)
@pytest.mark.timeout(1000)
def test_config5_batched_dcm_solve_b8192():
    '''
    Config 5 as a solve: the fig-8 drone raceline with the DCM pose, B = 8192 instances on
    one GPU -- perturbed point-mass warm starts (raceline/batch_instances.py: one point-mass solve, the
    drone guess, seeded perturbations of step sizes, lateral offsets and speeds), solved in lockstep by
    the batched interior-point solver with fp64 evaluation and fp64 KKT (the fp32 evaluation kernel is
    the config's evaluation line; the IPOPT algorithm runs in fp64 throughout). At least 90 % converge;
    every 1024th converged instance is a KKT point of the oracle's DCM NLP, and its interval starts lie
    on SO(3).
    '''
    import time
    from aircraft_trajectory_optimization_amd.raceline.batch_instances import warm_started_batch
    from aircraft_trajectory_optimization_amd.solver.batched_ipm import device_solver
    from aircraft_trajectory_optimization_amd.solver.ipm import IPMOptions
    from tests.helpers import kkt_certificate
    kw = dict(CFG, use_dcm=True)
    spec, W, LBW, UBW, plap = warm_started_batch(B, **{k: v for k, v in kw.items() if k != 'model'})
    t0 = time.time()
    solver = device_solver(spec, B, LBW, UBW, IPMOptions(max_iter=1000))
    try:
        res = solver.solve(W, progress=20)          # a line every 20 lockstep iterations
        torch.cuda.synchronize()
    finally:
        solver.kkt.close()
        del solver
        torch.cuda.empty_cache()
    st = res.status
    ok = [b for b, s in enumerate(st) if s in ('optimal', 'acceptable')]
    laps = res.x[:spec.N].sum(0).cpu().numpy()
    print(f'config 5 DCM solve, B = {B}: {time.time() - t0:.1f} s, statuses',
          {s: st.count(s) for s in sorted(set(st))}, f'median iterations {np.median(res.iters):.0f}, '
          f'lap {laps[ok].min():.4f} .. {laps[ok].max():.4f} s (point mass {plap:.4f} s)')
    assert len(ok) >= 0.9 * B, {s: st.count(s) for s in set(st)}
    nlp = oracle_nlp(**kw, quat_flip=spec.quat_flip)
    for i, b in enumerate(ok):
        if i % 1024:
            continue
        x = res.x[:, b].cpu().numpy()
        c = kkt_certificate(nlp, x, res.lam_g[:, b].cpu().numpy(), res.lam_x[:, b].cpu().numpy(), LBW[b], UBW[b])
        assert c['primal'] <= 1e-5 and c['dual'] <= 1e-6 and c['compl'] <= 1e-6, (b, c)
        orth = max(np.abs(x[spec.col_z(n, 0, 3):spec.col_z(n, 0, 12)].reshape(3, 3).T @
                          x[spec.col_z(n, 0, 3):spec.col_z(n, 0, 12)].reshape(3, 3) - np.eye(3)).max()
                   for n in range(1, spec.N))
        assert orth <= 1e-8, (b, orth)
