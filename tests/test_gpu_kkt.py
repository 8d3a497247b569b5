'''
Batched device KKT factorisation and solve (include/ato_kkt.h) against dense linear algebra:
inertia equals the eigenvalue signs of the dense KKT matrix, K x = b is solved to a small
residual, and the result agrees with the test-only CPU emulation of the same algorithm. The
full-size racetrack (50 x 4) is checked against the host block factorisation
(solver/kkt_blocks.py) and the sparse residual. Values are random Hessian / Jacobian values of
the real problem structures.
'''
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from aircraft_trajectory_optimization_amd.solver.ipm import _lower_to_full
from aircraft_trajectory_optimization_amd.solver.kkt_blocks import BlockKKT
from aircraft_trajectory_optimization_amd.solver.kkt_plan import build_plan
from tests.helpers import product_spec, var_stages
from tests.kkt_emulation import Factor, dense_kkt
from tests.test_kkt_plan_cpu import CASES, IDS, random_kkt_values

pytestmark = pytest.mark.gpu


def _dev(arrs):
    ''' list of per-instance 1-D arrays -> interleaved [elem][B] fp64 device tensor '''
    return torch.as_tensor(np.stack(arrs, axis=1), dtype=torch.float64, device='cuda').contiguous()


@pytest.mark.parametrize('ordering', ['nd', 'chain'])
@pytest.mark.parametrize('cfg', CASES, ids=IDS)
def test_device_kkt_matches_dense(cfg, ordering):
    from aircraft_trajectory_optimization_amd.solver.kkt_device import DeviceKKT
    spec = product_spec(**cfg)
    B = 3
    vals = [random_kkt_values(spec, seed) for seed in range(B)]
    ev = vals[0][0]
    plan = build_plan(ev.nw, ev.ng, var_stages(spec), ev.j_row_ptr, ev.j_col, ev.h_row_ptr, ev.h_col, ordering)
    kkt = DeviceKKT(plan, B)
    H = _dev([v[1] for v in vals])
    J = _dev([v[2] for v in vals])
    dx = _dev([v[3] for v in vals])
    dr = _dev([v[4] for v in vals])
    inertia = kkt.factor(H, J, dx, dr).cpu().numpy()
    rng = np.random.default_rng(7)
    rhs = rng.standard_normal((plan.dim, B))
    x = kkt.solve(torch.as_tensor(rhs, device='cuda').contiguous()).cpu().numpy()
    for b in range(B):
        _, Hb, Jb, dxb, drb = vals[b]
        K = dense_kkt(plan, Hb, Jb, dxb, drb, ev.h_row_ptr, ev.h_col, ev.j_row_ptr, ev.j_col)
        eig = np.linalg.eigvalsh(K)
        assert tuple(inertia[b]) == (int((eig > 0).sum()), int((eig < 0).sum()), 0)
        res = np.abs(K @ x[:, b] - rhs[:, b]).max()
        assert res <= 1e-8 * max(1.0, np.abs(K).max()), res
        fe = Factor(plan, Hb, Jb, dxb, drb)
        assert fe.inertia == tuple(inertia[b])
        xe = fe.solve(rhs[:, b])
        assert np.abs(x[:, b] - xe).max() <= 1e-8 * max(1.0, np.abs(xe).max())


def test_device_kkt_instance_list_and_refactor():
    ''' factorising a subset leaves the other instances' factors untouched '''
    from aircraft_trajectory_optimization_amd.solver.kkt_device import DeviceKKT
    spec = product_spec(track='race', N=6, K=4)
    vals = [random_kkt_values(spec, seed) for seed in range(4)]
    ev = vals[0][0]
    plan = build_plan(ev.nw, ev.ng, var_stages(spec), ev.j_row_ptr, ev.j_col, ev.h_row_ptr, ev.h_col)
    kkt = DeviceKKT(plan, 4)
    H, J = _dev([v[1] for v in vals]), _dev([v[2] for v in vals])
    dx, dr = _dev([v[3] for v in vals]), _dev([v[4] for v in vals])
    kkt.factor(H, J, dx, dr)
    rhs = torch.as_tensor(np.random.default_rng(3).standard_normal((plan.dim, 4)), device='cuda').contiguous()
    x_all = kkt.solve(rhs.clone()).cpu().numpy()
    dx2 = dx.clone()
    dx2[:, 2] += 5.0
    kkt.factor(H, J, dx2, dr, instances=[2])
    x2 = kkt.solve(rhs.clone(), instances=[0, 2]).cpu().numpy()
    assert np.array_equal(x2[:, 0], x_all[:, 0])
    _, Hb, Jb, dxb, drb = vals[2]
    K = dense_kkt(plan, Hb, Jb, dxb + 5.0, drb, ev.h_row_ptr, ev.h_col, ev.j_row_ptr, ev.j_col)
    assert np.abs(K @ x2[:, 2] - rhs.cpu().numpy()[:, 2]).max() <= 1e-8 * np.abs(K).max()


def test_device_kkt_is_deterministic():
    ''' repeated factorisations and solves of the same values are bitwise identical (every carried
    Schur entry has one writer; the diagonal tiles' upper copies differ from the lower ones by rounding) '''
    from aircraft_trajectory_optimization_amd.solver.kkt_device import DeviceKKT
    spec = product_spec(track='race', N=6, K=4)
    vals = [random_kkt_values(spec, seed) for seed in range(8)]
    ev = vals[0][0]
    plan = build_plan(ev.nw, ev.ng, var_stages(spec), ev.j_row_ptr, ev.j_col, ev.h_row_ptr, ev.h_col)
    kkt = DeviceKKT(plan, 8)
    H, J = _dev([v[1] for v in vals]), _dev([v[2] for v in vals])
    dx, dr = _dev([v[3] for v in vals]), _dev([v[4] for v in vals])
    rhs = torch.as_tensor(np.random.default_rng(5).standard_normal((plan.dim, 8)), device='cuda').contiguous()
    outs = []
    for _ in range(4):
        kkt.factor(H, J, dx, dr)
        outs.append(kkt.solve(rhs.clone()).clone())
    assert all(torch.equal(outs[0], o) for o in outs[1:])


def test_device_kkt_racetrack_full_size():
    ''' 50 x 4 racetrack (the bench structure): inertia and solution against the host block LDL^T '''
    from aircraft_trajectory_optimization_amd.solver.kkt_device import DeviceKKT
    spec = product_spec(track='race', N=50, K=4)
    B = 2
    vals = [random_kkt_values(spec, seed) for seed in range(B)]
    ev = vals[0][0]
    st = var_stages(spec)
    plan = build_plan(ev.nw, ev.ng, st, ev.j_row_ptr, ev.j_col, ev.h_row_ptr, ev.h_col)
    kkt = DeviceKKT(plan, B)
    inertia = kkt.factor(_dev([v[1] for v in vals]), _dev([v[2] for v in vals]), _dev([v[3] for v in vals]),
                         _dev([v[4] for v in vals])).cpu().numpy()
    rhs = np.random.default_rng(5).standard_normal((plan.dim, B))
    x = kkt.solve(torch.as_tensor(rhs, device='cuda').contiguous()).cpu().numpy()
    bk = BlockKKT(ev.nw, ev.ng, st, ev.j_row_ptr, ev.j_col, ev.h_row_ptr, ev.h_col)
    jr = np.repeat(np.arange(ev.ng), np.diff(ev.j_row_ptr))
    for b in range(B):
        _, Hb, Jb, dxb, drb = vals[b]
        W = _lower_to_full(ev.nw, ev.h_row_ptr, ev.h_col, Hb) + sp.diags(dxb)
        Jm = sp.csr_matrix((Jb, (jr, ev.j_col)), shape=(ev.ng, ev.nw))
        K = sp.bmat([[W, Jm.T], [Jm, sp.diags(drb)]], format='csr')
        fac, host_inertia = bk.factor(K)
        assert tuple(inertia[b]) == tuple(host_inertia)
        res = np.abs(K @ x[:, b] - rhs[:, b]).max()
        assert res <= 1e-8 * max(1.0, abs(K).max()), res


@pytest.mark.parametrize('with_h', [True, False])
def test_device_kkt_residual_matches_dense(with_h):
    ''' ato_kkt_residual (iterative refinement) = rhs - K x of the dense matrix, with and without W '''
    from aircraft_trajectory_optimization_amd.solver.kkt_device import DeviceKKT
    spec = product_spec(track='race', N=6, K=4)
    B = 3
    vals = [random_kkt_values(spec, seed) for seed in range(B)]
    ev = vals[0][0]
    plan = build_plan(ev.nw, ev.ng, var_stages(spec), ev.j_row_ptr, ev.j_col, ev.h_row_ptr, ev.h_col)
    kkt = DeviceKKT(plan, B)
    rng = np.random.default_rng(11)
    x = rng.standard_normal((plan.dim, B))
    rhs = rng.standard_normal((plan.dim, B))
    H = _dev([v[1] for v in vals]) if with_h else None
    out = kkt.residual(H, _dev([v[2] for v in vals]), _dev([v[3] for v in vals]), _dev([v[4] for v in vals]),
                       torch.as_tensor(x, device='cuda'), torch.as_tensor(rhs, device='cuda')).cpu().numpy()
    for b in range(B):
        _, Hb, Jb, dxb, drb = vals[b]
        K = dense_kkt(plan, Hb if with_h else np.zeros_like(Hb), Jb, dxb, drb, ev.h_row_ptr, ev.h_col,
                      ev.j_row_ptr, ev.j_col)
        ref = rhs[:, b] - K @ x[:, b]
        assert np.abs(out[:, b] - ref).max() <= 1e-12 * max(1.0, np.abs(ref).max())
    # ato_kkt_residual_list: the listed columns bitwise as above, the others zero
    args = (H, _dev([v[2] for v in vals]), _dev([v[3] for v in vals]), _dev([v[4] for v in vals]),
            torch.as_tensor(x, device='cuda'), torch.as_tensor(rhs, device='cuda'))
    part = kkt.residual(*args, instances=[2, 0]).cpu().numpy()
    assert np.array_equal(part[:, [0, 2]], out[:, [0, 2]]) and not part[:, 1].any()
    assert not kkt.residual(*args, instances=[]).cpu().numpy().any()


def test_device_kkt_wide_levels_match_narrow():
    ''' levels with many (front, instance) workgroups run other kernel variants (one wave per small
    front, 16-wide tiles for the interval blocks, the classes of a level on two streams) than
    small batches; every variant makes the same operations in the same order on the same
    (lower-triangle) entries, so batches of 48 and 224 copies of one racetrack KKT matrix
    factorise and solve bit for bit like the single instance '''
    from aircraft_trajectory_optimization_amd.solver.kkt_device import DeviceKKT
    spec = product_spec(track='race', N=50, K=4)
    _, Hb, Jb, dxb, drb = random_kkt_values(spec, 3)
    ev = random_kkt_values(spec, 3)[0]
    plan = build_plan(ev.nw, ev.ng, var_stages(spec), ev.j_row_ptr, ev.j_col, ev.h_row_ptr, ev.h_col)
    rhs = np.random.default_rng(9).standard_normal(plan.dim)
    outs = []
    # 48: 16-wide-tile leaves, one-wave pre-fronts; 224: also one-wave separators next to the
    # three-tile class of the same level on the side stream
    for B in (1, 48, 224):
        kkt = DeviceKKT(plan, B)
        inertia = kkt.factor(_dev([Hb] * B), _dev([Jb] * B), _dev([dxb] * B), _dev([drb] * B)).cpu().numpy()
        x = kkt.solve(torch.as_tensor(np.repeat(rhs[:, None], B, axis=1), device='cuda').contiguous())
        outs.append((inertia, x.cpu()))
    (i1, x1) = outs[0]
    for iw, xw in outs[1:]:
        assert all(tuple(iw[b]) == tuple(i1[0]) for b in range(iw.shape[0]))
        for b in range(iw.shape[0]):
            assert torch.equal(xw[:, b], x1[:, 0]), b



# ---------------------------------------------------------------- saddle fronts (k_front_saddle)
def _saddle_setup(cfg, B, seed0=0):
    from aircraft_trajectory_optimization_amd.solver.kkt_plan import collocation_saddle
    spec = product_spec(**cfg)
    vals = [list(random_kkt_values(spec, seed0 + s)) for s in range(B)]
    ev = vals[0][0]
    sad = collocation_saddle(spec.N, spec.K1, spec.nv, spec.nz, ev.ng, ev.j_row_ptr, ev.j_col)
    plan = build_plan(ev.nw, ev.ng, var_stages(spec), ev.j_row_ptr, ev.j_col, ev.h_row_ptr, ev.h_col, saddle=sad)
    return spec, ev, vals, sad, plan


@pytest.mark.parametrize('cfg', [dict(track='fig8', N=5, K=3), dict(track='race', N=6, K=4),
                                 dict(track='race', model='point', use_quat=False, N=8, K=3),
                                 dict(track='race', N=6, K=3, use_dcm=True)], ids=['fig8', 'race-K4', 'point', 'dcm'])
def test_device_saddle_fronts_match_dense(cfg):
    ''' structured saddle elimination on the device (delta_c = 0 on the defect rows of instances 0, 2;
    a row diagonal on instances 1, 3 sends their saddle fronts to Bunch-Kaufman): inertia of the
    dense matrix, dense residual, and the emulation's solution (which takes the same path) '''
    from aircraft_trajectory_optimization_amd.solver.kkt_device import DeviceKKT
    B = 4
    spec, ev, vals, (cols, rows), plan = _saddle_setup(cfg, B)
    for b in (0, 2):
        vals[b][4][rows] = 0.0
    kkt = DeviceKKT(plan, B)
    inertia = kkt.factor(_dev([v[1] for v in vals]), _dev([v[2] for v in vals]), _dev([v[3] for v in vals]),
                         _dev([v[4] for v in vals])).cpu().numpy()
    rhs = np.random.default_rng(9).standard_normal((plan.dim, B))
    x = kkt.solve(torch.as_tensor(rhs, device='cuda').contiguous()).cpu().numpy()
    for b in range(B):
        _, Hb, Jb, dxb, drb = vals[b]
        K = dense_kkt(plan, Hb, Jb, dxb, drb, ev.h_row_ptr, ev.h_col, ev.j_row_ptr, ev.j_col)
        eig = np.linalg.eigvalsh(K)
        assert tuple(inertia[b]) == (int((eig > 0).sum()), int((eig < 0).sum()), 0), b
        assert np.abs(K @ x[:, b] - rhs[:, b]).max() <= 1e-8 * max(1.0, np.abs(K).max()), b
        fe = Factor(plan, Hb, Jb, dxb, drb)
        assert len(fe.sad) == (spec.N if b in (0, 2) else 0)
        xe = fe.solve(rhs[:, b])
        assert np.abs(x[:, b] - xe).max() <= 1e-8 * max(1.0, np.abs(xe).max()), b


def test_device_saddle_racetrack_full_size_and_deterministic():
    ''' racetrack 50 x 4 with saddle fronts (delta_c = 0 on the equality rows): inertia of the
    emulation (which takes the structured path on every saddle front), sparse residual; bitwise
    repeatable '''
    from aircraft_trajectory_optimization_amd.solver.kkt_device import DeviceKKT
    B = 3
    spec, ev, vals, (cols, rows), plan = _saddle_setup(dict(track='race', N=50, K=4), B)
    eq = ev.lbg == ev.ubg
    for v in vals:
        v[4][eq] = 0.0
    kkt = DeviceKKT(plan, B)
    H, J = _dev([v[1] for v in vals]), _dev([v[2] for v in vals])
    dx, dr = _dev([v[3] for v in vals]), _dev([v[4] for v in vals])
    rhs = torch.as_tensor(np.random.default_rng(4).standard_normal((plan.dim, B)), device='cuda').contiguous()
    outs = []
    for _ in range(3):
        inertia = kkt.factor(H, J, dx, dr).cpu().numpy()
        outs.append(kkt.solve(rhs.clone()).clone())
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    x = outs[0].cpu().numpy()
    for b in range(B):
        _, Hb, Jb, dxb, drb = vals[b]
        W = _lower_to_full(ev.nw, ev.h_row_ptr, ev.h_col, Hb) + sp.diags(dxb)
        Jm = sp.csr_matrix((Jb, ev.j_col, ev.j_row_ptr), shape=(ev.ng, ev.nw))
        K = sp.bmat([[W, Jm.T], [Jm, sp.diags(drb)]]).tocsr()
        r = rhs.cpu().numpy()[:, b]
        assert np.abs(K @ x[:, b] - r).max() <= 1e-7 * max(1.0, abs(K).max()), b
        fe = Factor(plan, Hb, Jb, dxb, drb)
        assert tuple(inertia[b]) == fe.inertia
        assert len(fe.sad) == spec.N


def test_device_kkt_nine_tile_fronts_match_dense():
    ''' K = 7 collocation (obstacles.py's default degree): the interval leaves have 261-268
    positions, nine 32-wide tiles (the 512-thread factor kernel at T = 9 and the solve's doubled ring
    chunk); inertia, dense residual and the CPU emulation as above '''
    from aircraft_trajectory_optimization_amd.solver.kkt_plan import build_plan as bp
    cfg = dict(track='race', N=3, K=7)
    spec = product_spec(**cfg)
    ev = random_kkt_values(spec, 0)[0]
    plan = bp(ev.nw, ev.ng, var_stages(spec), ev.j_row_ptr, ev.j_col, ev.h_row_ptr, ev.h_col)
    assert plan.tiles == 9, plan.tiles
    test_device_kkt_matches_dense(cfg, 'nd')
