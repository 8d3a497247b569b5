'''
Config 4 on the GPU (BASELINE configs[3]: obstacle avoidance, sphere rows of the tube).

  * the tube search with the HIP mesh distance against the reference's own search
    (tests/golden/tube.npz, see tests/test_tube_cpu.py),
  * the drone 50 x 4 obstacle problem (obstacles.py track, r_c = 0.4, no gates, one sphere row per
    node from the product's tube) evaluated at full size for B = 4096 seeded cold starts on one
    GPU, against the oracle on instances spread over the batch (fp64, 1e-12 of the scale).
Per-instance tube perturbations are not modelled: a library handle carries
one sphere table, so the instances differ in their starts.
'''
import numpy as np
import pytest

from tests.helpers import REPO, csr_dense, oracle_nlp

pytestmark = pytest.mark.gpu
torch = pytest.importorskip('torch')

GOLD = np.load(f'{REPO}/tests/golden/tube.npz')


def _close(a, b, tol=1e-12):
    np.testing.assert_allclose(a, b, rtol=0, atol=tol * max(1.0, float(np.max(np.abs(b)))))


def test_gpu_tube_search_matches_reference():
    from aircraft_trajectory_optimization_amd.obstacles.mesh_obstacle import MeshObstacle
    from aircraft_trajectory_optimization_amd.tracks import make_line
    env = MeshObstacle()
    tube = env.compute_plannning_tube(make_line('obstacles'), GOLD['s'], float(GOLD['collision_r']))
    np.testing.assert_allclose(tube.ball_r, GOLD['ball_r'], rtol=0, atol=1e-10)
    np.testing.assert_allclose(tube.ball_center, GOLD['ball_center'], rtol=0, atol=1e-10)
    np.testing.assert_allclose(tube.ball_p, GOLD['ball_p'], rtol=0, atol=1e-10)


def _obstacle_problem(N=50, K=4):
    from aircraft_trajectory_optimization_amd.obstacles.mesh_obstacle import MeshObstacle
    from aircraft_trajectory_optimization_amd.pytypes import DroneConfig
    from aircraft_trajectory_optimization_amd.raceline.config import ParametricRacelineConfig
    from aircraft_trajectory_optimization_amd.raceline.problem import ProblemSpec
    from aircraft_trajectory_optimization_amd.tracks import make_line
    line = make_line('obstacles')
    line.config.gate_s = None                     # obstacles.py:21-24: the tube does the work
    cfg = ParametricRacelineConfig(verbose=False, N=N, K=K)
    cfg.closed = True
    cfg.fixed_gates = []
    veh = DroneConfig(global_r=True, use_quat=True, collision_radius=0.4)
    prov = ProblemSpec(line, cfg.copy(), veh, 'parametric')
    tube = MeshObstacle().compute_plannning_tube(line, prov.node_s, veh.collision_radius)
    table = tube.sphere_table(prov.node_s)
    return ProblemSpec(line, cfg, veh, 'parametric', sphere_table=table), table


def test_obstacle_drone_full_size_b4096_matches_oracle():
    from aircraft_trajectory_optimization_amd.raceline.batched import BatchedNLP
    from aircraft_trajectory_optimization_amd.raceline.instances import seeded_instances
    from oracle.ref_transcription import RefNLP
    from tests.helpers import oracle_line
    spec, table = _obstacle_problem()
    B = 4096
    W, _, _ = seeded_instances(spec, range(B))
    bn = BatchedNLP(spec, B)
    nw, ng, _ = bn.sizes
    assert nw == 5300
    bn.set_w(W)
    bn.evaluate()
    g, J, f, gf = bn.results()
    line = oracle_line('obstacles', True)
    nlp = RefNLP(line, 'drone', 'parametric', 50, 4, veh={'use_quat': True, 'global_r': True, 'collision_radius': 0.4},
                 fixed_gates=[], spheres=table)
    assert nlp.ng == ng
    np.testing.assert_array_equal(bn.lbg, nlp.lbg)
    np.testing.assert_array_equal(bn.ubg, nlp.ubg)
    rng = np.random.default_rng(0)
    for b in (0, 63, 64, 2047, 4095):
        _close(g[b], nlp.g(W[b]))
        _close(f[b], nlp.f(W[b]))
        _close(gf[b], nlp.grad_f(W[b]))
        V = rng.standard_normal((nw, 2))
        Jv = np.stack([np.add.reduceat(J[b] * V[bn.col, j], bn.row_ptr[:-1]) for j in range(2)], axis=1)
        _close(Jv, nlp.jvp(W[b], V), 1e-11)
    assert int(np.isin(nlp.ubg, table[:, 2] ** 2).sum()) >= spec.P     # one sphere row per node
