'''
The N > 1 path of bench.py on CPU: two gloo ranks shard seeded instances, each computes a
per-instance record (here with the oracle, since there is no GPU), the max-over-ranks time
and the rank-major all-gather must reproduce a single-process run over all seeds.
'''
import os
import socket
import tempfile

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from aircraft_trajectory_optimization_amd.raceline.instances import seeded_instances
from aircraft_trajectory_optimization_amd.raceline.shard import gather_records, max_over_ranks, shard_seeds
from aircraft_trajectory_optimization_amd.tracks import make_spec

CFG = dict(track='race', model='drone', frame='parametric', N=6, K=2, use_quat=True, global_r=True)
PER_RANK = 3


def _records(seeds):
    from tests.helpers import oracle_nlp
    spec = make_spec(**CFG)
    nlp = oracle_nlp(**CFG)
    W, _, _ = seeded_instances(spec, seeds)
    eq = nlp.lbg == nlp.ubg
    return np.stack([[w[:spec.N].sum(), nlp.f(w), np.abs(nlp.g(w)[eq]).max()] for w in W])


def _worker(rank, world, port, out):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        rec = torch.as_tensor(_records(shard_seeds(rank, world, PER_RANK)))
        gathered = gather_records(rec)
        slowest = max_over_ranks(1.0 + rank)
        if rank == 0:
            np.save(out, np.concatenate([gathered.numpy().reshape(-1), [slowest]]))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def test_shard_seeds_partition():
    seen = [s for r in range(4) for s in shard_seeds(r, 4, 5)]
    assert seen == list(range(20))


def test_two_rank_gather_matches_single_process():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, 'gathered.npy')
        mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = np.load(out)
    slowest = res[-1]
    gathered = res[:-1].reshape(world * PER_RANK, 3)
    np.testing.assert_array_equal(gathered, _records(range(world * PER_RANK)))
    assert slowest == 2.0
