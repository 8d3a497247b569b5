'''
Instance sharding across ranks (one process per GPU).

Problem instances are independent, so rank r of `world` owns the contiguous seed block
[r * per_rank, (r + 1) * per_rank) and evaluates / solves it with no communication. The only
collectives are the max-over-ranks wall time of a timed region and one all-gather of a small
per-instance record (lap time, cost, residual ...) at the end -- RCCL over xGMI on the GPU
box, gloo in the CPU tests. The optional audit gather of the converged decision vectors
(347 MB at B = 8192) is a DIRECT all-gather: every rank posts one send of its shard
to each peer and one receive from each (`batch_isend_irecv`, one RCCL group), so on the xGMI
mesh the shards move over the point-to-point links at once instead of around a ring.
'''
from typing import Optional

import torch
import torch.distributed as dist


def shard_seeds(rank: int, world: int, per_rank: int) -> range:
    ''' seeds owned by `rank` (weak scaling: per-rank work fixed as world grows) '''
    if not 0 <= rank < world:
        raise ValueError(f'rank {rank} outside world {world}')
    return range(rank * per_rank, (rank + 1) * per_rank)


def max_over_ranks(seconds: float, device: Optional[torch.device] = None) -> float:
    ''' slowest rank's time for a region every rank timed (the job's wall time) '''
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(seconds)
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_records(records: torch.Tensor) -> torch.Tensor:
    '''
    All-gather per-instance records [B_local, k] from every rank into [world * B_local, k],
    rank-major, so row i of the result is the instance with seed i.
    '''
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return records
    world = dist.get_world_size()
    records = records.contiguous()
    parts = [torch.empty_like(records) for _ in range(world)]
    dist.all_gather(parts, records)
    return torch.cat(parts, dim=0)


def gather_direct(shard: torch.Tensor) -> torch.Tensor:
    '''
    Direct (point-to-point) all-gather of per-rank shards [B_local, ...] into [world * B_local, ...],
    rank-major: rank r sends its shard to every peer and receives every peer's shard, all posted
    as one batch (an RCCL group on the GPU box), instead of the world - 1 ring steps of all_gather.
    '''
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return shard
    world, rank = dist.get_world_size(), dist.get_rank()
    shard = shard.contiguous()
    out = torch.empty((world,) + tuple(shard.shape), dtype=shard.dtype, device=shard.device)
    out[rank].copy_(shard)
    ops = []
    for k in range(1, world):                 # staggered peers: step k talks to rank +- k
        dst, src = (rank + k) % world, (rank - k) % world
        ops.append(dist.P2POp(dist.isend, shard, dst))
        ops.append(dist.P2POp(dist.irecv, out[src], src))
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    return out.reshape((world * shard.shape[0],) + tuple(shard.shape[1:]))
