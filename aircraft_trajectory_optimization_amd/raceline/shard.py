'''
Instance sharding across ranks (one process per GPU).

Problem instances are independent, so rank r of `world` owns the contiguous seed block
[r * per_rank, (r + 1) * per_rank) and evaluates / solves it with no communication. The only
collectives are the max-over-ranks wall time of a timed region and one all-gather of a small
per-instance record (lap time, cost, residual ...) at the end -- RCCL over xGMI on the GPU
box, gloo in the CPU tests.
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
