"""Data-parallel plumbing for the 4-view path: one process per GPU (torchrun env://),
groups sharded across ranks like the reference's DistributedSampler
(lib/utils/utils.py:134-141), no collective on the data path.  The only exchanges are
the benchmark's max-over-ranks wall time and the MPJPE sums (test_triangulate.py's
mean error over all groups), each one small all_reduce.
"""
import os

import torch
import torch.distributed as dist


def env_rank():
    return (int(os.environ.get('RANK', '0')), int(os.environ.get('LOCAL_RANK', '0')),
            int(os.environ.get('WORLD_SIZE', '1')))


def init(backend='nccl', device=None):
    """Initialise the default process group from torchrun's env (127.0.0.1 rendezvous)."""
    rank, local, world = env_rank()
    if world > 1 and not dist.is_initialized():
        kw = {}
        if backend == 'nccl' and device is not None:
            kw['device_id'] = device
        dist.init_process_group(backend, **kw)
    return rank, local, world


def shard_groups(ngroups, rank, world):
    """Strided shard of group indices (DistributedSampler order without shuffling):
    rank r takes r, r + world, ...; every group belongs to exactly one rank."""
    return list(range(rank, ngroups, world))


def max_over_ranks(value, device='cpu'):
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values, device='cpu'):
    """Element-wise sum of a small float vector over ranks (e.g. [error_sum, count])."""
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]


def throughput(frames_per_rank_step, steps, world, elapsed_max):
    """Whole-job frames/s: all ranks' frames over the slowest rank's wall time."""
    return world * frames_per_rank_step * steps / elapsed_max
