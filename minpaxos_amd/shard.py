"""Sharding of independent Paxos groups over ranks.

Groups are block-partitioned: rank p owns [p*G/P, (p+1)*G/P). Everything a group needs (replies,
instance state, commands, KV table) lives on its owner, so a step exchanges nothing but the
watermark vector: committed[G] and executed[G], owner's value, -1 elsewhere, reduced with MAX.
On GPUs that reduction is the engine's RCCL all-reduce (mpx_watermarks_allreduce_dev, one fused
buffer per step); `allreduce_watermarks` is the same step through torch.distributed for the host
side (gloo on CPU) and for tests.
"""
import numpy as np


def block_range(n_groups, world, rank):
    """[start, end) of the groups rank `rank` owns under a block partition."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    return (n_groups * rank) // world, (n_groups * (rank + 1)) // world


def owner_of(group, n_groups, world):
    """rank owning `group` under block_range"""
    r = (group * world) // n_groups
    while block_range(n_groups, world, r)[0] > group:
        r -= 1
    while block_range(n_groups, world, r)[1] <= group:
        r += 1
    return r


def watermark_vector(n_groups, start, committed_own, executed_own):
    """the fused int32 vector [committed[G] | executed[G]] with -1 outside [start, start+n)"""
    wm = np.full(2 * n_groups, -1, np.int32)
    n = len(committed_own)
    wm[start:start + n] = committed_own
    wm[n_groups + start:n_groups + start + n] = executed_own
    return wm


def allreduce_watermarks(wm, group=None):
    """max-all-reduce of the fused watermark vector through torch.distributed (in place for a
    torch tensor; numpy arrays are copied in and out)"""
    import torch
    import torch.distributed as dist
    t = wm if isinstance(wm, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(wm))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t if isinstance(wm, torch.Tensor) else t.numpy()
