"""Multi-GPU sharding of a robot batch.

Robot instances are independent: GPU g solves the contiguous shard [g*B/G, (g+1)*B/G); the only
exchange is one all-gather of the solved first-step forces u0 (12 doubles per robot) so every rank
holds the whole batch's GRFs (north_star: "RCCL all-gather of solved ground-reaction forces over
xGMI").  One process per GPU; torch.distributed with backend "nccl" (= RCCL on ROCm) on the GPUs,
"gloo" in the CPU tests.
"""
import torch
import torch.distributed as dist


def shard_range(total, world, rank):
    """Contiguous, balanced shard [begin, end) of `total` robots for `rank` of `world`."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    base, rem = divmod(total, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def allgather_forces(local, total, group=None):
    """All-gather per-rank [b_r, 12] force rows into [total, 12] on every rank.

    Shards may differ by one row (balanced split); they are padded to ceil(total/world) for a
    single all_gather_into_tensor and the padding is stripped.
    """
    world = dist.get_world_size(group)
    chunk = -(-total // world)
    pad = torch.zeros((chunk, local.shape[1]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    out = torch.empty((world * chunk, local.shape[1]), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, pad, group=group)
    rows = []
    for r in range(world):
        b, e = shard_range(total, world, r)
        rows.append(out[r * chunk: r * chunk + (e - b)])
    return torch.cat(rows, 0)
