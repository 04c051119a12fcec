"""Multi-GPU plumbing of the bench: one process per GPU, frames sharded by
rank, no collective on the data path.  torch.distributed is
used only for the start/stop barriers and the max-over-ranks wall time
(RCCL on GPUs, gloo in the CPU tests)."""
import os


def env():
    """(world, rank, local_rank) from the torchrun environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_seed(rank, stride=1_000_000):
    """First synthetic-frame seed of a rank's own sequence (s*10^6 + t)."""
    return stride * rank


def init(backend, device=None):
    import torch.distributed as dist
    if device is None:
        dist.init_process_group(backend)
    else:
        dist.init_process_group(backend, device_id=device)
    return dist


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(value, world, device="cpu"):
    """Wall time of the job = the slowest rank's."""
    if world == 1:
        return float(value)
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, world, device="cpu"):
    if world == 1:
        return int(value)
    import torch
    import torch.distributed as dist
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def gather_tables(tables, world):
    """SURVEY §8e / BASELINE C4: collect every rank's fixed-capacity per-frame
    tables (e.g. counts [B], keypoints [B, cap, 28 B], descriptors
    [B, cap, 32]) on every rank, rank-major — one all_gather_into_tensor per
    table (RCCL over xGMI on GPUs, gloo on CPU).  Tables are byte tensors of
    identical shape on all ranks; returns a list of [world, *shape] tensors.
    Not on the extract+match data path: frames are independent per rank."""
    import torch
    import torch.distributed as dist
    out = []
    for t in tables:
        t = t.contiguous()
        if world == 1:
            out.append(t.unsqueeze(0).clone())
            continue
        g = torch.empty((world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        if t.device.type == "cpu":  # gloo has no all_gather_into_tensor
            dist.all_gather(list(g.unbind(0)), t)
        else:
            dist.all_gather_into_tensor(g, t)
        out.append(g)
    return out
