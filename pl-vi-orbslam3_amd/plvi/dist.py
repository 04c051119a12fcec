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


class TableGather:
    """BASELINE C4's per-step collection of every rank's per-frame tables on
    rank 0 ("RCCL gather of per-frame descriptor tables"), the
    code bench.py runs inside its timed region.

    `sizes` are the byte sizes of the tables (counts, keypoints, descriptors,
    line counts, keylines, LBD descriptors).  `post(srcs, stream)` makes
    `stream` wait for this gatherer's previous gathers (a stream-side wait
    under RCCL, a host wait under gloo; the staging copies must be issued on
    `stream` for that to order them), stages each source into its own byte
    buffer (`copy(dst_tensor, src)`: a device-pointer copy on the step's
    stream in the bench, a tensor copy on CPU) and issues one asynchronous
    `dist.gather` per table to rank 0 on `stream` (RCCL over xGMI on GPUs,
    gloo in the CPU tests).  Staging decouples the gather from the extractor
    outputs, which the next step overwrites.  Rank 0 owns a receive buffer
    per (table, rank): `received(r)` is rank r's tables, rank-major, once
    `wait()` has returned.  At world 1 `post` only stages."""

    def __init__(self, sizes, world, rank, device="cpu", copy=None):
        import torch
        self.world, self.rank = world, rank
        self.sizes = tuple(int(n) for n in sizes)
        self.stage = [torch.empty(n, dtype=torch.uint8, device=device) for n in self.sizes]
        self.recv = None
        if world > 1 and rank == 0:
            self.recv = [[torch.empty(n, dtype=torch.uint8, device=device) for _ in range(world)]
                         for n in self.sizes]
        self.copy = copy if copy is not None else _copy_tensor
        self.pending = []
        self.posted = 0

    def wait(self):
        for w in self.pending:
            w.wait()
        self.pending.clear()

    def post(self, srcs, stream=None):
        import contextlib
        import torch
        if len(srcs) != len(self.stage):
            raise ValueError(f"TableGather.post: {len(srcs)} sources for {len(self.stage)} tables")
        ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
        with ctx:
            # Ordering: the staging buffers are still being read by the
            # previous gathers.  Work.wait() under RCCL/NCCL does not block
            # the host; it makes the CURRENT stream wait for the collective.
            # Calling it inside `stream`'s context puts that wait on the
            # stream the staging copies below are issued on, so they cannot
            # overwrite a buffer an earlier gather is still sending (gloo's
            # wait() blocks the host, which orders them as well).
            self.wait()
            for src, t in zip(srcs, self.stage):
                self.copy(t, src)
            self.posted += 1
            if self.world == 1:
                return
            import torch.distributed as dist
            for i, t in enumerate(self.stage):
                self.pending.append(dist.gather(t, self.recv[i] if self.rank == 0 else None, dst=0,
                                                async_op=True))

    def received(self, r):
        """Rank r's staged tables as rank 0 received them (rank 0 only)."""
        if self.world == 1:
            return list(self.stage)
        if self.recv is None:
            raise RuntimeError("TableGather.received: only rank 0 receives")
        return [self.recv[i][r] for i in range(len(self.sizes))]

    def digests(self):
        """SHA-256 (16 hex) of every rank's received tables, rank order (rank 0)."""
        import hashlib
        out = []
        for r in range(self.world):
            h = hashlib.sha256()
            for t in self.received(r):
                h.update(t.cpu().numpy().tobytes())
            out.append(h.hexdigest()[:16])
        return out


def _copy_tensor(dst, src):
    dst.copy_(src.contiguous().reshape(-1).view(dst.dtype))


def tables_digest(tables):
    """SHA-256 (16 hex) of a rank's own tables in TableGather order."""
    import hashlib
    h = hashlib.sha256()
    for t in tables:
        h.update(t.cpu().contiguous().numpy().tobytes())
    return h.hexdigest()[:16]


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
