"""Multi-process path of the bench (plvi.dist) with the gloo backend on CPU,
world size 2: rank-sharded frame sequences (no data-path collective), the
max-over-ranks wall time and the whole-job frame count."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    from plvi import dist as pdist
    from plvi import synth
    w, r, _ = pdist.env()
    pdist.init("gloo")
    frames = synth.batch(2, 64, 48, seed0=pdist.shard_seed(r))
    pdist.barrier(w)
    el = pdist.max_over_ranks(0.5 + r, w)
    total = pdist.sum_over_ranks(frames.shape[0], w)
    import torch
    counts = torch.tensor([10 * r + 1, 10 * r + 2], dtype=torch.int32)
    desc = torch.full((2, 5, 32), r + 7, dtype=torch.uint8)
    gc, gd = pdist.gather_tables([counts, desc], w)
    ok = (gc.tolist() == [[1, 2], [11, 12]] and gd.shape == (2, 2, 5, 32) and int(gd[0].max()) == 7
          and int(gd[1].min()) == 8)
    # bench.py's timed C4 gather (plvi.dist.TableGather): staged per-frame
    # tables of several steps gathered to rank 0, rank-major, the last step's
    # tables intact after the earlier gathers completed
    tabs = lambda s: (torch.tensor([s, 100 * r + s], dtype=torch.int32),  # noqa: E731
                      torch.full((3, 28), 16 * r + s, dtype=torch.uint8),
                      torch.arange(64, dtype=torch.uint8) + r)
    tg = pdist.TableGather([8, 84, 64], w, r)
    for s in range(3):
        tg.post(tabs(s))
    tg.wait()
    if r == 0:
        got = [[t.clone() for t in tg.received(k)] for k in range(w)]
        ok = ok and tg.posted == 3
        for k in range(w):
            ok = ok and got[k][0].view(torch.int32).tolist() == [2, 100 * k + 2]
            ok = ok and bool((got[k][1] == 16 * k + 2).all()) and got[k][2].tolist() == list(range(k, 64 + k))
        ok = ok and len(set(tg.digests())) == 2
    q.put((r, el, total, int(frames.astype(np.int64).sum()), ok))
    import torch.distributed as dist
    dist.destroy_process_group()


def test_gloo_world2_sharding_and_max_time():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [o[1] for o in out] == [1.5, 1.5]       # slowest rank's time on every rank
    assert [o[2] for o in out] == [4, 4]           # whole-job frame count
    assert out[0][3] != out[1][3]                  # each rank owns different frames
    assert all(o[4] for o in out)                  # per-frame tables gathered rank-major on every rank


def _bench(*a, timeout=300):
    import json
    import subprocess
    import sys
    from conftest import ROOT
    env = {k: v for k, v in __import__("os").environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *a], capture_output=True, text=True, timeout=timeout,
                       env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_gpus_n_launches_n_ranks():
    """`bench.py --gpus 2` starts 2 ranks itself (torch.distributed.run child)
    and reports n_gpus from the actual world size; the max-time and
    sum-frames reductions cover both ranks, each with its own sequence."""
    out = _bench("--gpus", "2", "--dry-run", "--batch", "3", "--steps", "2", "--width", "64", "--height", "48")
    assert out["n_gpus"] == 2 and out["frames_total"] == 2 * 2 * 3
    d = out["rank_digests"]
    assert len(d) == 2 and d[0] != d[1]
    # the default (non-C4) multi-rank run gathers every step's per-frame
    # tables to rank 0 too (north_star: RCCL gather of the descriptor tables)
    g = out["gather"]
    assert g is not None and g["posts"] == 2
    assert g["received"] == g["rank_tables"] and g["rank_tables"][0] != g["rank_tables"][1]


def test_bench_no_gather_opt_out():
    out = _bench("--gpus", "2", "--dry-run", "--no-gather", "--batch", "3", "--steps", "2", "--width", "64",
                 "--height", "48")
    assert out["gather"] is None


def test_bench_c4_dry_run_world2():
    """--c4: 752x480 windows with a one-frame halo (B-1 new frames per step)."""
    out = _bench("--gpus", "2", "--dry-run", "--c4", "--batch", "3", "--steps", "3")
    assert out["n_gpus"] == 2 and out["config"]["width"] == 752 and out["frames_total"] == 2 * 3 * 2
    # the dry run drives bench.py's TableGather every step (on by default for
    # --c4 at world > 1): rank 0 received each rank's own last-step tables
    g = out["gather"]
    assert g["posts"] == 3 and g["received"] == g["rank_tables"] and g["rank_tables"][0] != g["rank_tables"][1]


def test_bench_refuses_world_mismatch():
    import os
    import subprocess
    import sys
    from conftest import ROOT
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "4", "--dry-run"], capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
