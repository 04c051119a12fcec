"""bench.py — throughput of the MI355X feature front end (BASELINE.json metric).

A step = one pass of the hot path over one batch of B synthetic frames
already resident in HBM (default B = 3072 frames in flight per GPU):
  ORB extract (ORBextractor 1000/1.2/8/20/7) and LSD + LBD line extract
  (Lineextractor 200/0/0.8/2/2.0) as one schedule (plvi_frame_extract_batch:
  region growing concurrent with the ORB pipeline and the LBD Sobel pyramid),
  then matching of every frame against the previous one (B-1 pairs):
  ORB Hamming kNN-2 (~1000x1000) and LineMatcher::match (kNN-2 both ways,
  ratio 0.9, mutual check).
value = frames processed by all ranks / max-over-ranks wall time.

Launch: `python bench.py --gpus N` with N > 1 starts N ranks itself (a
torch.distributed.run child, before anything touches the GPU) unless it is
already running under torchrun, in which case WORLD_SIZE must equal N.  One
process per GPU; each rank owns its own synthetic sequence (seeds
rank*10^6 + t) -- no data-path collective, scaling "weak".
--c4: BASELINE config C4 -- 752x480 EuRoC-shaped frames, each rank walks its
own sequence in consecutive overlapping windows (one-frame halo, so every
consecutive pair is matched once), and every step's per-frame tables are
gathered to rank 0 over RCCL (on by default for world > 1).

Outside the timed region: the device error flags of every batch are checked
(any overflow fails the run), frames 0, B/2 and B-1 of the timed batch (and
their matches) are compared bit-exactly with the CPU oracle, and on rank 0
at N=1 the oracle is timed as the CPU baseline.  Also reported:
the rooflines of the two HBM passes (orb_blur_fast_kernel, lsd_prep_kernel;
HIP events on the launch streams) and the end-to-end HBM fraction, a
batch-64 line (C1/C2), the single-frame latency of the drop-in entry points
run as Frame runs them, and an overlapped pinned-H2D variant of the step.
"""
import argparse
import ctypes
import hashlib
import json
import os
import pathlib
import socket
import subprocess
import sys
import time
import types

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
sys.path.insert(0, str(ROOT / "tests"))

METRIC = "frames/sec ORB+LSD extract+match, 640×480 mono, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
E2E_BYTES_640 = 15_972_194  # reference-materialisation bytes per 640x480 frame
E2E_BYTES_752 = 18_775_975


def level_dims(w, h, nlevels=8, sf=1.2):
    scale = [1.0]
    for i in range(1, nlevels):
        scale.append(float(np.float32(np.float64(np.float32(scale[-1])) * np.float64(np.float32(sf)))))
    dims = []
    for s in scale:
        inv = np.float32(1.0) / np.float32(s)
        dims.append((int(np.rint(np.float32(w) * inv)), int(np.rint(np.float32(h) * inv))))
    return dims


def blur_fast_bytes(w, h):
    """SURVEY 8(d) algorithmic bytes/frame of the ORB blur + FAST pass (the
    roofline numerator): 7x7 blur of every level (read + write, 1 901 064 B at
    640x480) + FAST scoring read of every level (950 532 B) = 2 851 596 B."""
    planes = [a * b for a, b in level_dims(w, h)]
    return 3 * sum(planes)


def pyramid_bytes(w, h):
    """SURVEY 8(d) algorithmic bytes/frame of the ORB resize pass
    (ComputePyramid, orb_pyramid_kernel): level l >= 1 reads level l-1 and
    writes level l once = 1 569 878 B at 640x480."""
    planes = [a * b for a, b in level_dims(w, h)]
    return sum(planes[:-1]) + sum(planes[1:])


def blur_fast_kernel_bytes(w, h, copy0=False):
    """What orb_blur_fast_kernel itself materialises per frame (reported next
    to the SURVEY model, not used for frac): every level read once, its blur
    and FAST score planes written once, and -- only when the frames' rows are
    not packed (copy0) -- level 0's pyramid copy (u8).  Since r06 level 0 of
    packed frames is a view of the frame (the bench's case): the kernel's
    bytes are then the SURVEY model's."""
    planes = [a * b for a, b in level_dims(w, h)]
    return sum(planes) + 2 * sum(planes) + (planes[0] if copy0 else 0)


def lsd_prep_bytes(w, h, scale=0.8, noct=2):
    """Algorithmic bytes/frame of lsd_prep_kernel (one launch per octave): the
    octave's u8 image in; out per scaled pixel the f32 angle, the f64 modgrad
    and the float2 cos/sin pair region growing reads (20 B)."""
    tot = 0
    for o in range(noct):
        ow, oh = w >> o, h >> o
        sw, sh = int(np.rint(ow * scale)), int(np.rint(oh * scale))
        tot += ow * oh + 20 * sw * sh
    return tot


def lbd_sobel_bytes(w, h):
    """SURVEY 8(d) LBD bytes/frame (2 918 400 at 640x480) split over the two
    kernels that materialise them: lbd_sobel0_kernel = octave-0 5x5 blur
    (read + write) + Sobel of it (u8 in, two int16 planes out: 5 B/px) =
    2 150 400 B; lbd_sobel1_kernel = pyrDown (octave-0 blur read, quarter
    write) + Sobel of octave 1 = 768 000 B."""
    p0 = w * h
    p1 = (w // 2) * (h // 2)
    return (2 * p0 + 5 * p0, p0 + p1 + 5 * p1)


def committed_traffic(batch, kernel):
    """HBM bytes per launch of `kernel` from the committed PMC passes
    (profiles/*/pmc_traffic*.json, tools/pmc_traffic.py), taken at this batch
    size; else None.  Entries before r03 held lsd_prep_kernel's per-batch sum
    of its two octave launches: halved to a per-launch mean."""
    best = None
    for f in sorted(ROOT.glob("profiles/*/pmc_traffic*.json")):
        try:
            d = json.loads(f.read_text())
        except ValueError:
            continue
        for e in d if isinstance(d, list) else [d]:
            if e.get("batch") == batch and e.get("kernel") == kernel:
                best = e
    if best is None:
        return None
    v = best["bytes_per_launch"]
    if best.get("unit") != "bytes per launch" and kernel == "lsd_prep_kernel":
        v /= 2
    return v


def committed_pmc(batch, kernel, field):
    """A per-launch PMC field (e.g. valu_insts_per_launch) of `kernel` from the
    committed passes (profiles/*/pmc_traffic*.json), taken at this batch size."""
    best = None
    for f in sorted(ROOT.glob("profiles/*/pmc_traffic*.json")):
        try:
            d = json.loads(f.read_text())
        except ValueError:
            continue
        for e in d if isinstance(d, list) else [d]:
            if e.get("batch") == batch and e.get("kernel") == kernel and field in e:
                best = e[field]
    return best


# VALU issue peak: 256 CUs x 4 SIMDs, a wave64 VALU instruction issues over 2
# cycles on a SIMD-32 (MI355X_MICROARCH.md, execution model), 2.4 GHz
VALU_PEAK_WIPS = 256 * 4 * 2.4e9 / 2


def valu_roof(batch, kernel, ms_timed, ms_iso):
    """roofline.valu: the kernel's VALU wave-instructions per launch (committed
    PMC pass) / launch duration / the chip's VALU issue peak."""
    n = committed_pmc(batch, kernel, "valu_insts_per_launch")
    if not n:
        return None
    r = {"insts_per_launch": n, "peak": VALU_PEAK_WIPS, "unit": "wave-instructions/s",
         "source": "SQ_INSTS_VALU, tools/gpu_traffic.sh pass 3 (profiles/*/pmc_traffic.json)"}
    if ms_timed:
        r["achieved"] = n / (ms_timed * 1e-3)
        r["frac"] = r["achieved"] / VALU_PEAK_WIPS
    if ms_iso:
        r["isolated_frac"] = n / (ms_iso * 1e-3) / VALU_PEAK_WIPS
    return r


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n):
    """`bench.py --gpus N` outside torchrun: start the N ranks as a
    torch.distributed.run child (nothing in this process has touched the
    GPU) and exit with its status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", str(pathlib.Path(__file__).resolve())]
    cmd += sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


# ------------------------------------------------------------------ oracle leg
# The only part of bench.py that loads the CPU oracle (oracle/, test
# infrastructure): as the checker of the timed batch and as the timed CPU
# baseline.  Never on the measured GPU path.
def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def oracle_verify(checks):
    """Bit-exact comparison of downloaded GPU outputs with the oracle.
    checks: list of (kind, inputs, gpu_outputs).  Returns a list of failures."""
    import oracle_lib as ol
    bad = []
    for kind, inp, got in checks:
        if kind == "orb":
            m, k, d = ol.orb_extract(inp)
            ok = got[0] == m and got[1].tobytes() == k.tobytes() and np.array_equal(got[2], d)
        elif kind == "lines":
            k, d, f = ol.line_extract(inp)
            ok = got[0].tobytes() == k.tobytes() and np.array_equal(got[1], d) and got[2].tobytes() == f.tobytes()
        elif kind == "knn2":
            e = ol.knn2(*inp)
            ok = all(np.array_equal(g, x) for g, x in zip(got, e))
        elif kind == "lmatch":
            n, m = ol.match(inp[0], inp[1], 0.9)
            ok = got[0] == n and np.array_equal(got[1], m)
        else:
            ok = False
        if not ok:
            bad.append(kind)
    return bad


def cpu_baseline(frames, runs=5, par_s=5.0):
    """the oracle restatement timed on this box's host cores, in
    a child process (`bench.py --cpu-baseline-child`, no GPU) so that no host
    thread of the GPU process competes with it.  The oracle is rebuilt here
    with -O3 -march=native (MARCH=-march=native, into a temp dir; the
    checker's own build stays -march=x86-64-v3); on a build failure the
    checker's build is timed and the line says so."""
    import tempfile
    tmp = pathlib.Path(tempfile.mkdtemp(prefix="plvi_cpu_"))
    lib = tmp / "liboracle.so"
    march = "native"
    r = subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "MARCH=-march=native", f"OUT={lib}"],
                       capture_output=True, text=True)
    env = dict(os.environ)
    if r.returncode == 0 and lib.exists():
        env["ORACLE_LIB"] = str(lib)
    else:
        march = "x86-64-v3 (native build failed)"
    np.save(tmp / "frames.npy", np.stack(frames))
    out = tmp / "cpu.json"
    r = subprocess.run([sys.executable, str(pathlib.Path(__file__).resolve()), "--cpu-baseline-child",
                        str(tmp / "frames.npy"), str(out), str(runs), str(par_s)], env=env, capture_output=True,
                       text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(f"cpu baseline child failed: {r.stderr[-2000:]}")
    res = json.loads(out.read_text())
    res["build"] = f"oracle/ -O3 -march={march} -ffp-contract=off"
    return res


def cgroup_cpu_quota():
    """CPUs granted by the cgroup CPU quota (ceil(quota / period)), or None
    when unlimited / unreadable.  cgroup v2: the tightest `cpu.max` on the
    path from this process's cgroup (/proc/self/cgroup) up to the root;
    cgroup v1: the cfs quota files."""
    import math
    best = None
    try:
        rel = ""
        for line in pathlib.Path("/proc/self/cgroup").read_text().splitlines():
            if line.startswith("0::"):
                rel = line[3:].strip().strip("/")
        d = pathlib.Path("/sys/fs/cgroup") / rel
        while True:
            f = d / "cpu.max"
            if f.exists():
                q, per = f.read_text().split()[:2]
                if q != "max":
                    n = max(1, math.ceil(int(q) / int(per)))
                    best = n if best is None else min(best, n)
            if d == pathlib.Path("/sys/fs/cgroup") or d == d.parent:
                break
            d = d.parent
    except (OSError, ValueError):
        pass
    if best is not None:
        return best
    try:
        q = int(pathlib.Path("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read_text())
        per = int(pathlib.Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
        return None if q <= 0 else max(1, math.ceil(q / per))
    except (OSError, ValueError):
        return None


def cpu_baseline_child(frames_npy, out_json, runs, par_s):
    """The CPU-baseline measurement proper (child process, no GPU): per stage
    and end to end on the timed batch's frames, single thread pinned to one
    core (median of `runs`); frame-parallel throughput on every core this
    process may use; and BASELINE C0 (752x480 EuRoC-shaped frames, ORB 1000 +
    LineExtractor 100 lines, extraction only, single thread)."""
    import threading
    import oracle_lib as ol
    from plvi import synth
    ol.load()
    frames = list(np.load(frames_npy))
    cpus = sorted(os.sched_getaffinity(0))
    stages = ("orb_extract", "line_extract", "orb_knn2", "line_match")
    per = {k: [] for k in stages}
    tot = []
    os.sched_setaffinity(0, {cpus[0]})
    try:
        for _ in range(runs):
            acc = dict.fromkeys(stages, 0.0)
            prev = None
            t_run = time.perf_counter()
            for img in frames:
                t0 = time.perf_counter()
                _, _, d = ol.orb_extract(img)
                t1 = time.perf_counter()
                _, ld, _ = ol.line_extract(img)
                t2 = time.perf_counter()
                if prev is not None:
                    ol.knn2(d, prev[0])
                    t3 = time.perf_counter()
                    if len(ld) >= 2 and len(prev[1]) >= 2:
                        ol.match(ld, prev[1], 0.9)
                    t4 = time.perf_counter()
                    acc["orb_knn2"] += t3 - t2
                    acc["line_match"] += t4 - t3
                acc["orb_extract"] += t1 - t0
                acc["line_extract"] += t2 - t1
                prev = (d, ld)
            tot.append(time.perf_counter() - t_run)
            for k in stages:
                per[k].append(acc[k] * 1e3 / len(frames))
        # BASELINE C0 as named (640x480, 1000 ORB features, 100 lines,
        # extraction only), and the EuRoC frame shape (752x480) beside it
        c0s = {}
        for (cw, chh) in ((640, 480), (752, 480)):
            c0 = synth.device_sequence(16, cw, chh, seed=7).numpy()
            c0t = []
            for _ in range(3):
                t0 = time.perf_counter()
                for img in c0:
                    ol.orb_extract(img)
                    ol.line_extract(img, nfeatures=100)
                c0t.append(time.perf_counter() - t0)
            c0s[(cw, chh)] = (len(c0), float(np.median(c0t)))
    finally:
        os.sched_setaffinity(0, set(cpus))
    med = float(np.median(tot))
    quota = cgroup_cpu_quota()
    # frame-parallel leg: one thread per CPU the job may actually run on --
    # the affinity set capped by the cgroup CPU quota (a GPU job on the box
    # sees every CPU of the host but is granted far fewer).  Without a
    # readable quota the job's declared CPU share (OMP_NUM_THREADS, which the
    # GPU box sets to its per-GPU share) caps it instead.
    share = quota
    share_src = "cgroup cpu.max"
    if not share and os.environ.get("OMP_NUM_THREADS", "").isdigit():
        share, share_src = int(os.environ["OMP_NUM_THREADS"]), "OMP_NUM_THREADS (no cgroup quota)"
    nthr = max(1, min(len(cpus), share if share else len(cpus)))
    count = [0] * nthr
    stop = time.perf_counter() + par_s

    def worker(i):
        prev = None
        j = i
        while time.perf_counter() < stop:
            img = frames[j % len(frames)]
            _, _, d = ol.orb_extract(img)
            _, ld, _ = ol.line_extract(img)
            if prev is not None:
                ol.knn2(d, prev[0])
                if len(ld) >= 2 and len(prev[1]) >= 2:
                    ol.match(ld, prev[1], 0.9)
            prev = (d, ld)
            count[i] += 1
            j += nthr
    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker, args=(i,)) for i in range(nthr)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    par_fps = sum(count) / (time.perf_counter() - t0)
    res = {"value": len(frames) / med, "unit": "frames/s", "cores": 1, "kind": "port",
           "sample": f"{len(frames)} frames of the timed batch (640x480), median of {runs} single-thread runs "
                     f"pinned to core {cpus[0]} (sched_setaffinity): ORB extract + LSD/LBD extract + ORB kNN-2 + "
                     f"LineMatcher::match vs previous frame, CPU restatement (oracle/)",
           "stage_ms_per_frame": {k: round(float(np.median(v)), 3) for k, v in per.items()},
           "parallel": {"threads": nthr, "cores": nthr, "value": round(par_fps, 2), "unit": "frames/s",
                        "sample": f"{sum(count)} frames in {par_s:.0f}s, one frame-parallel thread per CPU the "
                                  f"job may use: min(affinity set {len(cpus)}, {share_src} "
                                  f"{share if share else 'none'}) = {nthr}"},
           "c0_640x480": {"value": round(c0s[(640, 480)][0] / c0s[(640, 480)][1], 3), "unit": "frames/s",
                          "cores": 1,
                          "sample": f"BASELINE configs[0] as named: {c0s[(640, 480)][0]} synthetic 640x480 frames, "
                                    "ORBextractor 1000 + Lineextractor 100 lines, extraction only, median of 3 "
                                    "single-thread runs"},
           "c0_752x480": {"value": round(c0s[(752, 480)][0] / c0s[(752, 480)][1], 3), "unit": "frames/s",
                          "cores": 1,
                          "sample": f"EuRoC frame shape: {c0s[(752, 480)][0]} synthetic 752x480 frames, "
                                    "ORBextractor 1000 + Lineextractor 100 lines, extraction only, median of 3 "
                                    "single-thread runs"},
           "host_cpu": _cpu_model(), "host_nproc": os.cpu_count(), "affinity_cpus": len(cpus),
           "cgroup_cpu_quota": quota}
    pathlib.Path(out_json).write_text(json.dumps(res))
    return 0


# ------------------------------------------------------------------ dry run
def dry_run(args, world, rank):
    """--dry-run: the launcher and the reductions without the GPU (gloo):
    each rank builds its own sequence on the CPU, "processes" it with a
    numpy checksum per frame, and the run reports the max-over-ranks time,
    the whole-job frame count and every rank's first-batch digest."""
    import torch
    from plvi import dist as pdist
    from plvi import synth
    if world > 1:
        pdist.init("gloo")
    W, H = (752, 480) if args.c4 else (args.width, args.height)
    B = args.batch
    nwin = 2 if args.c4 else max(1, args.inflight)  # the GPU run's windows (run())
    wstride = (B - 1) if args.c4 else B
    seq = synth.device_sequence(B + (nwin - 1) * wstride, W, H, seed=pdist.shard_seed(rank))
    digest = hashlib.sha256(seq[:B].numpy().tobytes()).hexdigest()[:16]
    gather = world > 1 if args.gather is None else args.gather

    def tables(lo):
        # stand-ins for the per-frame tables (counts, keypoints, descriptors,
        # line counts, keylines, LBD descriptors): fixed-capacity byte tables
        # derived from the window's frames, the shapes TableGather sees on a GPU
        win = seq[lo:lo + B]
        flat = win.reshape(B, -1)
        cnt = flat[:, :64].to(torch.int32).sum(1).to(torch.int32)
        return (cnt, flat[:, :28 * 4].contiguous(), flat[:, -32 * 4:].contiguous(), cnt + 1,
                flat[:, 1000:1000 + 68 * 2].contiguous(), flat[:, 2000:2000 + 32 * 2].contiguous())
    tg = None
    if gather:
        tg = pdist.TableGather([t.numel() * t.element_size() for t in tables(0)], world, rank)
    pdist.barrier(world)
    t0 = time.perf_counter()
    sums = 0
    for k in range(args.steps):
        lo = (k % nwin) * wstride
        sums += int(seq[lo:lo + B].to(torch.int64).sum())
        if tg is not None:
            tg.post(tables(lo))
    if tg is not None:
        tg.wait()
    el = pdist.max_over_ranks(time.perf_counter() - t0, world)
    new = (B - 1) if args.c4 else B
    total = pdist.sum_over_ranks(new * args.steps, world)
    digests = [digest]
    if world > 1:
        import torch.distributed as dist
        digests = [None] * world
        dist.all_gather_object(digests, digest)
    gathered = None
    if tg is not None:
        # the last step's tables of every rank, as rank 0 received them, next
        # to each rank's own digest of the same tables
        own = pdist.tables_digest(tables(((args.steps - 1) % nwin) * wstride))
        owns = [own]
        if world > 1:
            owns = [None] * world
            dist.all_gather_object(owns, own)
        gathered = {"posts": tg.posted, "rank_tables": owns,
                    "received": tg.digests() if rank == 0 else None}
    if rank == 0:
        print(json.dumps({"metric": METRIC, "dry_run": True, "n_gpus": world, "steps": args.steps,
                          "frames_total": total, "max_rank_s": el, "rank_digests": digests,
                          "gather": gathered,
                          "config": {"batch": B, "width": W, "height": H, "c4": bool(args.c4)}}), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


# ------------------------------------------------------------------ main
# The frame schedule's environment knobs (csrc/lines_pipeline.hip init(),
# csrc/orb_pipeline.hip) and the batch-size rules they select, recorded in the
# bench line so numbers from different schedules are not compared as like for
# like (r04 moved --inflight from 1 to 2 and made the ORB start depend on the
# batch size).
SCHEDULE_ENV = ("PLVI_STREAM_PRIO", "PLVI_ORB_AFTER_PREP", "PLVI_GROW_AFTER_BLUR", "PLVI_ORB_PRIO",
                "PLVI_SOBEL_WITH_GROW", "PLVI_SOBEL_GATE", "PLVI_SOBEL_AFTER_GROW", "PLVI_GROW_SPLIT", "PLVI_GROW_LDS",
                "PLVI_GROW_RB", "PLVI_GROW_RD", "PLVI_GROW_MW", "PLVI_GROW_GATE", "PLVI_ORB_STREAM_PRIO")


def schedule_knobs(batch):
    env = {k: os.environ[k] for k in SCHEDULE_ENV if k in os.environ}
    after_prep = int(os.environ.get("PLVI_ORB_AFTER_PREP", "2"))
    big = batch >= 1024
    return {"env": env,
            "orb_waits_for_lsd_prep": after_prep >= 2 or (after_prep == 1 and batch < 1024),
            "growth_waits_for_blur_fast": os.environ.get("PLVI_GROW_AFTER_BLUR", "1") != "0" and big,
            "sobel_after_growth": os.environ.get("PLVI_SOBEL_AFTER_GROW", "0") != "0" and
            os.environ.get("PLVI_GROW_AFTER_BLUR", "1") != "0" and big}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None, help="frames per step (default 3072; C4: 2000)")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--c4", action="store_true", help="BASELINE C4: 752x480 sequences, RCCL gather to rank 0")
    ap.add_argument("--gather", dest="gather", action="store_true", default=None,
                    help="gather every step's per-frame tables to rank 0 over RCCL (timed; default: on whenever "
                         "world > 1, the north_star's gather of the descriptor tables)")
    ap.add_argument("--no-gather", dest="gather", action="store_false")
    ap.add_argument("--dry-run", action="store_true", help="launcher + reductions on CPU (gloo), no GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=64, help="frames of the CPU-baseline sample (SURVEY 8(d): 64)")
    ap.add_argument("--cpu-baseline-child", nargs=4, metavar=("FRAMES_NPY", "OUT_JSON", "RUNS", "PAR_S"),
                    help=argparse.SUPPRESS)
    ap.add_argument("--no-check", action="store_true", help="skip the oracle check of the timed batch")
    ap.add_argument("--no-extra", action="store_true", help="skip the batch-64 / latency / H2D lines")
    ap.add_argument("--no-side", action="store_true", help="skip the BoW / projection / stereo stage timings")
    ap.add_argument("--inflight", type=int, default=2,
                    help="batches in flight: consecutive steps alternate over this many extractor/stream slots, "
                         "so one batch's ORB tail overlaps the next batch's LSD front")
    args = ap.parse_args()

    if args.cpu_baseline_child:
        f, o, runs, par_s = args.cpu_baseline_child
        return cpu_baseline_child(f, o, int(runs), float(par_s))
    world_env = int(os.environ.get("WORLD_SIZE", "0"))
    if world_env == 0 and args.gpus > 1:
        return spawn_ranks(args.gpus)
    world = max(world_env, 1)
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if args.batch is None:
        args.batch = 2000 if args.c4 else 3072
    if args.batch < 2:
        print("bench.py: --batch must be >= 2 (frames are matched against their predecessor)", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)
    if args.c4:
        args.width, args.height = 752, 480
    if args.gather is None:
        args.gather = world > 1
    return run(args, world, rank)


def run(args, world, rank):
    import torch
    import plvi
    from plvi import dist as pdist
    from plvi import synth

    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        pdist.init("nccl", torch.device("cuda", local))
    dev = torch.cuda.current_device()
    cuda = f"cuda:{dev}"
    B, W, H = args.batch, args.width, args.height
    i32 = dict(dtype=torch.int32, device=cuda)
    lib = plvi.load()
    seed0 = pdist.shard_seed(rank)

    # frames: C4 = one sequence per rank walked in windows [k(B-1), k(B-1)+B)
    # (one-frame halo; two windows per sequence, ~2B frames; the walk wraps to
    # the start); default = one resident batch of B distinct frames per batch
    # in flight (consecutive windows [kB, kB+B) of one sequence), so the
    # batches in flight never process the same frames
    nwin = 2 if args.c4 else max(1, args.inflight)
    wstride = (B - 1) if args.c4 else B
    seq = synth.device_sequence(B + (nwin - 1) * wstride, W, H, seed=seed0, device=cuda)
    torch.cuda.synchronize()
    first_digest = hashlib.sha256(seq[:B].cpu().numpy().tobytes()).hexdigest()[:16]

    # Slots: an ORB + line extractor pair with its own output tables, match
    # buffers and stream.  Step k runs on slot k % inflight, so batch k+1's
    # LSD front (prep, region growing) overlaps batch k's ORB tail.  Every step
    # still extracts and matches its full batch inside the timed region.
    tab_sizes = None

    def make_slot():
        nonlocal tab_sizes
        sl = types.SimpleNamespace()
        sl.orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=B, device=dev)
        sl.lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=B, device=dev)
        sl.kp_p, sl.de_p, sl.co_p, _, cap_ = sl.orb.outputs()
        sl.kl_p, sl.lde_p, _, sl.lco_p, lcap_ = sl.lx.outputs()
        sl.outs = [torch.empty((B - 1) * cap_, **i32) for _ in range(4)]
        sl.lscratch = torch.empty(4 * (B - 1) * 2 * lcap_, **i32)
        sl.lm12 = torch.empty((B - 1) * lcap_, **i32)
        sl.lnm = torch.empty(B - 1, **i32)
        sl.stream = torch.cuda.Stream()  # non-default: the legacy null stream would serialise
        sl.st = sl.stream.cuda_stream
        # C4 gather (plvi.dist.TableGather): tables staged on the slot's stream,
        # then one asynchronous RCCL gather per table to rank 0 (waited on
        # before the slot's staging is reused)
        tab_sizes = (4 * B, 28 * cap_ * B, 32 * cap_ * B, 4 * B, 68 * lcap_ * B, 32 * lcap_ * B)
        sl.tables = (sl.co_p, sl.kp_p, sl.de_p, sl.lco_p, sl.kl_p, sl.lde_p)
        sl.tg = None
        if args.gather:
            def dev_copy(t, src, st_=sl.st):
                if lib.plvi_memcpy_async(t.data_ptr(), src, t.numel(), 3, st_):
                    raise RuntimeError("gather copy")
            sl.tg = pdist.TableGather(tab_sizes, world, rank, device=cuda, copy=dev_copy)
        return sl, cap_, lcap_

    s0, cap, lcap = make_slot()
    slots = [s0] + [make_slot()[0] for _ in range(max(1, args.inflight) - 1)]
    # the single-frame (drop-in) handles are created here, next to the main
    # ones, as a SLAM process creates its extractors once at start-up: the
    # runtime maps each new stream to the least-used of its few hardware
    # queues, so handles created after many others were destroyed can land
    # on one queue and serialise ORB || lines
    lat_handles = None
    if rank == 0 and world == 1 and not args.no_extra:
        # (and the batch-64 line's pair and its stream, for the same reason)
        lat_handles = (plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, device=dev),
                       plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, device=dev),
                       plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=64, device=dev),
                       plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=64, device=dev),
                       torch.cuda.Stream())
    orb, lx, stream, st = s0.orb, s0.lx, s0.stream, s0.st
    kp_p, de_p, co_p, kl_p, lde_p, lco_p = s0.kp_p, s0.de_p, s0.co_p, s0.kl_p, s0.lde_p, s0.lco_p
    outs, lscratch, lm12, lnm = s0.outs, s0.lscratch, s0.lm12, s0.lnm
    for sl in slots:
        sl.orb.kernel_timing(True)  # event pair around every blur+FAST launch
        sl.lx.kernel_timing(True)   # and every lsd_prep launch

    def extract(fptr, n=B, sl=s0):
        plvi.frame_extract_batch(sl.orb, sl.lx, fptr, n, W * H, W, (0, 0), stream=sl.st)

    def match(n=B, sl=s0):
        rc = lib.plvi_hamming_knn2_batch(sl.de_p + cap * 32, sl.co_p + 4, cap, sl.de_p, sl.co_p, cap, n - 1,
                                         *[o.data_ptr() for o in sl.outs], sl.st)
        rc |= lib.plvi_line_match_batch(sl.lde_p + lcap * 32, sl.lco_p + 4, lcap, sl.lde_p, sl.lco_p, lcap, n - 1,
                                        0.9, sl.lscratch.data_ptr(), sl.lm12.data_ptr(), sl.lnm.data_ptr(), sl.st)
        if rc:
            raise RuntimeError(f"match {rc}")

    def gather(sl=s0):
        sl.tg.post(sl.tables, stream=sl.stream)

    def wait_gathers():
        for sl in slots:
            sl.tg.wait()

    step_no = [0]

    def fused(sl, fptr):
        # extract + match as one schedule (plvi_frame_extract_match_batch: the
        # matching issued on the schedule's own streams, same kernels and
        # tables as extract() + match())
        plvi.frame_extract_match_batch(sl.orb, sl.lx, fptr, B, W * H, W,
                                       [o.data_ptr() for o in sl.outs], 0.9, sl.lscratch.data_ptr(),
                                       sl.lm12.data_ptr(), sl.lnm.data_ptr(), stream=sl.st)

    def step():
        k = step_no[0]
        step_no[0] += 1
        sl = slots[k % len(slots)]
        lo = (k % nwin) * wstride
        fused(sl, seq[lo].data_ptr())
        if args.gather:
            gather(sl)

    for _ in range(max(args.warmup, len(slots))):
        step()
    torch.cuda.synchronize()
    if args.gather and world > 1:
        wait_gathers()
        torch.cuda.synchronize()
    # error flags of the warm-up batches
    err_warm = [0, 0]
    for sl in slots:
        err_warm[0] |= sl.orb.errors(sl.st)
        err_warm[1] |= sl.lx.errors(sl.st)

    # stage timing (separate from the timed region: events add markers); each
    # extractor alone so its stage times are uncontended
    f0 = seq.data_ptr()
    orb.profile(True)
    lx.profile(True)
    lx.kernel_timing(True)  # isolated per-launch times of the LBD Gaussian + Sobel kernels
    orb.kernel_timing(True)  # and of blur + FAST (the roofline kernel) with nothing beside it
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    match_ms = 0.0
    nprof = max(3, min(args.steps, 10))
    for _ in range(nprof):
        orb.extract_batch(f0, B, W * H, W, (0, 0), stream=st)
        torch.cuda.synchronize()
        lx.extract_batch(f0, B, W * H, W, stream=st)
        torch.cuda.synchronize()
        ev0.record(stream)
        match()
        ev1.record(stream)
        torch.cuda.synchronize()
        match_ms += ev0.elapsed_time(ev1)
    st_orb, runs = orb.profile_read()
    st_lines, lruns = lx.profile_read()
    lbd_iso = [lx.kernel_timing_read(k) for k in (1, 2)]
    bf_iso = orb.kernel_timing_read()
    pyr_iso = orb.kernel_timing_read(1)
    orb.kernel_timing(False)
    lx.kernel_timing(False)
    orb.profile(False)
    lx.profile(False)

    def part_fps(fn):
        fn()
        torch.cuda.synchronize()
        ev0.record(stream)
        for _ in range(nprof):
            fn()
        ev1.record(stream)
        torch.cuda.synchronize()
        return B * nprof / (ev0.elapsed_time(ev1) * 1e-3)
    parts = {"orb_only": part_fps(lambda: orb.extract_batch(f0, B, W * H, W, (0, 0), stream=st)),
             "lines_only": part_fps(lambda: lx.extract_batch(f0, B, W * H, W, stream=st)),
             "match_only": part_fps(match)}
    stage_ms = {f"orb.{k}": v / runs for k, v in st_orb.items()}
    stage_ms.update({f"lines.{k}": v / lruns for k, v in st_lines.items()})
    stage_ms["match"] = match_ms / nprof
    side = {}
    if not args.no_side and world == 1:
        side = side_stages(args, torch, plvi, synth, lib, orb, st, stream, B, W, H, cap, kp_p, de_p, co_p, nprof,
                           cuda, seed0)

    # ---------------------------------------------------------- timed region
    # the roofline events cover exactly the timed launches; a spin_kernel on
    # each side marks the same window in a rocprofv3 kernel trace
    # (tools/timed_stats.py)
    for sl in slots:
        sl.orb.kernel_timing(True)
        sl.lx.kernel_timing(True)
    torch.cuda._sleep(1000)
    pdist.barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if args.gather and world > 1:
        wait_gathers()
    torch.cuda.synchronize()
    pdist.barrier(world)
    el = pdist.max_over_ranks(time.perf_counter() - t0, world, cuda)
    torch.cuda._sleep(1000)

    new_frames = (B - 1) if args.c4 else B
    frames_total = new_frames * args.steps * world
    value = frames_total / el
    ms_step = el / args.steps * 1e3
    err = list(err_warm)
    ktot = kn = ltot = ln = ptot = pn = 0
    sob = [[0.0, 0], [0.0, 0]]  # LBD Gaussian + Sobel kernels: [total ms, launches] of octave 0 / 1
    for sl in slots:
        err[0] |= sl.orb.errors(sl.st)
        err[1] |= sl.lx.errors(sl.st)
        a, b = sl.orb.kernel_timing_read()
        c, d = sl.lx.kernel_timing_read()
        p_, q_ = sl.orb.kernel_timing_read(1)
        ktot, kn, ltot, ln, ptot, pn = ktot + a, kn + b, ltot + c, ln + d, ptot + p_, pn + q_
        for k in (0, 1):
            t_, n_ = sl.lx.kernel_timing_read(k + 1)
            sob[k][0] += t_
            sob[k][1] += n_
    # last timed batch's window (for the checks below)
    lo_last = ((step_no[0] - 1) % nwin) * wstride

    # ---------------------------------------------------------- rooflines
    bf_bytes = blur_fast_bytes(W, H) * B
    lp_bytes = lsd_prep_bytes(W, H) * B
    bf_ms = ktot / max(kn, 1)
    roof = {"bound": "hbm", "kernel": "orb_blur_fast_kernel (7x7 blur + FAST score, all 8 levels, one launch)",
            "achieved": bf_bytes / (bf_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "traffic": committed_traffic(B, "orb_blur_fast_kernel") if (W, H) == (640, 480) else None,
            "bytes_per_launch": bf_bytes, "bytes_model": "SURVEY 8(d): blur read+write + FAST read of all levels",
            "kernel_bytes_per_launch": blur_fast_kernel_bytes(W, H) * B,
            "kernel_bytes_frac": blur_fast_kernel_bytes(W, H) * B / (bf_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "avg_launch_ms": bf_ms, "launches": kn}
    roof["frac"] = roof["achieved"] / roof["peak"]
    if (W, H) == (640, 480):
        roof["valu"] = valu_roof(B, "orb_blur_fast_kernel", bf_ms if kn else None,
                                 bf_iso[0] / bf_iso[1] if bf_iso[1] else None)
    if bf_iso[1]:
        # the same launch with nothing beside it (stage-timing runs): the timed
        # figure above shares the CUs with region growing and the other batch
        i_ms = bf_iso[0] / bf_iso[1]
        roof["isolated"] = {"avg_launch_ms": i_ms, "launches": bf_iso[1], "achieved": bf_bytes / (i_ms * 1e-3) / 1e9,
                            "frac": bf_bytes / (i_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
    # the ORB resize pass (north_star: "pyramid" passes), same pricing
    py_bytes = pyramid_bytes(W, H) * B
    py_ms = ptot / max(pn, 1)
    roof_pyr = {"bound": "hbm", "kernel": "orb_pyramid_kernel (ComputePyramid: 7 chained INTER_LINEAR 8U resizes, "
                                          "one streaming launch)",
                "achieved": py_bytes / (py_ms * 1e-3) / 1e9 if pn else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "traffic": committed_traffic(B, "orb_pyramid_kernel") if (W, H) == (640, 480) else None,
                "bytes_per_launch": py_bytes,
                "bytes_model": "SURVEY 8(d): level l-1 read + level l written, l = 1..7 (1 569 878 B/frame)",
                "avg_launch_ms": py_ms, "launches": pn}
    if roof_pyr["achieved"]:
        roof_pyr["frac"] = roof_pyr["achieved"] / HBM_PEAK_GBS
    if (W, H) == (640, 480):
        roof_pyr["valu"] = valu_roof(B, "orb_pyramid_kernel", py_ms if pn else None,
                                     pyr_iso[0] / pyr_iso[1] if pyr_iso[1] else None)
    if pyr_iso[1]:
        i_ms = pyr_iso[0] / pyr_iso[1]
        roof_pyr["isolated"] = {"avg_launch_ms": i_ms, "launches": pyr_iso[1],
                                "achieved": py_bytes / (i_ms * 1e-3) / 1e9,
                                "frac": py_bytes / (i_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
    lp_ms = ltot / max(ln, 1)
    roof_lsd = {"bound": "hbm", "kernel": "lsd_prep_kernel (u8 -> f64 blur 7x7, resize x0.8, ll_angle; one launch "
                                          "per octave)",
                "achieved": (lp_bytes / 2) / (lp_ms * 1e-3) / 1e9 if ltot else None, "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "traffic": committed_traffic(B, "lsd_prep_kernel") if (W, H) == (640, 480) else None,
                "bytes_per_launch": lp_bytes / 2, "per_launch": "mean of the two octave launches (bytes and traffic)",
                "avg_launch_ms": lp_ms, "launches": ln}
    if roof_lsd["achieved"]:
        roof_lsd["frac"] = roof_lsd["achieved"] / HBM_PEAK_GBS
    roof_lbd = {}
    for k, (name, what) in enumerate((("lbd_sobel0_kernel", "octave-0 5x5 Gaussian + Sobel dx/dy"),
                                      ("lbd_sobel1_kernel", "pyrDown + Sobel dx/dy of octave 1"))):
        by = lbd_sobel_bytes(W, H)[k] * B
        t_ms = sob[k][0] / max(sob[k][1], 1)
        i_ms = lbd_iso[k][0] / max(lbd_iso[k][1], 1)
        e = {"bound": "hbm", "kernel": f"{name} ({what})", "bytes_per_launch": by,
             "bytes_model": "SURVEY 8(d) LBD split per octave (blur/pyrDown r+w, Sobel u8 in + 2 x i16 out)",
             "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "traffic": committed_traffic(B, name) if (W, H) == (640, 480) else None,
             "in_schedule": {"avg_launch_ms": t_ms, "launches": sob[k][1],
                             "achieved": by / (t_ms * 1e-3) / 1e9 if sob[k][1] else None},
             "isolated": {"avg_launch_ms": i_ms, "launches": lbd_iso[k][1],
                          "achieved": by / (i_ms * 1e-3) / 1e9 if lbd_iso[k][1] else None}}
        for part in ("in_schedule", "isolated"):
            if e[part]["achieved"]:
                e[part]["frac"] = e[part]["achieved"] / HBM_PEAK_GBS
        roof_lbd[name] = e
    e2e_b = E2E_BYTES_640 if (W, H) == (640, 480) else E2E_BYTES_752 if (W, H) == (752, 480) else None
    e2e = None if e2e_b is None else {"bytes_per_frame": e2e_b, "achieved": e2e_b * value / world / 1e9,
                                      "unit": "GB/s per GPU", "frac": e2e_b * value / world / 1e9 / HBM_PEAK_GBS,
                                      "model": "SURVEY 8(d) reference-materialisation bytes x FPS per GPU"}

    # ---------------------------------------------------------- checks
    checks, digests = [], {"first_batch_frames": first_digest}
    if not args.no_check:
        checks = collect_checks(torch, plvi, seq, lo_last, B, W, H, orb, lx, outs, lm12, lnm, cap, lcap, extract,
                                match)
    # per-rank digest of the first window's tables (what rank 0 receives)
    if args.gather:
        extract(seq.data_ptr())
        match()
        torch.cuda.synchronize()
        h = hashlib.sha256()
        for src, n in zip((co_p, kp_p, de_p, lco_p, kl_p, lde_p), tab_sizes):
            h.update(plvi.download(src, np.zeros(n, np.uint8)).tobytes())
        digests["first_batch_tables"] = h.hexdigest()[:16]
        if world > 1:
            gather()
            wait_gathers()
            torch.cuda.synchronize()
            if rank == 0:
                digests["gathered_tables"] = s0.tg.digests()
    all_digests = [digests]
    if world > 1:
        import torch.distributed as dist
        all_digests = [None] * world
        dist.all_gather_object(all_digests, digests)

    extra = {}
    if rank == 0 and world == 1 and not args.no_extra:
        extra = extra_lines(args, torch, plvi, synth, lib, stream, W, H, seed0, orb, lx, extract, match, seq, B,
                            lat_handles, slots, fused, nwin, wstride)
        if "h2d_overlapped" in extra:
            extra["h2d_overlapped"]["frac_of_resident"] = extra["h2d_overlapped"]["value"] / value

    result = {
        "metric": METRIC if (W, H) == (640, 480) else METRIC.replace("640×480", f"{W}×{H}"), "value": value,
        "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (plvi.synth.device_sequence: seeded scenes, integer camera shifts, sigma-2 noise)",
        "config": {"workload": ("C4: 752x480 sequence per rank, windows of B frames with a one-frame halo; "
                                if args.c4 else "C1+C2+C3: ") +
                               "ORB extract (1000 feats, 1.2, 8 levels, FAST 20/7) || LSD+LBD (200 lines, scale 0.8, "
                               "2 octaves) as one HIP-stream schedule, then ORB kNN-2 + LineMatcher::match vs "
                               "previous frame" + (", RCCL gather of per-frame tables to rank 0" if args.gather
                                                   else ""),
                   "batch": B, "frames_per_step": new_frames, "width": W, "height": H,
                   "parallelism": f"sequence-sharded x{world}", "gather": bool(args.gather),
                   "inflight": len(slots), "schedule": schedule_knobs(B)},
        "roofline": roof,
        "roofline_pyramid": roof_pyr,
        "roofline_lsd_prep": roof_lsd,
        "roofline_lbd": roof_lbd,
        "end_to_end_hbm": e2e,
        "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
        "dominant_stage": max(stage_ms, key=stage_ms.get),
        "part_fps": {k: round(v, 1) for k, v in parts.items()},
        "side_ms": side,
        "device_errors": {"orb": err[0], "lines": err[1]},
        "digests": all_digests,
    }
    result.update(extra)
    fail = []
    if err[0] or err[1]:
        fail.append(f"device error flags orb={err[0]} lines={err[1]}")
    if checks:
        bad = oracle_verify(checks)
        result["oracle_check"] = {"frames": [lo_last, lo_last + B // 2, lo_last + B - 1], "items": len(checks),
                                  "mismatches": bad}
        if bad:
            fail.append(f"oracle mismatch: {bad}")
    b64c = result.pop("_b64_checks", None)
    if b64c:
        bad = oracle_verify(b64c[1])
        result["batch64"]["oracle_check"] = {"frames": b64c[0], "items": len(b64c[1]), "mismatches": bad}
        if bad:
            fail.append(f"batch-64 oracle mismatch: {bad}")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        n = min(args.cpu_frames, B)
        result["cpu_baseline"] = cpu_baseline([seq[i].cpu().numpy() for i in range(n)])
    if world > 1:
        import torch.distributed as dist
        flags = [None] * world
        dist.all_gather_object(flags, fail)
        fail = [f"rank {r}: {m}" for r, fl in enumerate(flags) for m in fl]
        dist.destroy_process_group()
    if fail:
        result["failed"] = fail
    if rank == 0:
        print(json.dumps(result), flush=True)
    return 1 if fail else 0


def collect_checks(torch, plvi, seq, lo, B, W, H, orb, lx, outs, lm12, lnm, cap, lcap, extract, match):
    """Re-run the last timed batch and download frames 0, B/2, B-1 and the
    match of pair (B/2-1, B/2) for the oracle comparison."""
    extract(seq[lo].data_ptr())
    match()
    torch.cuda.synchronize()
    kp_p, de_p, co_p, mo_p, _ = orb.outputs()
    kl_p, lde_p, fn_p, lco_p, _ = lx.outputs()
    cnt = plvi.download(co_p, np.zeros(B, np.int32))
    mono = plvi.download(mo_p, np.zeros(B, np.int32))
    lcnt = plvi.download(lco_p, np.zeros(B, np.int32))
    checks = []
    tabs = {}
    for f in sorted({0, B // 2 - 1, B // 2, B - 1}):
        n, nl = int(cnt[f]), int(lcnt[f])
        k = plvi.download(kp_p + 28 * cap * f, np.zeros(n, plvi.KEYPOINT_DTYPE))
        d = plvi.download(de_p + 32 * cap * f, np.zeros((n, 32), np.uint8))
        kl = plvi.download(kl_p + 68 * lcap * f, np.zeros(nl, plvi.KEYLINE_DTYPE))
        ld = plvi.download(lde_p + 32 * lcap * f, np.zeros((nl, 32), np.uint8))
        fn = plvi.download(fn_p + 24 * lcap * f, np.zeros((nl, 3), np.float64))
        tabs[f] = (d, ld)
        if f != B // 2 - 1:
            img = seq[lo + f].cpu().numpy()
            checks.append(("orb", img, (int(mono[f]), k, d)))
            checks.append(("lines", img, (kl, ld, fn)))
    p = B // 2 - 1  # pair p matches frame p+1 (query) against frame p (train)
    n1 = int(cnt[p + 1])
    got = tuple(plvi.download(o.data_ptr() + 4 * cap * p, np.zeros(n1, np.int32)) for o in outs)
    checks.append(("knn2", (tabs[p + 1][0], tabs[p][0]), got))
    nl1 = len(tabs[p + 1][1])
    if nl1 and len(tabs[p][1]) >= 2:
        m = plvi.download(lm12.data_ptr() + 4 * lcap * p, np.zeros(nl1, np.int32))
        nm = int(plvi.download(lnm.data_ptr() + 4 * p, np.zeros(1, np.int32))[0])
        checks.append(("lmatch", (tabs[p + 1][1], tabs[p][1]), (nm, m)))
    return checks


def side_stages(args, torch, plvi, synth, lib, orb, st, stream, B, W, H, cap, kp_p, de_p, co_p, nprof, cuda, seed0):
    """Stages next to the per-frame step, timed separately on the
    same batch: DBoW2 transform, AssignFeaturesToGrid + SearchByProjection,
    rectified stereo (ORB SAD + line matchGrid)."""
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = {}

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ev0.record(stream)
        for _ in range(nprof):
            fn()
        ev1.record(stream)
        torch.cuda.synchronize()
        return ev0.elapsed_time(ev1) / nprof
    # DBoW2 transform of the batch's descriptors on a k=10, L=6 synthetic vocabulary
    pv = synth.vocabulary(10, 6, seed=1)
    voc = plvi.ORBVocabulary.from_nodes(10, 6, 0, 0, *pv, device=torch.cuda.current_device())
    bo = {k: torch.empty(B * (cap + 1) * sz, dtype=torch.uint8, device=cuda)
          for k, sz in (("bw", 4), ("bv", 8), ("bn", 4), ("fn", 4), ("fo", 4), ("fi", 4), ("fc", 4))}

    def run_bow():
        rc = lib.plvi_vocab_transform_batch(voc._h, de_p, co_p, cap, B, 4, *[bo[k].data_ptr() for k in
                                            ("bw", "bv", "bn", "fn", "fo", "fi", "fc")], None, None, st)
        if rc:
            raise RuntimeError(f"bow {rc}")
    out["bow.transform"] = timed(run_bow)
    # SearchByProjection: frame t vs frame t-1's keypoints as MapPoints
    gp = plvi.GridParams(0.0, 0.0, *[float(x) for x in plvi.grid_geometry(W, H)[4:]])
    cell_off = torch.empty(B * 3073, dtype=torch.int32, device=cuda)
    cell_idx = torch.empty(B * cap, dtype=torch.int32, device=cuda)
    kpt = torch.empty(B * cap * 7, dtype=torch.float32, device=cuda)
    lib.plvi_memcpy_async(kpt.data_ptr(), kp_p, B * cap * 28, 3, st)
    torch.cuda.synchronize()
    kv = kpt.view(B, cap, 7)
    fx, fy, cx, cy, z = 458.654, 457.296, 367.215, 248.375, 5.0
    x3 = torch.stack([(kv[..., 0] - cx) * z / fx, (kv[..., 1] - cy) * z / fy,
                      torch.full_like(kv[..., 0], z)], -1).contiguous()
    loct = kv[..., 5].view(torch.int32).contiguous()
    lang = kv[..., 3].contiguous()
    lflags = torch.full((B * cap,), 3, dtype=torch.uint8, device=cuda)
    pp = plvi.ProjParams()
    pp.fx, pp.fy, pp.cx, pp.cy, pp.mbf, pp.th = fx, fy, cx, cy, 40.0, 15.0
    pp.min_x, pp.max_x, pp.min_y, pp.max_y, pp.inv_w, pp.inv_h = [float(x) for x in plvi.grid_geometry(W, H)]
    pp.check_orientation, pp.nlevels = 1, 8
    for i, sfac in enumerate(orb.GetScaleFactors()):
        pp.scale_factors[i] = float(sfac)
    pm = torch.empty((B - 1) * cap, dtype=torch.int32, device=cuda)
    pn = torch.empty(B, dtype=torch.int32, device=cuda)

    def run_proj():
        plvi.assign_grid_batch(kp_p, co_p, cap, B, gp, cell_off.data_ptr(), cell_idx.data_ptr(), st)
        rc = lib.plvi_search_by_projection_batch(
            B - 1, ctypes.byref(pp), kp_p + 28 * cap, de_p + 32 * cap, co_p + 4, cap, None, None,
            cell_off.data_ptr() + 4 * 3073, cell_idx.data_ptr() + 4 * cap, x3.data_ptr(), loct.data_ptr(),
            lang.data_ptr(), de_p, lflags.data_ptr(), co_p, cap, pm.data_ptr(), pn.data_ptr(), st)
        if rc:
            raise RuntimeError(f"projection {rc}")
    out["proj.grid+search"] = timed(run_proj)
    # local-map search (ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>), Tracking.cc:5119):
    # frame t against frame t-1's keypoints as the local map (predicted position = keypoint,
    # level = octave, view cosine 1, their descriptors), th = 1, nnratio 0.8
    lpp = plvi.LocalParams()
    lpp.min_x, lpp.min_y, lpp.inv_w, lpp.inv_h = 0.0, 0.0, *[float(x) for x in plvi.grid_geometry(W, H)[4:]]
    lpp.th, lpp.nnratio, lpp.nlevels = 1.0, 0.8, 8
    for i, sfac in enumerate(orb.GetScaleFactors()):
        lpp.scale_factors[i] = float(sfac)
    mproj = torch.stack([kv[..., 0], kv[..., 1], kv[..., 0], torch.ones_like(kv[..., 0])], -1).contiguous()
    mflags = torch.full((B * cap,), 3, dtype=torch.uint8, device=cuda)
    lm = torch.empty((B - 1) * cap, dtype=torch.int32, device=cuda)
    ln = torch.empty(B, dtype=torch.int32, device=cuda)

    def run_local():
        rc = lib.plvi_search_local_batch(
            B - 1, ctypes.byref(lpp), kp_p + 28 * cap, de_p + 32 * cap, co_p + 4, cap, None, None,
            cell_off.data_ptr() + 4 * 3073, cell_idx.data_ptr() + 4 * cap, mflags.data_ptr(), mproj.data_ptr(),
            loct.data_ptr(), de_p, co_p, cap, lm.data_ptr(), ln.data_ptr(), st)
        if rc:
            raise RuntimeError(f"local search {rc}")
    out["local.search"] = timed(run_local)
    # stereo on S rectified pairs extracted by their own handles
    S = min(B, 256)
    pairs = [synth.stereo_pair(seed0 + 10 ** 5 + i, W, H) for i in range(S)]
    sl = torch.from_numpy(np.stack([p[0] for p in pairs])).to(cuda)
    sr = torch.from_numpy(np.stack([p[1] for p in pairs])).to(cuda)
    dev = torch.cuda.current_device()
    o_l = plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=S, device=dev)
    o_r = plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=S, device=dev)
    l_l = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=S, device=dev)
    l_r = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=S, device=dev)
    for e, fr in ((o_l, sl), (o_r, sr), (l_l, sl), (l_r, sr)):
        e.extract_batch(fr.data_ptr(), S, W * H, W, stream=st)
    torch.cuda.synchronize()
    scap = o_l.kp_cap
    st_f = torch.empty(2 * S * scap, dtype=torch.float32, device=cuda)
    st_i = torch.zeros(S + 1, dtype=torch.int32, device=cuda)
    a_kl, a_de, _, a_co, a_cap = l_l.outputs()
    b_kl, b_de, _, b_co, b_cap = l_r.outputs()
    idx_cap = 32768
    sbytes = plvi.stereo_lines_scratch_bytes(S, a_cap, b_cap, idx_cap)
    s_scr = torch.empty(sbytes, dtype=torch.uint8, device=cuda)
    s_lo = torch.empty(S * a_cap * 11, dtype=torch.float64, device=cuda)
    lo = s_lo.data_ptr()
    mbf_, mb_ = 47.90639384423901, 0.11
    out["stereo.orb"] = timed(lambda: plvi.stereo_match_batch(
        o_l, o_r, S, mb_, mbf_, st_f.data_ptr(), st_f.data_ptr() + 4 * S * scap, st_i.data_ptr(),
        st_i.data_ptr() + 4 * S, stream=st))
    out["stereo.lines"] = timed(lambda: plvi.stereo_lines_batch(
        S, a_kl, a_de, a_co, a_cap, b_kl, b_de, b_co, b_cap, None, W, H, mbf_, 1, idx_cap, s_scr.data_ptr(), sbytes,
        lo, lo + 4 * S * a_cap, lo + 12 * S * a_cap, lo + 20 * S * a_cap, lo + 44 * S * a_cap,
        st_i.data_ptr() + 4 * S, stream=st))
    if int(st_i[S].item()) != 0:
        raise RuntimeError(f"stereo err {int(st_i[S].item())}")
    out["stereo.pairs"] = S
    return {k: round(v, 4) if isinstance(v, float) else v for k, v in out.items()}


def extra_lines(args, torch, plvi, synth, lib, stream, W, H, seed0, orb, lx, extract, match, seq, B, lat_handles,
                main_slots, fused, nwin, wstride):
    """Rank 0, N=1: (1) the same step at batch 64 (BASELINE C1/C2 as stated),
    on distinct frames every step, the last step's frames 0 / 31 / 32 / 63 and
    pair (31, 32) checked against the oracle; (2) single-frame latency of the
    drop-in entry points run the way Frame runs them (plvi_orb_extract ||
    plvi_lines_extract on two host threads, host image in, host tables out;
    Frame.cc:558-561); (3) the headline schedule (same slots, same fused
    extract + match) with every batch's frames streamed from pinned host
    memory: per slot a copy stream and two device frame buffers, the H2D of a
    slot's next batch overlapped with the step in flight."""
    import threading
    out = {}
    # the batch-64 pair's own stream, created with its extractors at start-up
    # (on slot 0's stream the step measured 8.46-8.53 ms instead of 7.90:
    # that stream shares one of the runtime's few hardware queues with a
    # stream of the pair's schedule)
    st = lat_handles[4].cuda_stream
    dev = torch.cuda.current_device()
    cuda = f"cuda:{dev}"
    # (1) batch 64
    b64 = 64
    o64, l64 = lat_handles[2], lat_handles[3]  # created at start-up
    kp, de, co, _, cap = o64.outputs()
    _, lde, _, lco, lcap = l64.outputs()
    i32 = dict(dtype=torch.int32, device=cuda)
    o4 = [torch.empty((b64 - 1) * cap, **i32) for _ in range(4)]
    lsc = torch.empty(4 * (b64 - 1) * 2 * lcap, **i32)
    lm = torch.empty((b64 - 1) * lcap, **i32)
    lnm = torch.empty(b64 - 1, **i32)
    # the step's matching issued inside the frame schedule: the ORB kNN-2
    # right behind the ORB chain, LineMatcher::match right behind the LBD
    # descriptors (plvi_frame_extract_match_batch; same kernels and outputs as
    # the calls after the schedule, minus the stream joins in between)
    # every step on its own 64 distinct resident frames (consecutive windows
    # of the bench's sequence)
    nwin64 = max(1, (seq.shape[0] - b64) // b64 + 1)

    def step64(i):
        lo64 = (i % nwin64) * b64
        plvi.frame_extract_match_batch(o64, l64, seq[lo64].data_ptr(), b64, W * H, W, [o.data_ptr() for o in o4],
                                       0.9, lsc.data_ptr(), lm.data_ptr(), lnm.data_ptr(), stream=st)
        return lo64
    for i in range(3):
        step64(i)
    torch.cuda.synchronize()
    n64 = 50
    t0 = time.perf_counter()
    for i in range(n64):
        lo64 = step64(3 + i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out["batch64"] = {"value": b64 * n64 / el, "unit": "frames/s", "ms_per_step": el / n64 * 1e3,
                      "distinct_frames": min(n64, nwin64) * b64,
                      "config": "C1/C2/C3 at batch 64 (BASELINE.json configs[1..2]): same extract+match step, "
                                "distinct frames every step"}
    if o64.errors(st) or l64.errors(st):
        raise RuntimeError("batch-64 device error flags")
    # the last timed step's tables against the oracle (outputs as the timed
    # step left them: the re-run below writes the same tables)
    if not args.no_check:
        def ex64(fptr):
            plvi.frame_extract_match_batch(o64, l64, fptr, b64, W * H, W, [o.data_ptr() for o in o4], 0.9,
                                           lsc.data_ptr(), lm.data_ptr(), lnm.data_ptr(), stream=st)
        out["_b64_checks"] = ([lo64, lo64 + b64 // 2 - 1, lo64 + b64 // 2, lo64 + b64 - 1],
                              collect_checks(torch, plvi, seq, lo64, b64, W, H, o64, l64, o4, lm, lnm, cap, lcap,
                                             ex64, lambda: None))
    del o64, l64
    # (1b) batch 64 with K batches in flight: K independent extractor slots
    # (own tables and streams), step i on slot i % K over its own 64 frames;
    # every step is the full 64-frame extract + match
    K = 16
    slots = []
    for k in range(K):
        sl_ = types.SimpleNamespace()
        sl_.o = plvi.ORBextractor(1000, 1.2, 8, 20, 7, W, H, max_batch=b64, device=dev)
        sl_.l = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, W, H, max_batch=b64, device=dev)
        sl_.kp, sl_.de, sl_.co, _, _ = sl_.o.outputs()
        _, sl_.lde, _, sl_.lco, _ = sl_.l.outputs()
        sl_.o4 = [torch.empty((b64 - 1) * cap, **i32) for _ in range(4)]
        sl_.lsc = torch.empty(4 * (b64 - 1) * 2 * lcap, **i32)
        sl_.lm = torch.empty((b64 - 1) * lcap, **i32)
        sl_.lnm = torch.empty(b64 - 1, **i32)
        sl_.s = torch.cuda.Stream()
        sl_.f = seq[(k * b64) % max(1, seq.shape[0] - b64)].data_ptr()
        slots.append(sl_)

    def step64k(i):
        q = slots[i % K]
        sq = q.s.cuda_stream
        plvi.frame_extract_batch(q.o, q.l, q.f, b64, W * H, W, (0, 0), stream=sq)
        rc = lib.plvi_hamming_knn2_batch(q.de + cap * 32, q.co + 4, cap, q.de, q.co, cap, b64 - 1,
                                         *[o.data_ptr() for o in q.o4], sq)
        rc |= lib.plvi_line_match_batch(q.lde + lcap * 32, q.lco + 4, lcap, q.lde, q.lco, lcap, b64 - 1, 0.9,
                                        q.lsc.data_ptr(), q.lm.data_ptr(), q.lnm.data_ptr(), sq)
        if rc:
            raise RuntimeError("b64 pipelined match")
    for i in range(K):
        step64k(i)
    torch.cuda.synchronize()
    nk = 8 * K

    def timed_steps(fn):
        t0 = time.perf_counter()
        for i in range(nk):
            fn(i)
        torch.cuda.synchronize()
        return b64 * nk / (time.perf_counter() - t0)
    v_api = timed_steps(step64k)
    # the same step replayed from HIP graphs, one capture per slot; the graph
    # holds the step on the slot's one stream (ORB extract, line extract,
    # matches).  This process imports torch, so the library runs on
    # PyTorch's bundled HIP 7.0 runtime, which crashes capturing the
    # multi-stream frame schedule's fork/join; plvi_frame_extract_batch
    # refuses capture there (PLVI_E_CAPTURE), while ROCm 7.2's runtime
    # captures it.  The 16 slots provide the concurrency.
    def step64g(q, sq):
        q.o.extract_batch(q.f, b64, W * H, W, (0, 0), stream=sq)
        q.l.extract_batch(q.f, b64, W * H, W, stream=sq)
        rc = lib.plvi_hamming_knn2_batch(q.de + cap * 32, q.co + 4, cap, q.de, q.co, cap, b64 - 1,
                                         *[o.data_ptr() for o in q.o4], sq)
        rc |= lib.plvi_line_match_batch(q.lde + lcap * 32, q.lco + 4, lcap, q.lde, q.lco, lcap, b64 - 1, 0.9,
                                        q.lsc.data_ptr(), q.lm.data_ptr(), q.lnm.data_ptr(), sq)
        if rc:
            raise RuntimeError("b64 graph match")
    for q in slots:
        q.g = plvi.StepGraph(lambda sq, q=q: step64g(q, sq), q.s.cuda_stream)
    for q in slots:
        q.g.launch()
    torch.cuda.synchronize()
    v_graph = timed_steps(lambda i: slots[i % K].g.launch())
    out["batch64_in_flight"] = {
        "value": max(v_api, v_graph), "unit": "frames/s", "batches_in_flight": K, "api_calls": v_api,
        "hip_graphs": v_graph, "ms_per_batch_latency_floor": out["batch64"]["ms_per_step"],
        "config": f"batch 64 per step, {K} independent batches in flight (own extractors and streams, "
                  f"{K * b64} frames resident): the C1/C2 step as a stream of 64-frame batches; steps issued "
                  f"call by call (frame schedule) and as one HIP-graph launch each (plvi_graph_*, the step "
                  f"on one stream)"}
    for q in slots:
        if q.o.errors(q.s.cuda_stream) or q.l.errors(q.s.cuda_stream):
            raise RuntimeError("pipelined batch-64 device error flags")
    del slots
    # (2) single-frame latency: host image -> host tables, ORB || lines on two threads
    so, sl = lat_handles[0], lat_handles[1]
    imgs = [seq[i].cpu().numpy() for i in range(24)]
    lat, lo_, ll_ = [], [], []
    for rep in range(len(imgs) + 4):
        img = imgs[rep % len(imgs)]
        res = {}

        def ro():
            t = time.perf_counter()
            so(img)
            res["orb"] = time.perf_counter() - t

        def rl():
            t = time.perf_counter()
            sl(img)
            res["lines"] = time.perf_counter() - t
        t0 = time.perf_counter()
        th = [threading.Thread(target=ro), threading.Thread(target=rl)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if rep >= 4:
            lat.append(time.perf_counter() - t0)
            lo_.append(res["orb"])
            ll_.append(res["lines"])
    out["single_frame_latency"] = {
        "median_ms": float(np.median(lat)) * 1e3, "p90_ms": float(np.percentile(lat, 90)) * 1e3,
        "orb_median_ms": float(np.median(lo_)) * 1e3, "lines_median_ms": float(np.median(ll_)) * 1e3,
        "frames": len(lat), "how": "plvi_orb_extract || plvi_lines_extract on two host threads (Frame.cc:558-561), "
                                   "host frame in, host keypoints/keylines/descriptors out"}
    # the same measurement in a child process that holds only the two
    # extractors (a SLAM process's drop-in situation; this process holds ~20
    # more handles whose streams share the runtime's hardware queues)
    try:
        cp = subprocess.run([sys.executable, str(ROOT / "tools" / "latency_pair.py"), "--json"], capture_output=True,
                            text=True, timeout=180)
        if cp.returncode == 0:
            fp = json.loads(cp.stdout.strip().splitlines()[-1])
            fp["how"] = "tools/latency_pair.py in a child process holding only the ORB and line extractors"
            out["single_frame_latency"]["drop_in_process"] = fp
    except (subprocess.SubprocessError, ValueError, IndexError) as e:
        out["single_frame_latency"]["drop_in_process"] = {"error": str(e)[:200]}
    del so, sl
    # (3) host-fed headline schedule: the timed step's slots and fused
    # extract + match, each batch's frames copied from pinned host memory.
    # Per slot: its own pinned host window, a copy stream and two device
    # buffers; the copy of a slot's next batch waits only for the step that
    # last used that buffer, so it overlaps the steps in flight.
    nsl = len(main_slots)
    hosts = []
    for j in range(nsl):
        lo_j = (j % nwin) * wstride
        hb = torch.empty((B, H, W), dtype=torch.uint8, pin_memory=True)
        hb.copy_(seq[lo_j:lo_j + B].cpu())
        hosts.append(hb)
    dbuf = [[torch.empty((B, H, W), dtype=torch.uint8, device=cuda) for _ in range(2)] for _ in range(nsl)]
    cstreams = [torch.cuda.Stream() for _ in range(nsl)]
    ev_copied = [[torch.cuda.Event() for _ in range(2)] for _ in range(nsl)]
    ev_free = [[torch.cuda.Event() for _ in range(2)] for _ in range(nsl)]
    for j in range(nsl):
        for b in range(2):
            ev_free[j][b].record(main_slots[j].stream)

    def h2d(k):
        j, b = k % nsl, (k // nsl) % 2
        cstreams[j].wait_event(ev_free[j][b])
        with torch.cuda.stream(cstreams[j]):
            dbuf[j][b].copy_(hosts[j], non_blocking=True)
        ev_copied[j][b].record(cstreams[j])

    def hstep(k):
        j, b = k % nsl, (k // nsl) % 2
        sl_ = main_slots[j]
        sl_.stream.wait_event(ev_copied[j][b])
        fused(sl_, dbuf[j][b].data_ptr())
        ev_free[j][b].record(sl_.stream)

    # H2D alone (one batch, pinned), for the bandwidth the schedule can draw on
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(cstreams[0])
    for _ in range(3):
        with torch.cuda.stream(cstreams[0]):
            dbuf[0][0].copy_(hosts[0], non_blocking=True)
    e1.record(cstreams[0])
    torch.cuda.synchronize()
    h2d_alone = 3 * B * W * H / (e0.elapsed_time(e1) * 1e-3) / 1e9
    nh = max(args.steps, 6)
    nw = 2 * nsl
    for k in range(nsl):
        h2d(k)
    for k in range(nw):  # warm-up steps, copies kept nsl steps ahead
        h2d(k + nsl)
        hstep(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(nw, nw + nh):
        h2d(k + nsl)
        hstep(k)
    for sl_ in main_slots:
        sl_.stream.synchronize()
    el = time.perf_counter() - t0
    torch.cuda.synchronize()  # the copies issued ahead of the last steps
    out["h2d_overlapped"] = {"value": B * nh / el, "unit": "frames/s", "ms_per_step": el / nh * 1e3,
                             "pcie_gbs": B * W * H * nh / el / 1e9, "h2d_alone_gbs": h2d_alone,
                             "inflight": nsl,
                             "how": "the headline schedule (same slots, plvi_frame_extract_match_batch) with every "
                                    "batch copied from pinned host memory: per slot a copy stream and two device "
                                    "buffers, the copy of a slot's next batch overlapped with the steps in flight"}
    for sl_ in main_slots:
        if sl_.orb.errors(sl_.st) or sl_.lx.errors(sl_.st):
            raise RuntimeError("h2d device error flags")
    return out


if __name__ == "__main__":
    sys.exit(main())
