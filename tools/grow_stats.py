"""Diagnostic: cycle accounting of the LSD region-growing kernel on one batch
(the bench's device sequence, so B = 3072 shows the contended per-wave times).
usage: python tools/grow_stats.py [B]"""
import ctypes
import pathlib
import sys

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
import plvi  # noqa: E402
from plvi import synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
seq = synth.device_sequence(B, 640, 480, seed=0, device="cuda:0")
torch.cuda.synchronize()
lx = plvi.Lineextractor(200, 0, 0.8, 2, 2.0, 0, 640, 480, max_batch=B)
st = torch.zeros(B * 2 * 24, dtype=torch.int64, device="cuda:0")
lib = plvi.load()
lx.extract_batch(seq.data_ptr(), B, 640 * 480, 640)
lib.plvi_device_synchronize()
lib.plvi_lines_debug_stats(lx._h, ctypes.c_void_p(st.data_ptr()))
lx.extract_batch(seq.data_ptr(), B, 640 * 480, 640)
lib.plvi_device_synchronize()
lib.plvi_lines_debug_stats(lx._h, ctypes.c_void_p(0))
raw = st.cpu().numpy().reshape(B, 2, 24)
s = raw[:, :, :16].astype(np.float64)
names = ["total", "block_setup", "rounds", "rect", "seeds", "blocks", "rounds_n", "rect_pts", "commits", "ph_decide",
         "ph_angles", "ph_verify", "ph_commit", "seed_scan", "seed_start", "init"]
# 64-pixel chunks of the seed scan per octave (octave 0 = 0.8 x 640 x 480, octave 1 half of it)
dims = [(512, 384), (256, 192)]
names_chunks = [((w - 1 + 63) // 64) * (h - 1) for w, h in dims]
print(f"B = {B}")
for o in range(2):
    print(f"octave {o}:")
    for i, n in enumerate(names):
        print(f"  {n:10s} mean {s[:, o, i].mean():14.0f}  max {s[:, o, i].max():14.0f}")
    t = s[:, o]
    print("  setup cycles/block %.0f  round cycles/round %.0f  rounds/block %.2f  commits/round %.2f  "
          "rect cycles/pt %.0f  total cycles/commit %.0f" % (
              (t[:, 1] / t[:, 5]).mean(), (t[:, 2] / t[:, 6]).mean(), (t[:, 6] / t[:, 5]).mean(),
              (t[:, 8] / t[:, 6]).mean(), (t[:, 3] / np.maximum(t[:, 7], 1)).mean(),
              (t[:, 0] / np.maximum(t[:, 8], 1)).mean()))
    print("  per round: decide %.0f  angles %.0f  verify %.0f  commit %.0f" % tuple(
        (t[:, 9 + k] / t[:, 6]).mean() for k in range(4)))
    print("  seed scan %.0f (%.1f %%, %.0f per 64-pixel chunk)  seed starts %.0f (%.0f per seed)  init %.0f" % (
        t[:, 13].mean(), 100 * (t[:, 13] / t[:, 0]).mean(), t[:, 13].mean() / max(1, names_chunks[o]),
        t[:, 14].mean(), (t[:, 14] / np.maximum(t[:, 4], 1)).mean(), t[:, 15].mean()))
    print("  unaccounted %.1f %%" % (100 * ((t[:, 0] - t[:, 1] - t[:, 2] - t[:, 3] - t[:, 13] - t[:, 14] - t[:, 15])
                                          / t[:, 0]).mean()))
    print("  wave time: mean %.0f  max %.0f cycles" % (t[:, 0].mean(), t[:, 0].max()))
# work vs time: is the slowest wave the one with the most work, or a contended one?
for o in range(2):
    t = s[:, o]
    cyc, blk = t[:, 0], t[:, 5]
    r = np.corrcoef(cyc, blk)[0, 1]
    per = cyc / np.maximum(blk, 1)
    top = np.argsort(cyc)[-5:][::-1]
    print(f"octave {o}: corr(cycles, blocks) {r:.3f}; cycles/block mean {per.mean():.0f} min {per.min():.0f} "
          f"max {per.max():.0f}; blocks max {blk.max():.0f} (wave {int(np.argmax(blk))})")
    for i in top:
        print(f"   wave {i:5d} cycles {cyc[i]:12.0f} blocks {blk[i]:6.0f} cycles/block {per[i]:6.0f} "
              f"seeds {t[i, 4]:5.0f}")

# placement: waves per SIMD (same XCC / SE / SH / CU / SIMD) vs cycles per block
hw = raw[:, :, 16].astype(np.int64) & 0xFFFFFFFF
xcc = raw[:, :, 17].astype(np.int64) & 0xF
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
key = ((xcc * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
cuk = key // 4
uk, cnt = np.unique(key, return_counts=True)
ucu, ccnt = np.unique(cuk, return_counts=True)
print(f"placement: {len(uk)} SIMDs and {len(ucu)} CUs used; waves per SIMD min {cnt.min()} max {cnt.max()} "
      f"mean {cnt.mean():.2f}; waves per CU min {ccnt.min()} max {ccnt.max()}")
hist = np.bincount(cnt)
print("  SIMDs by wave count:", {i: int(h) for i, h in enumerate(hist) if h})
per_simd = dict(zip(uk, cnt))
for o in range(2):
    c = np.array([per_simd[k] for k in key[:, o]])
    cpb = s[:, o, 0] / np.maximum(s[:, o, 5], 1)
    for n in sorted(set(c)):
        m = c == n
        print(f"  octave {o}: waves on a SIMD with {n} grow waves: {m.sum():5d}, cycles/block {cpb[m].mean():6.0f}, "
              f"wave cycles mean {s[m, o, 0].mean():12.0f} max {s[m, o, 0].max():12.0f}")
    oc = np.array([np.sum((key[:, 0] == k)) for k in key[:, o]])
    for n in sorted(set(oc)):
        m = oc == n
        print(f"  octave {o}: SIMD holding {n} octave-0 waves: {m.sum():5d}, wave cycles mean {s[m, o, 0].mean():12.0f}")
t0 = raw[:, :, 18].astype(np.float64)
t0 -= t0.min()
print("  start-time spread (cycles): octave 0 max %.0f, octave 1 min %.0f max %.0f" % (
    t0[:, 0].max(), t0[:, 1].min(), t0[:, 1].max()))

# drains: commit rounds with USED rows beyond the LDS window (global atomics) or a queue spill
for o in range(2):
    far, sp = raw[:, o, 19].astype(np.float64), raw[:, o, 20].astype(np.float64)
    cyc = s[:, o, 0]
    print(f"octave {o}: far-row drains mean {far.mean():.0f} max {far.max():.0f}, spill drains mean {sp.mean():.0f} "
          f"max {sp.max():.0f}; corr(cycles, far) {np.corrcoef(cyc, far)[0, 1]:.3f} corr(cycles, spill) "
          f"{np.corrcoef(cyc, sp)[0, 1] if sp.std() > 0 else 0:.3f}")
    top = np.argsort(cyc)[-3:][::-1]
    print("   slowest:", [(int(i), int(far[i]), int(sp[i])) for i in top])

# start / end on the 100 MHz clock (s_memrealtime): do the slowest tasks start late?
r0, r1 = raw[:, :, 21].astype(np.float64), raw[:, :, 22].astype(np.float64)
base = r0.min()
for o in range(2):
    st, en = (r0[:, o] - base) / 100.0, (r1[:, o] - base) / 100.0  # microseconds
    cyc = s[:, o, 0]
    top = np.argsort(en)[-5:][::-1]
    print(f"octave {o}: start us mean {st.mean():.0f} max {st.max():.0f}; end us mean {en.mean():.0f} max {en.max():.0f}; "
          f"latest ends: {[(int(i), round(float(st[i])), round(float(en[i]))) for i in top]}")
    late = st > 100
    print(f"   tasks starting > 100 us late: {int(late.sum())}; their mean cycles/block "
          f"{(cyc[late] / np.maximum(s[late, o, 5], 1)).mean() if late.any() else 0:.0f}")
# end time by hardware location (averaged over the 8 XCCs): is the tail tied to particular CUs?
for o in range(2):
    en = (r1[:, o] - base) / 100.0
    loc = (se[:, o] * 2 + sh[:, o]) * 16 + cu[:, o]
    ul = np.unique(loc)
    means = sorted(((float(en[loc == u].mean()), int(u)) for u in ul), reverse=True)
    print(f"octave {o}: end us by (SE, SH, CU): slowest {[(round(m), u // 32, (u // 16) % 2, u % 16) for m, u in means[:4]]} "
          f"fastest {[(round(m), u // 32, (u // 16) % 2, u % 16) for m, u in means[-3:]]}")
    xs = np.unique(xcc[:, o])
    print(f"   by XCC: {[(int(x), round(float(en[xcc[:, o] == x].mean()))) for x in xs]}")
    top = np.argsort(en)[-6:]
    print(f"   slowest tasks at (XCC, SE, SH, CU, SIMD): {[(int(xcc[i, o]), int(se[i, o]), int(sh[i, o]), int(cu[i, o]), int(simd[i, o])) for i in top]}")
