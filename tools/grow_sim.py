"""Model of intra-frame speculative region growing (tools/grow_sim.cpp) on
synthetic and real frames: region statistics of flsd's sequential loop and
the modelled makespan of K concurrent waves (owner plane + in-order commit).
Diagnostic only: `python tools/grow_sim.py`."""
import ctypes
import pathlib
import subprocess
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    so = pathlib.Path("/tmp/grow_sim.so")
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-o", str(so), str(ROOT / "tools/grow_sim.cpp")], check=True)
    lib = ctypes.CDLL(str(so))
    import oracle_lib as ol
    from plvi import synth
    frames = [("synth%d" % s, synth.frame(s)) for s in (0, 3, 7)]
    g = np.load(ROOT / "tests/golden/frames.npz")
    for k in list(g.keys())[:2]:
        frames.append((k, g[k]))
    Ks = [int(x) for x in (sys.argv[1:] or ["1", "4", "8", "16", "32"])]
    for name, img in frames:
        for octv in (0, 1):
            im = img if octv == 0 else img[::2, ::2].copy()  # octave 1 ~ half size (stats only)
            _, ang, mod = ol.lsd_planes(im)
            h, w = ang.shape
            ang = np.ascontiguousarray(ang)
            mod = np.ascontiguousarray(mod)
            line = []
            base = None
            for K in Ks:
                for slots, view in ((1, 0), (2, 0), (1, 1), (2, 1)):
                    st = np.zeros(16)
                    lib.grow_sim(ang.ctypes.data_as(ctypes.c_void_p), w, h, K, slots, view, 2,
                                 st.ctypes.data_as(ctypes.c_void_p))
                    if base is None:
                        base = st[2]
                        print(f"{name} oct{octv} {w}x{h}: defined {int(st[8])} regions {int(st[0])} "
                              f"(>=10px {int(st[9])}) pts {int(st[1])} seq_cost {st[2]:.0f}")
                    line.append(f"K={K} slots={slots} view={view}: span {st[3]:.0f} x{base / st[3]:.2f} "
                                f"exact={int(st[4])} disp {int(st[5])} drop {int(st[6])} regrow {int(st[7])} "
                                f"head {int(st[10])}")
            print("   " + "\n   ".join(line))


if __name__ == "__main__":
    main()
