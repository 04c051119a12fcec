"""VALU / SALU / LDS census per kernel from gpurun_out/pmc_k_table.txt (tools/gpu_pmc_k.sh),
per launch-set (divide by REPS): python tools/census.py [REPS]"""
import re
import sys

reps = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
txt = open("gpurun_out/pmc_k_table.txt").read()
tot = 0
rows = []
for b in re.split(r"\n(?=\S)", txt):
    ls = b.strip().split("\n")
    d = {}
    for line in ls[1:]:
        m = re.match(r"\s+(\w+)\s+(\d+)", line)
        if m:
            d[m.group(1)] = int(m.group(2))
    v = d.get("SQ_INSTS_VALU", 0) / reps
    tot += v
    rows.append((v, ls[0][:34], d.get("SQ_INSTS_SALU", 0) / reps, d.get("SQ_INSTS_LDS", 0) / reps,
                 d.get("SQ_WAVE_CYCLES", 0) * 4 / reps))
for v, n, sa, ld, wc in sorted(rows, reverse=True)[:22]:
    print(f"{n:34s} valu {v / 1e9:7.2f}G  salu {sa / 1e9:6.2f}G lds {ld / 1e9:6.2f}G wavecyc {wc / 1e9:7.1f}G")
print("total valu/step %.2fG -> %.1f ms at one wave64 VALU op per 4 cycles per SIMD (1024 SIMDs, 2.4 GHz)"
      % (tot / 1e9, tot * 4 / (1024 * 2.4e9) * 1e3))
