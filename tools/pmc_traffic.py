"""Per-launch HBM traffic of the roofline kernels from two separate
rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over tools/pmc_frame.py,
calibrated per MI355X_MICROARCH.md (HBM/rocprofv3): FETCH_SIZE reads 1/2 of
the bytes of 16-B/lane streams and other widths are uncalibrated, so the
calibration kernels (tools/calib/pmc_calib.hip) stream a known byte count
with the widths the kernels use and give the bytes-per-counted-byte factor:
  reads  of orb_blur_fast_kernel: dword loads  -> calib_dword_read
  writes of orb_blur_fast_kernel: dword stores -> calib_dword_copy (writes)
  reads  of lsd_prep_kernel:      dword loads  -> calib_dword_read
  writes of lsd_prep_kernel:      4/8-B stores -> calib_dword_copy / calib_dwordx2_store (mean)
  reads  of lbd_sobel0/1_kernel:  dword loads  -> calib_dword_read
  writes of lbd_sobel0_kernel:    dword blur stores (1 B/px) + 16-B Sobel stores (4 B/px): 1/5 dword, 4/5 dwordx4
  writes of lbd_sobel1_kernel:    4-B Sobel stores (short2 per pixel) -> calib_dword_copy
  reads  of orb_pyramid_kernel:   dword loads of level 0 -> calib_dword_read
  writes of orb_pyramid_kernel:   1 B per lane stores (levels 1..7) -> calib_byte_copy
A third pass (SQ_INSTS_VALU, SQ_INSTS_SALU, SQ_INSTS_LDS, SQ_WAVES; pmc_VALU/)
adds the per-launch wave-instruction counts of each kernel (valu_insts_per_launch
...), the numerator of bench.py's roofline.valu.
Writes profiles/<round>/pmc_traffic.json (a list, one entry per kernel) for bench.py.
usage: python tools/pmc_traffic.py <pmc_dir> profiles/r03 BATCH CAL_BYTES"""
import csv
import json
import pathlib
import sys
from collections import defaultdict


def per_kernel(path, counter):
    """KiB values per dispatch (FETCH_SIZE / WRITE_SIZE are KiB) -> bytes, by kernel."""
    out = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("plvi::", "")
            out[name].append(float(r["Counter_Value"]) * 1024.0)
    return out


def per_kernel_all(path):
    """{counter: {kernel: [value per dispatch]}} of one pass."""
    out = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("plvi::", "")
        out[r["Counter_Name"]][name].append(float(r["Counter_Value"]))
    return out


def main():
    d, dst, batch, cal_bytes = pathlib.Path(sys.argv[1]), pathlib.Path(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    fe = per_kernel(next(d.glob("pmc_FETCH_SIZE/**/*counter_collection.csv")), "FETCH_SIZE")
    wr = per_kernel(next(d.glob("pmc_WRITE_SIZE/**/*counter_collection.csv")), "WRITE_SIZE")
    mean = lambda v: sum(v) / len(v)  # noqa: E731
    f_rd = cal_bytes / mean(fe["calib_dword_read"])
    f_wr4 = cal_bytes / mean(wr["calib_dword_copy"])
    f_wr8 = cal_bytes / mean(wr["calib_dwordx2_store"])
    f_rd1 = cal_bytes / mean(fe["calib_byte_copy"])
    f_wr1 = cal_bytes / mean(wr["calib_byte_copy"])
    f_wr16 = cal_bytes / mean(wr["calib_dwordx4_store"]) if "calib_dwordx4_store" in wr else f_wr8
    calib = {"read_dword": f_rd, "read_byte": f_rd1, "write_dword": f_wr4, "write_dwordx2": f_wr8,
             "write_dwordx4": f_wr16, "write_byte": f_wr1,
             "note": "true bytes per counted byte, from calibration kernels streaming %d B" % cal_bytes}
    entries = []
    vp = list(d.glob("pmc_VALU/**/*counter_collection.csv"))
    sq = per_kernel_all(vp[0]) if vp else {}
    for k, fr, fw in (("orb_blur_fast_kernel", f_rd, f_wr4), ("lsd_prep_kernel", f_rd, (f_wr4 + f_wr8) / 2),
                      ("lbd_sobel0_kernel", f_rd, 0.2 * f_wr4 + 0.8 * f_wr16), ("lbd_sobel1_kernel", f_rd, f_wr4),
                      ("orb_pyramid_kernel", f_rd, f_wr1)):
        if k not in fe or k not in wr:
            continue
        if k == "lsd_prep_kernel":  # two launches per batch (octaves): mean of the first pair
            rf, rw = (fe[k][0] + fe[k][1]) / 2, (wr[k][0] + wr[k][1]) / 2
        else:
            rf, rw = mean(fe[k]), mean(wr[k])
        entries.append({"kernel": k, "batch": batch, "dispatches": [len(fe[k]), len(wr[k])],
                        "fetch_bytes_raw": rf, "write_bytes_raw": rw,
                        "fetch_bytes": rf * fr, "write_bytes": rw * fw, "bytes_per_launch": rf * fr + rw * fw,
                        "unit": "bytes per launch",
                        "calibration": calib})
        for c, field in (("SQ_INSTS_VALU", "valu_insts_per_launch"), ("SQ_INSTS_SALU", "salu_insts_per_launch"),
                         ("SQ_INSTS_LDS", "lds_insts_per_launch"), ("SQ_WAVES", "waves_per_launch")):
            v = sq.get(c, {}).get(k)
            if v:
                # lsd_prep: two launches per batch (octaves), the mean of the first pair
                entries[-1][field] = (v[0] + v[1]) / 2 if k == "lsd_prep_kernel" and len(v) > 1 else mean(v)
    dst.mkdir(parents=True, exist_ok=True)
    (dst / "pmc_traffic.json").write_text(json.dumps(entries, indent=1) + "\n")
    print(json.dumps(entries, indent=1))


if __name__ == "__main__":
    main()
