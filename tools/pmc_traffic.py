"""Per-launch HBM traffic of the roofline kernel from separate rocprofv3 --pmc
passes of the bench command (tools/gpu_session.sh: pmc_FETCH_SIZE/,
pmc_WRITE_SIZE/).  Writes profiles/<round>/pmc_traffic.json for bench.py.

FETCH_SIZE / WRITE_SIZE are KiB per dispatch (TCC_EA0_RDREQ/WRREQ based).
MI355X_MICROARCH.md: FETCH_SIZE counts 1/2 of the bytes of 16-B/lane
streaming reads; this kernel reads 1 B per lane (byte loads), a width the
guide leaves uncalibrated, so the raw value is reported, uncorrected, next
to the x2 reading for comparison.

usage: python tools/pmc_traffic.py gpurun_out profiles/r01 BATCH"""
import csv
import json
import pathlib
import sys

KERNEL = "orb_blur_fast_kernel"


def per_dispatch(path, counter):
    vals = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and KERNEL in r["Kernel_Name"]:
            vals.append(float(r["Counter_Value"]) * 1024.0)
    return vals


def main():
    out, dst, batch = pathlib.Path(sys.argv[1]), pathlib.Path(sys.argv[2]), int(sys.argv[3])
    fe = per_dispatch(out / "pmc_FETCH_SIZE" / "run_counter_collection.csv", "FETCH_SIZE")
    wr = per_dispatch(out / "pmc_WRITE_SIZE" / "run_counter_collection.csv", "WRITE_SIZE")
    f, w = sum(fe) / len(fe), sum(wr) / len(wr)
    d = {"kernel": KERNEL, "batch": batch, "dispatches": [len(fe), len(wr)], "fetch_bytes_raw": f,
         "fetch_bytes_x2": 2 * f, "write_bytes": w, "bytes_per_launch": f + w,
         "note": "FETCH_SIZE raw (byte-wide loads: the guide's x2 rule is for 16 B/lane reads) + WRITE_SIZE"}
    dst.mkdir(parents=True, exist_ok=True)
    (dst / "pmc_traffic.json").write_text(json.dumps(d, indent=1) + "\n")
    print(json.dumps(d))


if __name__ == "__main__":
    main()
