"""tools/timed_stats.py: per-kernel statistics of the window between bench.py's
two spin_kernel markers (the launch set the bench's roofline events average)."""
import csv
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _trace(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for r in rows:
            w.writerow(r)


def test_timed_window_only(tmp_path):
    rows = [
        ("void plvi::orb_blur_fast_kernel(int)", 0, 5_000_000),          # before: excluded
        ("spin_kernel(long)", 10_000_000, 10_001_000),
        ("void plvi::orb_blur_fast_kernel(int)", 10_002_000, 18_002_000),
        ("plvi::lsd_grow_kernel<false>(int)", 10_003_000, 40_003_000),
        ("void plvi::orb_blur_fast_kernel(int)", 50_000_000, 60_000_000),
        ("spin_kernel(long)", 70_000_000, 70_001_000),
        ("void plvi::orb_blur_fast_kernel(int)", 80_000_000, 99_000_000),  # after: excluded
    ]
    tr, out = tmp_path / "trace.csv", tmp_path / "stats.csv"
    _trace(tr, rows)
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "timed_stats.py"), str(tr), str(out)],
                       capture_output=True, text=True, check=True)
    assert "3 launches" in r.stdout
    stats = {row["Name"]: row for row in csv.DictReader(open(out))}
    blur = stats["plvi::orb_blur_fast_kernel"]
    assert int(blur["Calls"]) == 2 and float(blur["AverageNs"]) == 9_000_000
    assert int(stats["plvi::lsd_grow_kernel<false>"]["Calls"]) == 1


def test_no_markers_fails(tmp_path):
    tr = tmp_path / "trace.csv"
    _trace(tr, [("void plvi::orb_blur_fast_kernel(int)", 0, 1)])
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "timed_stats.py"), str(tr), str(tmp_path / "o.csv")],
                       capture_output=True, text=True)
    assert r.returncode != 0
