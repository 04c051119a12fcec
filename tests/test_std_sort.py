"""The product's libstdc++ std::sort restatement (csrc/std_sort.h, used by
the top-k line filter, src/LineExtractor.cc:75-84) vs the host std::sort on
tie-heavy inputs."""
import pathlib
import subprocess

ROOT = pathlib.Path(__file__).resolve().parent.parent


def test_std_sort_restatement_matches_host_libstdcxx():
    src = ROOT / "tests" / "native" / "sort_check.cpp"
    exe = ROOT / "tests" / "native" / "_build" / "sort_check"
    exe.parent.mkdir(exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), str(src)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
