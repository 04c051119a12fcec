import os
import sys
import pathlib

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pl-vi-orbslam3_amd"))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — parity tests through the C-ABI")
    config.addinivalue_line("markers", "slow: long-running CPU check")


def gpu_available():
    try:
        import plvi
        return plvi.load().plvi_device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib
    return oracle_lib.load()


@pytest.fixture(scope="session")
def plvi_lib():
    import plvi
    lib = plvi.load()
    if lib.plvi_device_count() <= 0:
        pytest.fail("gpu-marked test but no HIP device visible")
    return lib
