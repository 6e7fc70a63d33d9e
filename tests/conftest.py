import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the oracle (gcc) if needed; the HIP library is built by __graft_entry__.build()."""
    so = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(so):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    yield


@pytest.fixture(scope="session")
def nyc_zones():
    import mosaic_amd as M
    return M.Polygons.from_npz(os.path.join(GOLDEN, "nyc_taxi_zones.npz"))


@pytest.fixture(scope="session")
def nyc_chips_r9(nyc_zones):
    import mosaic_amd as M
    return M.tessellate(nyc_zones, M.H3IndexSystem(), 9)


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)
