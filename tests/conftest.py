"""Shared pytest setup: import paths for the product binding (uc-tcp-ip_amd/netcsum.py) and the
test-only oracle (oracle/), the `gpu` marker, and on-demand builds of both libraries."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("", "uc-tcp-ip_amd", "oracle", "tests"):
    p = os.path.join(REPO, sub)
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session", autouse=True)
def _built_libraries():
    """Build oracle (gcc) and product (hipcc, gfx950) libraries if they are not present."""
    if not os.path.exists(os.path.join(REPO, "oracle", "build", "liboracle_netutil.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    if not os.path.exists(os.path.join(REPO, "uc-tcp-ip_amd", "libnetcsum_mi355x.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "uc-tcp-ip_amd")], check=True)
    yield


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
