import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "svt-av1-mirror_amd")
if PKG not in sys.path:
    sys.path.insert(0, PKG)
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def ref_available() -> bool:
    return os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libsvtref.so"))


@pytest.fixture(scope="session")
def svtme():
    import svtme as S

    return S


@pytest.fixture(scope="session")
def gpu(svtme):
    # torch's HIP runtime first (as bench.py does): tests allocate device and
    # pinned buffers with torch, whose lazy init fails after the library's
    import torch

    torch.cuda.set_device(0)
    g = svtme.GpuME(0)
    yield g
    g.close()
