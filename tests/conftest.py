import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "recommend-sys_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device; runs through the C-ABI")


@pytest.fixture(scope="session")
def ml100k():
    d = np.load(os.path.join(REPO, "tests", "golden", "ml100k.npz"))
    return (d["users"].astype(np.int64), d["items"].astype(np.int64),
            d["ratings"].astype(np.float64))


@pytest.fixture(scope="session")
def ctx():
    import rsgpu
    try:  # bring up torch's HIP runtime first: tests hand torch device buffers to the C-ABI
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except ImportError:
        pass
    c = rsgpu.Context(0)
    yield c
    c.close()
