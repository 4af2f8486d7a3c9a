import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN_DIR, "crc32_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def data400():
    with open(os.path.join(GOLDEN_DIR, "400kb.txt"), "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def cuda():
    """The GPU device for -m gpu tests.  Fails (does not skip) without one."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("-m gpu tests need a GPU (torch.cuda.is_available() is False)")
    import chunkio_amd
    chunkio_amd.lib()   # raises if the HIP library is not built
    return torch.device("cuda:0")
