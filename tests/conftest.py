import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope="session")
def pkg():
    import _pkgload
    return _pkgload.load()


@pytest.fixture(scope="session")
def ref_tables():
    """PatchNorm tables fitted by the reference's own training path (golden)."""
    import torch
    from oracle import ref_cpu
    g = golden("patchnorm_ref.npz")
    return ref_cpu.NormTables(torch.from_numpy(g["n"]), torch.from_numpy(g["median"]), torch.from_numpy(g["b"]))
