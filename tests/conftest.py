import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtdstar's HIP kernels)")


@pytest.fixture(scope="session")
def tt():
    import tonga

    return tonga.load()


@pytest.fixture(scope="session")
def orc():
    import oracle

    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def ds(tt):
    return tt.load_data_Tonga()


@pytest.fixture(scope="session")
def kat():
    return np.load(os.path.join(GOLDEN, "model_jld_kat.npz"), allow_pickle=False)
