import os
import sys

import pytest

# One process drives up to 4 ranks on one GPU in the single-process ring tests;
# each rank's stream needs its own hardware queue for the kernels to be
# co-resident (HIP default is 4 queues per process).  Read at HIP init.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return np.load(os.path.join(ROOT, "tests", "golden", "reduce_golden.npz"))
