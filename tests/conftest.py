import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: larger CPU cases")
    # the oracle libraries are built with the reference's -ffast-math, whose startup code sets flush-to-zero /
    # denormals-are-zero for the whole process, as in a RASR binary; numpy then reports a zero smallest subnormal
    config.addinivalue_line("filterwarnings",
                            "ignore:The value of the smallest subnormal for <class 'numpy.float64'> type is zero")


@pytest.fixture(scope="session")
def built():
    """Build the native library and the oracle once per session (no-op when up to date)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", ROOT, "all"], check=True)
    return True


@pytest.fixture(scope="session")
def gpu(built):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
