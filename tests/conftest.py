import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests through the C-ABI")


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle

    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def gpu():
    """torch (imported first, so it owns the HIP runtime) + the loaded product library."""
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test on a machine without a GPU (run with -m 'not gpu')")
    torch.cuda.set_device(0)
    torch.empty(1, device="cuda")  # initialise the runtime before loading the library
    from cocytus_amd import ec

    ec.lib()
    rc = ec.device_check()
    assert rc == ec.CEC_OK, ec.lib().cec_last_error()
    return torch, ec
