import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: large-size parity (GPU box)")


@pytest.fixture(scope="session", autouse=True)
def built_libraries():
    """Incremental `make` so the in-tree C-ABI libraries and the oracle exist (no-op when up to date)."""
    r = subprocess.run(["make", "-s", "-C", ROOT, "all"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.exit(f"make failed:\n{r.stdout}\n{r.stderr}", returncode=2)
    yield


@pytest.fixture(scope="session")
def torch_cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but torch sees no GPU (run with -m 'not gpu' on a CPU-only host)")
    return torch


@pytest.fixture
def gpu_knob():
    """set(name, value): a netc_gpu_knob (include/ws/mask.h) for this test, restored to its
    default afterwards (None leaves it alone)."""
    from netc_amd import mask as nm

    touched = []

    def set_(name, value):
        if value is None:
            return
        nm.set_knob(name, int(value))
        touched.append(name)

    yield set_
    for name in touched:
        nm.set_knob(name, -1)
