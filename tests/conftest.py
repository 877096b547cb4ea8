"""Test configuration: `gpu` marks tests that need a gfx950 device (run on the MI355X box with
`pytest -m gpu`); everything else runs on CPU (`pytest -m "not gpu"`)."""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")


@pytest.fixture(scope="session", autouse=True)
def _built():
    from opensearch_amd import build
    from oracle import oracle
    build.build(verbose=False)
    oracle.build()


_torch_cuda_ready = False


@pytest.fixture(autouse=True)
def _torch_cuda_first(request):
    """Initialise torch's HIP context before a GPU test's first native call: torch reports "No HIP GPUs are
    available" when libosknn initialised the device first in the process (seen when a torch-using GPU test
    runs on its own, -k), whereas the other order works."""
    global _torch_cuda_ready
    if not _torch_cuda_ready and request.node.get_closest_marker("gpu") is not None:
        try:
            import torch
            if torch.cuda.device_count() > 0:
                torch.cuda.init()
        except Exception:   # pragma: no cover - a GPU test then fails on its own terms
            pass
        _torch_cuda_ready = True
    yield
