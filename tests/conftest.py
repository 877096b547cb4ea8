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
