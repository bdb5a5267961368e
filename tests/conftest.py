import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running parity case")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    # GPU tests must fail loudly on a GPU box when the extension is missing; on a CPU-only
    # container they are skipped only when explicitly deselected (-m "not gpu").
    pass


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.build()
    return O
