import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
for p in (REPO, REPO / "mlff-preconditioner_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = REPO / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libmlffpcg.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def load_golden(golden_dir, name):
    """Committed reference fixture (data only: allow_pickle=False)."""
    import numpy as np

    return np.load(Path(golden_dir) / f"{name}.npz", allow_pickle=False)
