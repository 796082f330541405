import faulthandler
import os
import sys
import time
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
for p in (REPO, REPO / "mlff-preconditioner_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = REPO / "tests" / "golden"

# Crash attribution.  Every test start is written (flushed, fsync'ed) to a progress
# file and, as one short line, to stderr, and a fatal signal dumps ALL Python threads
# to a file of its own, so that an abort inside native code names its test even when
# only the tail of the captured output survives.  MLFF_TEST_LOG_DIR overrides the
# directory (default <repo>/gpurun_out, which gpurun copies back).
_LOG_DIR = Path(os.environ.get("MLFF_TEST_LOG_DIR", REPO / "gpurun_out"))
_progress = None
_fault_file = None


def _open_logs():
    global _progress, _fault_file
    if _progress is not None:
        return
    try:
        _LOG_DIR.mkdir(parents=True, exist_ok=True)
        _progress = open(_LOG_DIR / "pytest_progress.log", "a", buffering=1)
        _fault_file = open(_LOG_DIR / "pytest_faulthandler.log", "a", buffering=1)
        _progress.write(f"=== session pid={os.getpid()} {time.strftime('%H:%M:%S')} argv={sys.argv}\n")
    except OSError:
        _progress = _fault_file = None


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libmlffpcg.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.hookimpl(trylast=True)
def pytest_sessionstart(session):
    # after pytest's own faulthandler plugin has pointed it at stderr: the all-thread
    # dump goes to a file, so stderr's tail keeps the progress lines and whatever the
    # runtime printed before aborting
    _open_logs()
    if _fault_file is not None:
        faulthandler.enable(file=_fault_file, all_threads=True)


def pytest_runtest_logstart(nodeid, location):
    line = f"[start {time.strftime('%H:%M:%S')}] {nodeid}"
    if _progress is not None:
        _progress.write(line + "\n")
        _progress.flush()
        os.fsync(_progress.fileno())
    if "gpu" in nodeid or os.environ.get("MLFF_TEST_PROGRESS"):
        sys.__stderr__.write(line + "\n")
        sys.__stderr__.flush()


def pytest_runtest_logfinish(nodeid, location):
    if _progress is not None:
        _progress.write(f"[done  {time.strftime('%H:%M:%S')}] {nodeid}\n")
        _progress.flush()


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def load_golden(golden_dir, name):
    """Committed reference fixture (data only: allow_pickle=False)."""
    import numpy as np

    return np.load(Path(golden_dir) / f"{name}.npz", allow_pickle=False)
