import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libphx.so HIP kernels)")


@pytest.fixture(scope="session")
def d0_manifest():
    from mladversarialobjectdetection_amd import _lib
    return _lib.Context("efficientdet-d0").manifest()


def pytest_sessionstart(session):
    """A line every 30 s while a GPU session runs (to stderr, or to the file PHX_HEARTBEAT names;
    PHX_HEARTBEAT=0 turns it off), so a long oracle comparison (a minute or more of fp64 CPU work
    inside one test) is not mistaken for a hung GPU job."""
    path = os.environ.get("PHX_HEARTBEAT", "stderr")
    if path == "0" or "gpu" not in (session.config.getoption("markexpr", "") or "") or \
            "not gpu" in session.config.getoption("markexpr", ""):
        return
    import threading
    import time

    def beat():
        t0 = time.time()
        while True:
            time.sleep(30)
            line = f"alive {time.time() - t0:.0f}s\n"
            if path == "stderr":
                sys.__stderr__.write(line)
                sys.__stderr__.flush()
            else:
                with open(path, "a") as f:
                    f.write(line)

    threading.Thread(target=beat, daemon=True).start()
