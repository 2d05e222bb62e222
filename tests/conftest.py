import faulthandler
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); parity tests through the C ABI")


_FAULT_FILE = None


def pytest_sessionstart(session):
    """Fatal-signal tracebacks (SIGABRT / SIGSEGV) go to gpurun_out/faulthandler_<pid>.txt instead of stderr, so the
    tail of a crashed run's output ends with the RUN line of the test that was running and the native error message
    (glibc, HIP), not a Python stack dump of the pytest frames (GPUTEST_r05's record was cut exactly there)."""
    global _FAULT_FILE
    d = os.path.join(ROOT, "gpurun_out")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"faulthandler_{os.getpid()}.txt")
    _FAULT_FILE = open(path, "w")
    faulthandler.enable(file=_FAULT_FILE, all_threads=True)


def pytest_unconfigure(config):
    global _FAULT_FILE
    if _FAULT_FILE is not None:
        faulthandler.disable()
        _FAULT_FILE.close()
        _FAULT_FILE = None


def pytest_runtest_logstart(nodeid, location):
    # one unbuffered line per test on stderr: a crash record names the test it happened in
    os.write(2, f"RUN {nodeid}\n".encode())


@pytest.fixture(scope="session")
def O():
    from oracle import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu test needs a GPU (run with -m 'not gpu' on CPU)")
    torch.cuda.set_device(0)
    return torch.device("cuda:0")
