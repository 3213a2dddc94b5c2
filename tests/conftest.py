import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

_LAUNCHER = None


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")


def pytest_sessionstart(session):
    # Start the process launcher before any test initialises HIP in this process: node and
    # daemon processes are spawned through it (a HIP process must not fork+exec itself).
    global _LAUNCHER
    markexpr = session.config.getoption("markexpr") or ""
    if "not gpu" not in markexpr:
        from dora_amd.launcher import Launcher
        _LAUNCHER = Launcher()


def pytest_sessionfinish(session, exitstatus):
    if _LAUNCHER is not None:
        _LAUNCHER.close()


@pytest.fixture(scope="session")
def launcher():
    assert _LAUNCHER is not None, "launcher not started (run with -m gpu)"
    return _LAUNCHER


@pytest.fixture(scope="session")
def lib():
    from dora_amd import _lib
    return _lib.load()
