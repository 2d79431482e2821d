import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def oracle():
    """The CPU restatement (test infrastructure), built on demand."""
    from tests.oracle_bind import Oracle
    return Oracle.load(build=True)


@pytest.fixture(scope="session")
def ref_available():
    return os.path.isdir("/root/reference/src")
