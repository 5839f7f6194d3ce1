import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def pytest_terminal_summary(terminalreporter):
    from tests import parity_log
    if parity_log.ENTRIES:
        terminalreporter.write_sep("-", "observed parity per case (GPU vs oracle)")
        for line in parity_log.lines():
            terminalreporter.write_line(line)


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.build(ref=True)
    return oracle


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
