import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "python-audio-mastering_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    from oracle import mastering_oracle as mo
    mo.build()
    return mo


# identical-sample fractions of the GPU parity tests (printed at the end of the run,
# so the -q output of `pytest -m gpu` carries every test's measured exactness)
EXACTNESS = []


def record_exact(value, what="out"):
    test = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    EXACTNESS.append((test, what, float(value)))


def pytest_terminal_summary(terminalreporter):
    if EXACTNESS:
        terminalreporter.write_sep("-", "identical-sample fractions (GPU vs oracle / reference fixtures)")
        for test, what, v in EXACTNESS:
            terminalreporter.write_line(f"exact {v:.7f} {what:5s} {test}")
