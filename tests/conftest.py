import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long CPU reference runs")


@pytest.fixture(scope="session")
def restatement():
    from oracle_lib import Restatement, restatement_available
    if not restatement_available():
        pytest.skip("oracle restatement not built (make -C oracle restatement)")
    return Restatement()
