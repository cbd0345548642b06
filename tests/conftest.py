import os
import sys

import pytest


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# every rsa_extend / rsa_seed call timed (the library samples one in 4 by default):
# the tests check per-kernel launch counts of single calls
os.environ.setdefault("RSA_KTIMER_EVERY", "1")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


@pytest.fixture(scope="session")
def root():
    return ROOT
