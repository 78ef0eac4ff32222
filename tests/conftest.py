import os
import sys

import pytest

# the flood's fixpoint check runs in every test and a violation is an error
os.environ.setdefault('CTWS_VERIFY', '2')

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through libctws.so)")


@pytest.fixture(scope='session')
def gpu_handle():
    from cluster_tools_amd import ctws
    h = ctws.Handle(0)
    yield h
    h.close()
