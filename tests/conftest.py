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


def luigi_build(task, tmp_folder):
    """luigi.build, and on failure the failed jobs' error logs in the assertion message."""
    import glob
    from cluster_tools_amd import luigi_compat as luigi
    ok = luigi.build([task], local_scheduler=True)
    if not ok:
        msgs = []
        for p in sorted(glob.glob(os.path.join(str(tmp_folder), 'error_logs', '*.err'))):
            txt = open(p).read().strip()
            if txt and 'amdgpu.ids' not in txt.splitlines()[-1]:
                msgs.append('%s:\n%s' % (os.path.basename(p), txt[-2000:]))
        raise AssertionError('workflow failed\n' + '\n'.join(msgs))
