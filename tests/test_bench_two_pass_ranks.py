"""the bench's N-rank two-pass leg runs the workflow's sequential-equivalent
schedule.  Two ranks (sharing the GPU over gloo) and one rank run the same small two-pass
volume through bench.run_workload; the assembled labels must be identical, and the 2-rank run
must re-exchange the z halos after pass-2 levels (sharded.pass2_rank_schedule; the CPU proof of
the schedule is tests/test_pass2_ranks.py)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _run(world, out_dir):
    from bench import free_port
    port = str(free_port())
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, 'two_pass_ranks_worker.py'), out_dir],
                                      env=env))
    for p in procs:
        assert p.wait(timeout=300) == 0
    parts = []
    for r in range(world):
        meta = json.load(open(os.path.join(out_dir, 'rank%d_of%d.json' % (r, world))))
        parts.append((meta['z0'], np.load(os.path.join(out_dir, 'rank%d_of%d.npy' % (r, world))), meta))
    parts.sort(key=lambda p: p[0])
    return np.concatenate([p[1] for p in parts]), [p[2] for p in parts]


def test_two_ranks_equal_one_rank(tmp_path):
    one, m1 = _run(1, str(tmp_path))
    two, m2 = _run(2, str(tmp_path))
    assert one.shape == two.shape == (128, 128, 128)
    assert (one != 0).any()
    assert m1[0]['n_exchanges'] == 1 and all(m['n_exchanges'] > 1 for m in m2), (m1, m2)
    np.testing.assert_array_equal(one, two)
