"""The multi-GPU exchange path on hardware: sharded.gather_counts / compact_offsets over a
1-rank RCCL process group (backend "nccl", the path bench.py --gpus N takes per GPU), compared
with the local computation.  The 8-GPU run itself is the driver's; the partitioning and the
2-rank exchanges are covered with gloo on CPU (tests/test_sharded.py)."""
import os
import socket

import numpy as np
import pytest

from cluster_tools_amd.watershed import sharded

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.fixture(scope='module')
def nccl_group():
    import torch
    import torch.distributed as dist
    os.environ.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % _free_port(), rank=0, world_size=1,
                            device_id=dev)
    yield dev
    dist.destroy_process_group()


def test_rccl_counts_scan(nccl_group):
    counts = np.array([5, 0, 17, 1, 3, 0, 9], np.int64)
    got = sharded.gather_counts(counts, device=nccl_group)
    np.testing.assert_array_equal(got, counts)
    offs, n = sharded.compact_offsets(got)
    np.testing.assert_array_equal(offs, np.concatenate([[0], np.cumsum(counts)[:-1]]))
    assert n == counts.sum()


def test_rccl_halo_exchange_single_rank(nccl_group):
    import torch
    vol = torch.arange(6 * 4 * 4, dtype=torch.int64, device=nccl_group).reshape(6, 4, 4)
    ref = vol.clone()
    out = sharded.exchange_z_halos(vol, 1, 1)   # no neighbour ranks: unchanged
    assert torch.equal(out, ref)
