"""The relabel folded into the watershed jobs (cluster_tools_amd/watershed/job_relabel.py): two
job processes (gloo, world size 2) exchange their per-block id rows, scan, write their blocks
with the final ids, and job 0 writes the assignment table and maxId -- equal to RelabelWorkflow's
FindUniques + FindLabeling + Write (relabel/find_labeling.py:104-116, write/write.py:153-278)
restated with numpy, on watershed-like block outputs including: gaps in the local ids, an
all-background block, empty blocks (constant offset; block 0's is 0), a mask-skipped block
(nothing written), and the one id collision the id ranges allow (block b - 1's local label V
equals block b's bare offset b * V), which np.unique counts once."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as tmp

from cluster_tools_amd.watershed import job_relabel as jr

BLOCK = (2, 4, 8)
V = int(np.prod(BLOCK))
SHAPE = (2, 8, 32)   # 2 x 4 grid of blocks along y, x: 8 blocks


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _blocks():
    from cluster_tools_amd.utils.blocking import Blocking
    from cluster_tools_amd.utils import volume_utils as vu
    rng = np.random.RandomState(3)
    blocking = Blocking([0, 0, 0], list(SHAPE), list(BLOCK))
    out = {}
    for b in range(blocking.numberOfBlocks):
        bb = vu.block_to_bb(blocking.getBlock(b))
        if b == 0:
            lab = np.zeros(BLOCK, np.uint64)                 # empty block 0: constant offset 0
        elif b == 3:
            lab = np.full(BLOCK, b * V, np.uint64)           # empty block: bare offset
        elif b == 5:
            lab = None                                       # mask-skipped: nothing written
        else:
            loc = rng.choice(np.arange(1, V), size=6, replace=False)
            lab = (b * V + rng.choice(loc, size=V)).astype(np.uint64).reshape(BLOCK)
            lab.ravel()[rng.rand(V) < 0.2] = 0
            if b == 2:
                lab.ravel()[0] = 3 * V                       # local label V: collides with block 3
        out[b] = (bb, lab)
    return out


def _reference(blocks):
    vol = np.zeros(SHAPE, np.uint64)
    for b, (bb, lab) in blocks.items():
        if lab is not None:
            vol[bb] = lab
    u, inv = np.unique(vol, return_inverse=True)
    start = 0 if u[0] == 0 else 1
    new = (inv.reshape(SHAPE) + start).astype(np.uint64)
    return vol, new, np.stack([u, np.arange(start, start + len(u), dtype=np.uint64)], 1)


def _worker(rank, world, port, root, fail_rank=-1):
    from cluster_tools_amd.utils import volume_utils as vu
    jr.init_group(rank, world, port, 'gloo', timeout_s=120)
    try:
        blocks = _blocks()
        mine = [b for b in sorted(blocks) if b % world == rank]   # block_list[job::n_jobs]
        results = []
        for b in mine:
            bb, lab = blocks[b]
            results.append((b, bb, None if lab is None else lab.copy(), None if lab is None else np.unique(lab)))

        def mapper(lab, keys, vals):
            if rank == fail_rank:
                raise OSError("injected write failure")
            nz = lab != 0
            if len(keys):
                lab[nz] = vals[np.searchsorted(keys, lab[nz])]
            return lab

        with vu.file_reader(os.path.join(root, 'ws.n5')) as f:
            ds = f['ws']
            try:
                jr.relabel_in_job(rank, results, ds, root, os.path.join(root, 'ws.n5'), 'relabel_watershed',
                                  mapper, log=lambda m: None)
            except Exception as e:
                if fail_rank < 0:
                    raise
                with open(os.path.join(root, 'err_%d.txt' % rank), 'w') as fe:
                    fe.write(str(e))
    finally:
        dist.destroy_process_group()


def test_scan_counts_the_collision_once():
    offs, n = jr.scan([[2, 3, 10, 20, 0], [3, 2, 20, 24, 1], [1, 0, -1, -1, 1], [5, 1, 40, 40, 0]])
    assert offs[2] == (0, 0) and offs[3] == (3, 1) and offs[5] == (4, 0) and n == 5
    k, v = jr.block_table(np.array([0, 20, 24], np.uint64), *offs[3])
    assert k.tolist() == [20, 24] and v.tolist() == [3, 4]   # 20 keeps block 2's new id 3


def test_two_jobs_relabel_like_relabel_workflow(tmp_path):
    from cluster_tools_amd.utils import volume_utils as vu
    root = str(tmp_path)
    with vu.file_reader(os.path.join(root, 'ws.n5')) as f:
        f.create_dataset('ws', shape=SHAPE, dtype='uint64', chunks=BLOCK)
    # the file-store rendezvous the watershed task hands its jobs (watershed.relabel_job_config)
    tmp.spawn(_worker, args=(2, 'file://' + os.path.join(root, 'rendezvous'), root), nprocs=2, join=True)
    vol, new, table = _reference(_blocks())
    with vu.file_reader(os.path.join(root, 'ws.n5'), 'r') as f:
        got = f['ws'][:]
        assert f['ws'].attrs['maxId'] == int(new.max())
        got_table = f['relabel_watershed'][:]
    np.testing.assert_array_equal(got, new)
    np.testing.assert_array_equal(got_table, table)
    assert not any(n.startswith('watershed_relabel_rows') for n in os.listdir(root))



def test_a_job_failing_while_writing_fails_every_job_fast(tmp_path):
    """a job that raises after the id exchange (here in its block mapping) must not
    leave its peers in the final barrier until the group timeout: every job raises."""
    import time
    from cluster_tools_amd.utils import volume_utils as vu
    root = str(tmp_path)
    with vu.file_reader(os.path.join(root, 'ws.n5')) as f:
        f.create_dataset('ws', shape=SHAPE, dtype='uint64', chunks=BLOCK)
    t0 = time.time()
    tmp.spawn(_worker, args=(2, _free_port(), root, 1), nprocs=2, join=True)
    assert time.time() - t0 < 60
    assert open(os.path.join(root, 'err_1.txt')).read() == "injected write failure"
    assert "failed while writing its blocks" in open(os.path.join(root, 'err_0.txt')).read()
