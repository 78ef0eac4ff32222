"""Multi-process (world_size 2, gloo on CPU) tests of the block-sharding exchanges
(cluster_tools_amd/watershed/sharded.py):

* per-block label counts all-gathered + exclusively scanned give exactly the consecutive ids
  RelabelWorkflow's FindLabeling assigns (relabel/find_labeling.py:104-116) on the same
  blocks — including blocks with gaps in their ids, all-zero blocks, the constant-offset
  empty blocks and ranks holding different numbers of blocks;
* the two-pass z-halo exchange delivers each neighbour's boundary rows.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as tmp

from cluster_tools_amd.watershed import sharded

V = 4 * 16 * 16          # prod(block_shape) of the synthetic blocks
N_BLOCKS = 7             # odd: the two ranks hold 3 and 4 blocks


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _ws_like_outputs(seed=0):
    """Per-block uint64 outputs shaped like watershed outputs: block_id * V + local ids with
    gaps (size-filtered labels), some background 0, block 2 empty (constant offset), block 5
    all background."""
    rng = np.random.RandomState(seed)
    outs = []
    for b in range(N_BLOCKS):
        if b == 2:
            outs.append(np.full(V, b * V, np.uint64))
            continue
        if b == 5:
            outs.append(np.zeros(V, np.uint64))
            continue
        local = rng.choice(np.arange(1, V), size=rng.randint(5, 40), replace=False)
        x = (b * V + rng.choice(local, size=V)).astype(np.uint64)
        x[rng.rand(V) < 0.1] = 0
        outs.append(x)
    return outs


def _find_labeling_reference(outs):
    """FindUniques + FindLabeling + Write on the whole set, as the reference numbers them."""
    u = np.unique(np.concatenate(outs))
    start = 0 if u[0] == 0 else 1
    new = np.arange(start, start + len(u), dtype=np.uint64)
    lut = dict(zip(u.tolist(), new.tolist()))
    return [np.array([lut[v] for v in o.tolist()], np.uint64) for o in outs]


def _worker(rank, world, port, outdir):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        outs = _ws_like_outputs()
        mine = sharded.shard_blocks(list(range(N_BLOCKS)), rank, world)
        uniques = {b: np.unique(outs[b]) for b in mine}
        counts = [int((uniques[b] != 0).sum()) for b in mine]
        all_counts = sharded.gather_counts(counts)
        offs, n_ids = sharded.compact_offsets(all_counts)
        for b in mine:
            old, new = sharded.block_relabel_table(uniques[b], int(offs[b]))
            lut = dict(zip(old.tolist(), new.tolist()))
            np.save(os.path.join(outdir, 'block_%d.npy' % b), np.array([lut[v] for v in outs[b].tolist()], np.uint64))
        np.save(os.path.join(outdir, 'n_ids_%d.npy' % rank), np.array([n_ids]))
        # two-pass z-halo exchange: rank r's own rows hold 100 * r + row index
        hz, Z = 2, 5
        vol = torch.full((Z + 2 * hz, 3, 4), -1, dtype=torch.int64)
        for z in range(Z):
            vol[hz + z] = 100 * rank + z
        sharded.exchange_z_halos(vol, hz, hz)
        np.save(os.path.join(outdir, 'halo_%d.npy' % rank), vol.numpy())
    finally:
        dist.destroy_process_group()


def test_sharding_is_contiguous_and_complete():
    for n, w in ((7, 2), (256, 8), (3, 8)):
        parts = [sharded.shard_blocks(list(range(n)), r, w) for r in range(w)]
        assert sum(parts, []) == list(range(n))
        assert max(map(len, parts)) - min(map(len, parts)) <= 1


def test_compact_offsets_single_process_equals_find_labeling():
    outs = _ws_like_outputs(seed=3)
    ref = _find_labeling_reference(outs)
    uniques = [np.unique(o) for o in outs]
    offs, n_ids = sharded.compact_offsets([int((u != 0).sum()) for u in uniques])
    for o, u, off, r in zip(outs, uniques, offs, ref):
        old, new = sharded.block_relabel_table(u, int(off))
        lut = dict(zip(old.tolist(), new.tolist()))
        assert np.array_equal(np.array([lut[v] for v in o.tolist()], np.uint64), r)
    assert n_ids == max(int(r.max()) for r in ref)


def test_two_ranks_gloo_offsets_and_halo_exchange(tmp_path):
    world = 2
    tmp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    outs = _ws_like_outputs()
    ref = _find_labeling_reference(outs)
    for b in range(N_BLOCKS):
        got = np.load(tmp_path / ('block_%d.npy' % b))
        assert np.array_equal(got, ref[b]), b
    n0, n1 = (int(np.load(tmp_path / ('n_ids_%d.npy' % r))[0]) for r in range(world))
    assert n0 == n1 == max(int(r.max()) for r in ref)
    h0 = np.load(tmp_path / 'halo_0.npy')
    h1 = np.load(tmp_path / 'halo_1.npy')
    hz, Z = 2, 5
    assert (h0[:hz] == -1).all()                          # outer slab: untouched
    assert (h0[Z + hz:] == h1[hz:2 * hz]).all()            # rank 1's first own rows
    assert (h1[:hz] == h0[Z:Z + hz]).all()                 # rank 0's last own rows
    assert (h1[Z + hz:] == -1).all()


@pytest.mark.parametrize('cfg_id', [2, 3, 4, 5])
@pytest.mark.parametrize('world', [1, 2, 3, 8])
def test_strong_scaling_partition(cfg_id, world):
    """bench.py --scaling strong: the ranks' z-slabs partition the config's whole block grid --
    every block of the volume on exactly one rank, with its full halo inside the rank's
    generated region."""
    import bench
    cfg = bench.CONFIGS[cfg_id]
    full = tuple(cfg.get('full_shape', cfg['shape']))
    every = {b['block_id'] for b in bench.blocking(full, cfg['block_shape'], cfg['halo'])}
    seen = []
    for r in range(world):
        geo = bench.volume_geometry(cfg, r, world, 'strong')
        assert geo['full'] == full
        for b in geo['blocks']:
            assert 0 <= b['obeg'][0] and b['oend'][0] <= geo['gshape'][0]
            assert geo['lo'] <= b['beg'][0] < geo['gshape'][0] - geo['hi']
        seen += [b['block_id'] for b in geo['blocks']]
    assert sorted(seen) == sorted(every)


def _boxes_worker(rank, world, port, outdir):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        hz, Z = 2, 5
        vol = torch.full((Z + 2 * hz, 6, 8), -1, dtype=torch.int64)
        for z in range(Z):
            vol[hz + z] = (100 * rank + z) * 1000 + torch.arange(48).view(6, 8)
        # every rank sends box A down and box B up; receives the neighbours' opposite boxes
        a, b = [(0, 2, 1, 4)], [(3, 6, 0, 2), (1, 2, 6, 8)]
        sharded.exchange_z_halo_boxes(vol, hz, hz, a, b, b, a)
        np.save(os.path.join(outdir, 'boxes_%d.npy' % rank), vol.numpy())
    finally:
        dist.destroy_process_group()


def test_two_ranks_gloo_halo_exchange_boxes(tmp_path):
    """exchange_z_halo_boxes (the bench's two-pass levels after the first): only the listed
    (y, x) boxes of the halo rows change, with the neighbour's own rows there."""
    world, hz, Z = 3, 2, 5
    tmp.spawn(_boxes_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    own = lambda r, z: ((100 * r + z) * 1000 + np.arange(48).reshape(6, 8))  # noqa: E731
    for r in range(world):
        v = np.load(os.path.join(str(tmp_path), 'boxes_%d.npy' % r))
        exp = np.full(v.shape, -1, np.int64)
        for z in range(Z):
            exp[hz + z] = own(r, z)
        if r > 0:   # lower halo: rank r-1's last hz own rows, in the boxes r-1 sends up
            for y0, y1, x0, x1 in [(3, 6, 0, 2), (1, 2, 6, 8)]:
                for k in range(hz):
                    exp[k, y0:y1, x0:x1] = own(r - 1, Z - hz + k)[y0:y1, x0:x1]
        if r + 1 < world:   # upper halo: rank r+1's first hz own rows, in the box it sends down
            for y0, y1, x0, x1 in [(0, 2, 1, 4)]:
                for k in range(hz):
                    exp[hz + Z + k, y0:y1, x0:x1] = own(r + 1, k)[y0:y1, x0:x1]
        np.testing.assert_array_equal(v, exp)
