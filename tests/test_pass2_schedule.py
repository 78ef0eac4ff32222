"""Pass-2 batches by dependency level (watershed.pass2_levels / make_batches) give every block
exactly the ds_out[input_bb] the reference's sequential loop gives it
(two_pass_watershed.py:224-228, 296-299): simulated with a toy "watershed" whose output depends
on everything it reads, on checkerboard lists with halos (the config 5 geometry, scaled)."""
import numpy as np
import pytest

from cluster_tools_amd.utils.blocking import Blocking
from cluster_tools_amd.utils import volume_utils as vu
from cluster_tools_amd.watershed.watershed import pass2_levels, make_batches, _get_bbs, _overlaps


def _toy(block_id, seen):
    # output depends on every value read (order-sensitive checksum) and on the block id
    return np.uint64((int(np.uint64(seen.sum()) * np.uint64(1000003)) + block_id * 7919) % (1 << 40))


@pytest.mark.parametrize('shape,block_shape,halo', [
    ((32, 64, 64), (8, 16, 16), (2, 4, 4)),     # 4x4x4 grid, the config-5 halo ratio
    ((16, 48, 80), (8, 16, 16), (1, 8, 8)),     # 2x3x5 grid (even block count)
    ((24, 24, 24), (8, 12, 12), (4, 4, 4)),
])
def test_levels_match_sequential_loop(shape, block_shape, halo):
    blocking = Blocking([0, 0, 0], list(shape), list(block_shape))
    a, b = vu.make_checkerboard_block_lists(blocking)
    config = {'halo': list(halo)}
    rng = np.random.RandomState(0)
    pass1 = rng.randint(0, 1 << 20, size=shape).astype(np.uint64)
    for bid in a:
        _, _, ob = _get_bbs(blocking, bid, config)
        pass1[ob] += np.uint64(bid)
    # the reference: sequential loop over b
    seq = pass1.copy()
    for bid in b:
        ib, _, ob = _get_bbs(blocking, bid, config)
        seq[ob] = _toy(bid, seq[ib])
    # the batched schedule: each batch reads all its inputs, then writes all its outputs
    got = pass1.copy()
    batches = make_batches(blocking, b, config, 1, batch_blocks=3)
    assert sorted(x for bt in batches for x in bt) == sorted(b)
    for bt in batches:
        reads = {bid: got[_get_bbs(blocking, bid, config)[0]].copy() for bid in bt}
        for bid in bt:
            got[_get_bbs(blocking, bid, config)[2]] = _toy(bid, reads[bid])
    np.testing.assert_array_equal(got, seq)


def test_levels_separate_every_overlapping_pair():
    blocking = Blocking([0, 0, 0], [64, 128, 128], [16, 32, 32])
    _, b = vu.make_checkerboard_block_lists(blocking)
    config = {'halo': [4, 8, 8]}
    bbs = [_get_bbs(blocking, bid, config)[0::2] for bid in b]
    lv = pass2_levels(bbs)
    for j in range(len(b)):
        for i in range(j):
            if _overlaps(bbs[j][0], bbs[i][1]) or _overlaps(bbs[i][0], bbs[j][1]):
                assert lv[i] < lv[j]
    assert max(lv) + 1 < len(b)   # more parallel than one block per batch
