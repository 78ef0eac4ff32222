"""Hop distances past the packed key's d range on the GPU.

The corridor blocks (tests/corridor.py) make the two floods meet ~9,800 hops from their seeds on
one exact hmap plateau, far past kDMax = 4095.  The packed flood must report the saturation
(BlockStat::dsat, ctws_dev.h note_dsat) and run_batch must flood those blocks again on the wide
keys (k_flood, 32-bit d): the result is then bit-exact against the unbounded flood model
(oracle/ctws_oracle.cpp:watersheds_model), and the handle's timings count the re-runs.  Each
test asserts both: the re-run happened and the output equals the model.  Reference semantics:
utils/volume_utils.py:123-139 (vu.watershed, apply_size_filter)."""
import numpy as np
import pytest

from corridor import CASES, FS_CASES, BLOCK_SHAPE, corridor_map, meeting_depth, run_model, run_model_fs
from cases import make_cases
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('name', sorted(CASES))
def test_corridor_ws_block(gpu_handle, name):
    cfg, blk = CASES[name]
    ref = run_model(name)
    res = gpu_handle.ws_blocks(cfg, BLOCK_SHAPE, [dict(blk, block_id=3)])[0]
    t = gpu_handle.timings()
    assert res['status'] == ref['status'] == 0
    assert t.get('flood_wide_reruns', 0) >= 1, t
    np.testing.assert_array_equal(res['output'], ref['output'])


@pytest.mark.parametrize('name', sorted(FS_CASES))
def test_corridor_from_seeds(gpu_handle, name):
    cfg, blk = FS_CASES[name]
    ref = run_model_fs(name)
    res = gpu_handle.ws_from_seeds(cfg, [blk])[0]
    t = gpu_handle.timings()
    assert res['status'] == ref['status'] == 0
    assert t.get('flood_wide_reruns', 0) >= 1, t
    np.testing.assert_array_equal(res['output'], ref['output'])
    a, seeds = corridor_map()
    assert meeting_depth(res['output'].astype(np.int64), a == 0, seeds) > 4095


def test_corridor_device_path(gpu_handle):
    import torch
    cfg, blk = CASES['2d_mask']
    ref = run_model('2d_mask')
    inp = torch.from_numpy(blk['input']).cuda()
    m = torch.from_numpy(blk['mask']).cuda()
    out = torch.zeros(blk['input'].shape, dtype=torch.int64, device='cuda')
    st = gpu_handle.ws_blocks_device(cfg, BLOCK_SHAPE, [dict(input=inp, mask=m, output=out, block_id=3)])
    assert st[0][0] == 0
    assert gpu_handle.timings().get('flood_wide_reruns', 0) >= 1
    np.testing.assert_array_equal(out.cpu().numpy().astype(np.uint64), ref['output'])


def test_corridor_in_a_batch(gpu_handle):
    """Only the saturated block is flooded again; the other blocks of the batch keep their packed
    result, and every block equals its model."""
    cases = make_cases()
    names = ['2d_default', '2d_sparse_fg']
    cfg = dict(CASES['2d'][0])
    blocks = [dict(cases[n][1], block_id=i + 1) for i, n in enumerate(names)]
    blocks.insert(1, dict(CASES['2d'][1], block_id=7))
    res = gpu_handle.ws_blocks(cfg, BLOCK_SHAPE, blocks)
    assert gpu_handle.timings().get('flood_wide_reruns', 0) == 1
    with O.flood_model():
        ref = O.ws_blocks(cfg, BLOCK_SHAPE, blocks)
    for r, m in zip(res, ref):
        assert r['status'] == m['status'] == 0
        np.testing.assert_array_equal(r['output'], m['output'])


@pytest.mark.parametrize('nd', [2, 3])
def test_corridor_pass2(gpu_handle, nd):
    """_ws_pass2 (two_pass_watershed.py:210-255) of a corridor block whose halo holds pass-1
    labels: the wide re-run keeps the pass-2 relabel and exclusions."""
    cfg = dict(CASES['2d' if nd == 2 else '3d'][0])
    a, seeds = corridor_map()
    init = np.zeros(a.shape, np.uint64)
    init[0, 0, :] = 12345  # pass-1 labels in the top halo row (a wall row)
    blk = dict(input=a, initial_seeds=init, block_id=5)
    with O.flood_model():
        ref = O.ws_blocks(cfg, BLOCK_SHAPE, [blk], pass_id=1)[0]
    res = gpu_handle.ws_blocks(cfg, BLOCK_SHAPE, [blk], pass_id=1)[0]
    assert res['status'] == ref['status']
    np.testing.assert_array_equal(res['output'], ref['output'])
