"""GPU (libctws.so, gfx950 kernels) vs CPU oracle on the same inputs.

Bars (BASELINE.json north_star): threshold mask / normalized input, EDT, seed map, hmap and
seed labelling bit-exact; final fragments VI (split + merge, log2) <= 0.01 and adapted Rand
error <= 1e-3 against the oracle, reference label 0 ignored when a mask is used
(evaluation/evaluation_workflow.py:53,60).
"""
import os

import numpy as np
import pytest

from cluster_tools_amd.metrics import vi_scores, rand_scores
from oracle import oracle as O
from cases import make_cases, BLOCK_SHAPE

pytestmark = pytest.mark.gpu

CASES = make_cases()
VI_TOL = 0.01
ARE_TOL = 1e-3
# Inputs whose hmap is dominated by exact ties (4-level quantized, no smoothing): vigra orders
# equal priorities by binary-heap position, which no deterministic parallel schedule
# reproduces.  There the GPU must equal the flood model exactly (test_flood_matches_model_
# exactly), the whole VI gap must be the model's tie order (VI(GPU, heap) == VI(model, heap)),
# and the gap stays below the recorded synthetic worst case.  Every BASELINE
# config meets the VI bar itself (tests/test_config_blocks.py).  The sparse-foreground cases
# are tie-dominated too: a distance transform of a few isolated points has exactly equal
# values on every symmetric position.
TIE_DOMINATED = {'3d_plateaus': 1.2, '2d_sparse_fg': 0.1, '3d_sparse_fg': 0.2}


def _oracle_seeds(config, dt):
    if not config.get('apply_ws_2d', True):
        return O.make_seeds(dt, config)
    out = np.zeros(dt.shape, np.uint32)
    n = 0
    for z in range(dt.shape[0]):
        s = O.make_seeds(dt[z], config)
        s[s > 0] += n
        n = max(n, int(s.max()))
        out[z] = s
    return out


def _oracle_hmap(config, fin, dt):
    if not config.get('apply_ws_2d', True):
        return O.make_hmap(fin, dt, config)
    return np.stack([O.make_hmap(fin[z], dt[z], config) for z in range(dt.shape[0])])


@pytest.mark.parametrize('name', sorted(CASES))
def test_stages_bit_exact(gpu_handle, name):
    config, block = CASES[name]
    ref = O.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=3)], with_stages=True)[0]
    shape = ref['input'].shape
    gpu_handle.debug_set_stop(1)
    try:
        gpu_handle.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=3)])
        fin = gpu_handle.debug_read('fin', 0, shape)
        dt = gpu_handle.debug_read('dt', 0, shape)
        hm = gpu_handle.debug_read('hmap', 0, shape)
        seeds = gpu_handle.debug_read('labels', 0, shape) & np.uint32(0x7FFFFFFF)
    finally:
        gpu_handle.debug_set_stop(0)
    assert np.array_equal(fin, ref['input']), 'normalized input / threshold input differs'
    np.testing.assert_array_equal(dt, ref['dt'])
    np.testing.assert_array_equal(hm, _oracle_hmap(config, ref['input'], ref['dt']))
    np.testing.assert_array_equal(seeds, _oracle_seeds(config, ref['dt']))


@pytest.mark.parametrize('name', sorted(CASES))
def test_flood_matches_model_exactly(gpu_handle, name):
    """The GPU flood computes the (C, d, label) fixpoint: bit-exact vs the oracle's model,
    after the first flood and for the final uint64 block."""
    config, block = CASES[name]
    with O.flood_model():
        ref = O.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=3)], with_stages=True)[0]
    res = gpu_handle.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=3)])[0]
    assert res['status'] == ref['status']
    np.testing.assert_array_equal(res['output'], ref['output'])
    if ref['status'] == 0:
        gpu_handle.debug_set_stop(3)
        try:
            gpu_handle.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=3)])
            ws = gpu_handle.debug_read('labels', 0, ref['ws'].shape)
        finally:
            gpu_handle.debug_set_stop(0)
        np.testing.assert_array_equal(ws, ref['ws'])


@pytest.mark.parametrize('name', sorted(CASES))
def test_fragments_vi(gpu_handle, name):
    config, block = CASES[name]
    ref = O.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=3)])[0]
    res = gpu_handle.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=3)])[0]
    assert res['status'] == ref['status']
    out, gt = res['output'], ref['output']
    ign = [0] if block.get('mask') is not None else None
    vis, vim = vi_scores(out, gt, ign)
    are, _ = rand_scores(out, gt, ign)
    print('%s: VI split %.2e merge %.2e, ARE %.2e, exact %s' % (name, vis, vim, are, np.array_equal(out, gt)))
    if name in TIE_DOMINATED:
        with O.flood_model():
            model = O.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=3)])[0]
        gap = sum(vi_scores(model['output'], gt, ign))
        print('%s: tie-dominated, VI(model, heap) %.3f' % (name, gap))
        assert abs((vis + vim) - gap) <= 1e-9, (vis + vim, gap)
        assert gap <= TIE_DOMINATED[name], gap
        return
    assert vis + vim <= VI_TOL, (vis, vim)
    assert are <= ARE_TOL, are
    # ids live in this block's offset range; masked voxels are 0 (watershed.py:331-337)
    off = 3 * int(np.prod(BLOCK_SHAPE))
    if block.get('mask') is None:
        assert out.min() > off
    else:
        assert (out[out != 0] > off).all()


def test_empty_block_constant_offset(gpu_handle):
    x = np.full((16, 40, 40), 0.7, np.float32)   # constant: normalize -> all 0 < threshold
    # masked-out voxels become boundary (input 1, watershed.py:301-303): only a full mask
    # keeps the block empty; a partial mask makes it a regular block
    for mask, status in ((None, 2), (np.ones(x.shape, np.uint8), 2), (np.ones(x.shape, np.uint8), 0)):
        if status == 0:
            mask[:8] = 0
        b = dict(input=x, block_id=5, mask=mask, inner_begin=(2, 3, 4), inner_shape=(12, 30, 30),
                 crop_relabel=True)
        ref = O.ws_blocks({}, BLOCK_SHAPE, [b])[0]
        res = gpu_handle.ws_blocks({}, BLOCK_SHAPE, [b])[0]
        assert res['status'] == ref['status'] == status
        assert np.array_equal(res['output'], ref['output'])


def test_empty_inner_mask_skips_block(gpu_handle):
    x = CASES['3d_default'][1]['input']
    m = np.zeros(x.shape, np.uint8)
    m[:, :4] = 1  # only in the halo
    out = np.full((20, 64, 64), 7, np.uint64)
    b = dict(input=x, mask=m, inner_begin=(2, 16, 16), inner_shape=(20, 64, 64), crop_relabel=True, out=out)
    res = gpu_handle.ws_blocks({}, BLOCK_SHAPE, [b])[0]
    assert res['status'] == 1
    assert (out == 7).all()


def test_batch_of_mixed_blocks_equals_single_blocks(gpu_handle):
    """Several blocks of different shapes in one launch give the per-block results."""
    from cluster_tools_amd.synthetic import boundary_map
    cfg = dict(apply_dt_2d=False, apply_ws_2d=False)
    blocks = [dict(input=boundary_map(s, seed=i), block_id=i)
              for i, s in enumerate([(32, 96, 96), (20, 70, 130), (32, 96, 40)])]
    together = gpu_handle.ws_blocks(cfg, BLOCK_SHAPE, blocks)
    for b, t in zip(blocks, together):
        single = gpu_handle.ws_blocks(cfg, BLOCK_SHAPE, [b])[0]
        assert np.array_equal(single['output'], t['output'])
        ref = O.ws_blocks(cfg, BLOCK_SHAPE, [b])[0]
        vis, vim = vi_scores(t['output'], ref['output'])
        assert vis + vim <= VI_TOL


def test_device_path_matches_host_path(gpu_handle):
    import torch
    config, block = CASES['3d_aniso_halo']
    host = gpu_handle.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=2)])[0]
    inp = torch.from_numpy(block['input']).cuda()
    out = torch.zeros(block['inner_shape'], dtype=torch.int64, device='cuda')
    st = gpu_handle.ws_blocks_device(config, BLOCK_SHAPE, [dict(input=inp, output=out, block_id=2,
                                                                 inner_begin=block['inner_begin'],
                                                                 crop_relabel=True)])
    assert st[0][0] == 0
    assert np.array_equal(out.cpu().numpy().astype(np.uint64), host['output'])


def test_deterministic(gpu_handle):
    config, block = CASES['3d_plateaus']
    a = gpu_handle.ws_blocks(config, BLOCK_SHAPE, [dict(block)])[0]['output']
    b = gpu_handle.ws_blocks(config, BLOCK_SHAPE, [dict(block)])[0]['output']
    assert np.array_equal(a, b)


@pytest.mark.parametrize('name', ['2d_sparse_fg', '3d_sparse_fg', '3d_plateaus', '2d_plateaus', '2d_empty_slice', '2d_default'])
def test_seeds_repeatable(gpu_handle, name):
    """The seed stage (plateau CC, seed CC, scan-order ranks: concurrent union-find) gives the
    same labels on every run: 8 runs of one block in a batch of 3 copies, each equal to the
    oracle's seeds.  (The 2-D seed union over the listed plateau maxima, in its first form with
    plain parent loads and path halving, returned a stray root label on 2d_sparse_fg in about one
    run in 24)"""
    config, block = CASES[name]
    ref = O.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=3)], with_stages=True)[0]
    want = _oracle_seeds(config, ref['dt'])
    shape = ref['input'].shape
    gpu_handle.debug_set_stop(1)
    try:
        for _ in range(int(os.environ.get('CTWS_TEST_REPS', '8'))):
            gpu_handle.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=3 + k) for k in range(3)])
            for b in range(3):
                seeds = gpu_handle.debug_read('labels', b, shape) & np.uint32(0x7FFFFFFF)
                np.testing.assert_array_equal(seeds, want)
    finally:
        gpu_handle.debug_set_stop(0)


@pytest.mark.parametrize('name', ['2d_sparse_fg', '3d_sparse_fg', '3d_plateaus', '2d_empty_slice', '3d_mask_halo',
                                  '2d_sizefilter_noise_halo'])
def test_pipeline_repeatable(gpu_handle, name):
    """The whole block (plateau / seed / crop CCs: global union-find merges across workgroups,
    the flood's fixpoint, the size filter) gives the same uint64 output on every run: 8 runs of a
    batch of 3 copies of the block."""
    config, block = CASES[name]
    first = None
    for _ in range(int(os.environ.get('CTWS_TEST_REPS', '8'))):
        res = gpu_handle.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=3) for _ in range(3)])
        for r in res:
            if first is None:
                first = r['output'].copy()
            np.testing.assert_array_equal(r['output'], first)


def test_config2_block_full_size(gpu_handle):
    """One full 64x256x256 block of the bench workload against the oracle."""
    from cluster_tools_amd.synthetic import boundary_map
    x = boundary_map((64, 256, 256), seed=0)
    cfg = dict(apply_dt_2d=False, apply_ws_2d=False)
    ref = O.ws_blocks(cfg, BLOCK_SHAPE, [dict(input=x, block_id=1)])[0]
    res = gpu_handle.ws_blocks(cfg, BLOCK_SHAPE, [dict(input=x, block_id=1)])[0]
    vis, vim = vi_scores(res['output'], ref['output'])
    assert vis + vim <= VI_TOL
    assert rand_scores(res['output'], ref['output'])[0] <= ARE_TOL


def test_refusals_are_per_block(gpu_handle):
    """A block the reference would fail on (vigra: kernel longer than line) fails alone: the
    other blocks of the call are written, as the reference job writes the blocks before the one
    that raises."""
    config, block = CASES['3d_default']
    short = dict(input=np.ascontiguousarray(block['input'][:4]), block_id=5)   # Z = 4 < radius 6 + 1
    res = gpu_handle.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=3), short, dict(block, block_id=4)])
    assert [r['status'] for r in res] == [0, 4, 0]
    ref = O.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=4)])[0]
    vis, vim = vi_scores(res[2]['output'], ref['output'])
    assert vis + vim <= VI_TOL


def test_edt_integer_sqrt_exhaustive(gpu_handle):
    """The EDT's final sqrt (k_edt.hip sqrt_rn_int: v_sqrt_f32 + exact integer midpoint tests)
    equals the correctly rounded float32 sqrt (vigra: sqrt on the float32 dest) for every squared
    distance n < 2^24."""
    n = 1 << 24
    got = gpu_handle.debug_sqrt_int(0, n)
    want = np.sqrt(np.arange(n, dtype=np.float64)).astype(np.float32)  # double sqrt -> float: correctly rounded
    bad = np.flatnonzero(got.view(np.uint32) != want.view(np.uint32))
    assert bad.size == 0, (bad[:10], got[bad[:10]], want[bad[:10]])
