"""Pass 2 of the two-pass watershed (`_ws_pass2`, two_pass_watershed.py:122-255) on the GPU
against the oracle, with the same initial seeds (pass-1 labels of the neighbours).

Bars: bit-exact against the oracle's flood model (the GPU's (C, d, label) order), and
VI <= 0.01 / adapted Rand <= 1e-3 against the vigra heap order (reference label 0 ignored
when a mask is used).
"""
import numpy as np
import pytest

from cluster_tools_amd.metrics import vi_scores, rand_scores
from oracle import oracle as O
from pass2_cases import SCENARIOS, scenario

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('name', sorted(SCENARIOS))
def test_pass2_matches_model_exactly(gpu_handle, name):
    config, block_shape, blocks = scenario(name)
    with O.flood_model():
        ref = O.ws_blocks(config, block_shape, blocks, pass_id=1)
    res = gpu_handle.ws_blocks(config, block_shape, blocks, pass_id=1)
    for r, g in zip(ref, res):
        assert g['status'] == r['status']
        np.testing.assert_array_equal(g['output'], r['output'])
        assert g['max_label'] == r['max_label']


@pytest.mark.parametrize('name', sorted(SCENARIOS))
def test_pass2_fragments_vi(gpu_handle, name):
    config, block_shape, blocks = scenario(name)
    ref = O.ws_blocks(config, block_shape, blocks, pass_id=1)
    res = gpu_handle.ws_blocks(config, block_shape, blocks, pass_id=1)
    for b, r, g in zip(blocks, ref, res):
        assert g['status'] == r['status'] == 0
        ign = [0] if b.get('mask') is not None else None
        vis, vim = vi_scores(g['output'], r['output'], ign)
        are, _ = rand_scores(g['output'], r['output'], ign)
        print('%s block %d: VI %.2e, ARE %.2e' % (name, b['block_id'], vis + vim, are))
        assert vis + vim <= 0.01
        assert are <= 1e-3
        # the initial seeds survive as ids of the output (stitching across the checkerboard)
        init = b['initial_seeds']
        ib, ish = b['inner_begin'], g['output'].shape
        sl = tuple(slice(a, a + s) for a, s in zip(ib, ish))
        halo_ids = set(np.unique(init[init != 0] & np.uint64(0xFFFFFFFF)).tolist())
        assert halo_ids & set(np.unique(g['output']).tolist()) or not halo_ids
        assert g['output'].shape == init[sl].shape


def test_pass2_empty_block_writes_nothing(gpu_handle):
    x = np.full((16, 40, 40), 0.7, np.float32)   # normalize -> all 0 < threshold: dt is None
    init = np.zeros(x.shape, np.uint64)
    init[:, :4] = 12345
    out = np.full((16, 32, 40), 9, np.uint64)
    b = dict(input=x, block_id=5, inner_begin=(0, 8, 0), inner_shape=(16, 32, 40), initial_seeds=init, out=out)
    res = gpu_handle.ws_blocks({}, (16, 32, 40), [b], pass_id=1)[0]
    assert res['status'] == 3
    assert (out == 9).all()


def test_pass2_device_path(gpu_handle):
    import torch
    config, block_shape, blocks = scenario('3d')
    host = gpu_handle.ws_blocks(config, block_shape, blocks, pass_id=1)
    dev = []
    for b in blocks:
        dev.append(dict(input=torch.from_numpy(b['input']).cuda(), block_id=b['block_id'],
                        inner_begin=b['inner_begin'],
                        initial_seeds=torch.from_numpy(b['initial_seeds'].view(np.int64)).cuda(),
                        output=torch.zeros(tuple(b['inner_shape']), dtype=torch.int64, device='cuda')))
    st = gpu_handle.ws_blocks_device(config, block_shape, dev, pass_id=1)
    for h, d, s in zip(host, dev, st):
        assert s[0] == 0
        assert np.array_equal(d['output'].cpu().numpy().view(np.uint64), h['output'])
