"""GPU against the committed golden fixtures (tests/golden, made by scripts/make_golden.py from
the oracle and cross-checked by scripts/crosscheck_py39.py): normalized input and seeds
bit-exact, final blocks within VI <= 0.01 / ARand <= 1e-3 (bit-exact where the flood has no
exact ties)."""
import json
import os

import numpy as np
import pytest

from cluster_tools_amd.metrics import vi_scores, rand_scores

pytestmark = pytest.mark.gpu
GDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
INDEX = json.load(open(os.path.join(GDIR, 'index.json')))


@pytest.mark.parametrize('name', sorted(INDEX))
def test_gpu_reproduces_golden(gpu_handle, name):
    meta = INDEX[name]
    z = np.load(os.path.join(GDIR, name + '.npz'))
    b = dict(meta['block'], input=z['input'], block_id=meta['block_id'])
    if 'mask' in z.files:
        b['mask'] = z['mask']
    res = gpu_handle.ws_blocks(meta['config'], meta['block_shape'], [b])[0]
    assert res['status'] == meta['status']
    if meta['status'] != 0:
        assert np.array_equal(res['output'], z['output'])
        return
    shape = z['fin'].shape
    gpu_handle.debug_set_stop(1)
    try:
        gpu_handle.ws_blocks(meta['config'], meta['block_shape'], [b])
        fin = gpu_handle.debug_read('fin', 0, shape)
        seeds = gpu_handle.debug_read('labels', 0, shape) & np.uint32(0x7FFFFFFF)
    finally:
        gpu_handle.debug_set_stop(0)
    assert np.array_equal(fin, z['fin'])
    ref_seeds = z['seeds'].copy()
    if meta['config'].get('apply_ws_2d', True):   # GPU numbers seeds block-wide, slice-major
        n = 0
        for k in range(ref_seeds.shape[0]):
            s = ref_seeds[k]
            m = int(s.max())
            s[s > 0] += n
            n += m
    assert np.array_equal(seeds, ref_seeds)
    ign = [0] if 'mask' in z.files else None
    vis, vim = vi_scores(res['output'], z['output'], ign)
    assert vis + vim <= 0.01
    assert rand_scores(res['output'], z['output'], ign)[0] <= 1e-3
