"""The frontier relaxation's schedule knobs change the order of work, never the result.

The flood's fixpoint (K = f(min of the neighbours' keys), k_flood.hip) is unique, so every
chunk brick (CTWS_FRONTIER_CHUNK2D / _3D), a one-sweep limit (CTWS_FRONTIER_REPS=1: every changed chunk hits the limit, so the
non-converged re-queue path runs), the masked-plateau fill switched off (CTWS_PLATEAU_FILL=0) and the wide keys
(CTWS_FORCE_WIDE=1) must reproduce the oracle's flood model bit for bit on every
parity case, as the default schedule does (test_gpu_parity.py::test_flood_matches_model_exactly).
The knobs are read when a handle is opened.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
from cases import make_cases, BLOCK_SHAPE

pytestmark = pytest.mark.gpu

CASES = make_cases()
VARIANTS = {
    'bricks_a': {'CTWS_FRONTIER_CHUNK2D': '4x16x1', 'CTWS_FRONTIER_CHUNK3D': '1x32x2'},
    'bricks_b': {'CTWS_FRONTIER_CHUNK3D': '8x8x1'},
    'rows_3d_one_sweep': {'CTWS_FRONTIER_CHUNK3D': '8x8x1', 'CTWS_FRONTIER_REPS': '1'},
    'one_sweep': {'CTWS_FRONTIER_REPS': '1'},
    # masked blocks' plateaus relaxed hop by hop instead of filled by run scans (k_plateau.hip)
    'no_plateau_fill': {'CTWS_PLATEAU_FILL': '0'},
    # cropped blocks' uint64 output through the word-tiled k_output instead of k_output_crop
    'output_words': {'CTWS_OUTPUT_TILE': '0'},
    # every flood on the wide keys (k_flood, labels apart, 32-bit d): the path run_batch re-runs a
    # block on when its packed flood saturated d (tests/test_corridor_gpu.py)
    'wide_keys': {'CTWS_FORCE_WIDE': '1'},
    # the size filter's regrow initialised by the scan of every voxel instead of the walk over
    # the removed segments (k_sf_sparse, the default for size_filter <= 64)
    'sf_scan': {'CTWS_SF_SPARSE': '0'},
    # the seed components by the tile CC (k_tile_cc / k_tile_merge<.., CC_SEED>) instead of from
    # the classes (k_seed_members: 3-D the plateau CC's maximal plateaus, 2-D maxima as roots and
    # the listed plateau maxima united, k_seed_union2; the default)
    'seed_tilecc': {'CTWS_SEED_TILECC': '1'},
}


@pytest.fixture(scope='module', params=sorted(VARIANTS))
def variant_handle(request):
    from cluster_tools_amd import ctws
    env = VARIANTS[request.param]
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        h = ctws.Handle(0)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    yield h
    h.close()


_REF = {}


def _model(name):
    if name not in _REF:
        config, block = CASES[name]
        with O.flood_model():
            _REF[name] = O.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=3)])[0]
    return _REF[name]


@pytest.mark.parametrize('name', sorted(CASES))
def test_variant_matches_model(variant_handle, name):
    config, block = CASES[name]
    ref = _model(name)
    res = variant_handle.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=3)])[0]
    assert res['status'] == ref['status']
    np.testing.assert_array_equal(res['output'], ref['output'])


_REF2 = {}


@pytest.mark.parametrize('name', ['2d', '3d', '3d_mask', '2d_collide'])
def test_variant_pass2_matches_model(variant_handle, name):
    """_ws_pass2 under every knob: pass 2's size filter keeps the excluded initial ids whatever
    their size, on the sparse walk (first positions of the relabelled ids) and on the scan."""
    from pass2_cases import scenario
    config, block_shape, blocks = scenario(name)
    if name not in _REF2:
        with O.flood_model():
            _REF2[name] = O.ws_blocks(config, block_shape, blocks, pass_id=1)
    res = variant_handle.ws_blocks(config, block_shape, blocks, pass_id=1)
    for r, g in zip(_REF2[name], res):
        assert g['status'] == r['status']
        np.testing.assert_array_equal(g['output'], r['output'])
