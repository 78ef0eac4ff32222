"""WatershedFromSeeds on the GPU (ctws_ws_from_seeds) vs the CPU oracle
(watershed/watershed_from_seeds.py:143-199 restated in oracle/ctws_oracle.cpp:orc_ws_from_seeds).

Bars: bit-exact against the oracle's flood model (the GPU's tie order; the order-preserving
seed compaction keeps ties ordered by seed VALUE, as the model orders them); VI <= 0.01 and
adapted Rand <= 1e-3 against vigra's heap order (label 0 ignored under a mask).  Edge cases
the reference's code paths have: ids above 2^20 and up to 2^32 - 2, a seed id spread over
disconnected blobs, 4-D input, uint8 input, a mask, no seed at all (vigra seeds from the hmap
minima), a size filter that removes every segment (auto-seeded regrow), and the
`max_id < uint32 max` assert (block failure)."""
import numpy as np
import pytest

from cluster_tools_amd.metrics import vi_scores, rand_scores
from cluster_tools_amd.synthetic import boundary_map, ellipsoid_mask
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SHAPE = (24, 80, 72)


def _seeds(shape, n, rng, max_id=5000, blob=1):
    s = np.zeros(shape, np.uint64)
    ids = np.unique(rng.integers(1, max_id, size=4 * n, dtype=np.int64))
    ids = rng.permutation(ids)[:n].astype(np.uint64)
    for k in range(n):
        c = [int(rng.integers(0, e)) for e in shape]
        sl = tuple(slice(max(0, ci - blob // 2), ci + (blob + 1) // 2) for ci in c)
        s[sl] = ids[k]
    return s


def _cases():
    from scipy.ndimage import gaussian_filter
    rng = np.random.default_rng(7)
    raw = boundary_map(SHAPE, seed=11)
    # a boundary-probability-like map: the synthetic map's clamped plateaus smoothed away
    x = gaussian_filter(raw, 1.0).astype(np.float32)
    c = {}
    c['points'] = (dict(size_filter=0), dict(input=x, seeds=_seeds(SHAPE, 60, rng)))
    c['blobs_big_ids_filter'] = (dict(size_filter=25),
                                 dict(input=x, seeds=_seeds(SHAPE, 80, rng, max_id=2 ** 32 - 2, blob=3)))
    s = _seeds(SHAPE, 40, rng, blob=2)
    s[s == s.max()] = 0
    s[2:4, 5:7, 5:7] = 77  # the same id on disconnected blobs
    s[20:22, 60:62, 60:62] = 77
    c['shared_id'] = (dict(size_filter=10), dict(input=x, seeds=s))
    m = ellipsoid_mask(SHAPE)
    c['mask'] = (dict(size_filter=25), dict(input=x, seeds=_seeds(SHAPE, 60, rng, blob=2), mask=m))
    x4 = np.stack([raw, boundary_map(SHAPE, seed=12)])
    c['4d_max'] = (dict(size_filter=25, agglomerate_channels='max'),
                   dict(input=x4, seeds=_seeds(SHAPE, 60, rng, blob=2)))
    xu = np.round(x * 255).astype(np.uint8)
    c['uint8'] = (dict(size_filter=25), dict(input=xu, seeds=_seeds(SHAPE, 60, rng, blob=2)))
    c['no_seeds'] = (dict(size_filter=0), dict(input=x, seeds=np.zeros(SHAPE, np.uint64)))
    c['filter_all'] = (dict(size_filter=10 ** 9), dict(input=x, seeds=_seeds(SHAPE, 30, rng)))
    c['raw_plateaus'] = (dict(size_filter=25), dict(input=raw, seeds=_seeds(SHAPE, 80, rng, blob=3)))
    # one flat plateau 64 x 4096 with three seeds: hop distances to the nearest seed up to 1,099
    # (tie order on a wide plateau; the floods that meet past kDMax = 4095 hops are the corridor
    # cases, tests/test_corridor_gpu.py)
    dp = np.zeros((1, 64, 4096), np.uint64)
    dp[0, 0, 0], dp[0, 63, 4095], dp[0, 40, 2000] = 9, 4, 7
    c['wide_plateau'] = (dict(size_filter=0), dict(input=np.full((1, 64, 4096), .5, np.float32), seeds=dp))
    return c


CASES = _cases()
# WatershedFromSeeds floods the normalized input itself (no smoothing): an input with exact
# plateaus — the synthetic map's clamped boundaries unsmoothed, or 256-level uint8 — is
# tie-dominated, and vigra orders equal priorities by binary-heap position, which no parallel
# schedule reproduces.  There the GPU must equal the flood model exactly and the whole VI gap to
# the heap order must be the model's tie order (gaps measured with the oracle: 4d_max 0.012,
# uint8 0.54, raw_plateaus 1.78; other tie orders: profiles/r05/tie_order_experiment.json).
TIE_GAP = {'4d_max': 0.02, 'uint8': 0.7, 'raw_plateaus': 2.0, 'wide_plateau': 1.8}  # wide_plateau: 1.774


@pytest.mark.parametrize('name', sorted(CASES))
def test_from_seeds_matches_oracle(gpu_handle, name):
    config, block = CASES[name]
    with O.flood_model():
        model = O.ws_from_seeds(config, [block])[0]
    ref = O.ws_from_seeds(config, [block])[0]
    res = gpu_handle.ws_from_seeds(config, [block])[0]
    assert res['status'] == ref['status'] == 0
    np.testing.assert_array_equal(res['output'], model['output'])
    ign = [0] if block.get('mask') is not None else None
    vis, vim = vi_scores(res['output'], ref['output'], ign)
    are, _ = rand_scores(res['output'], ref['output'], ign)
    print('%s: VI %.2e ARE %.2e exact-vs-heap %s' % (name, vis + vim, are, np.array_equal(res['output'], ref['output'])))
    if name in TIE_GAP:
        gap = sum(vi_scores(model['output'], ref['output'], ign))
        assert abs((vis + vim) - gap) <= 1e-9 and gap <= TIE_GAP[name], gap
    else:
        assert vis + vim <= 0.01 and are <= 1e-3
    assert res['max_label'] == int(res['output'].max())
    if name not in ('no_seeds', 'filter_all'):
        # every output id is one of the block's seed ids (labels map back to the values)
        assert set(np.unique(res['output'])) - {0} <= set(np.unique(block['seeds'])) - {0}


def test_from_seeds_overflow_fails_block(gpu_handle):
    x = boundary_map(SHAPE, seed=11)
    s = np.zeros(SHAPE, np.uint64)
    s[3, 3, 3] = 2 ** 32 - 1
    ok = dict(input=x, seeds=_seeds(SHAPE, 20, np.random.default_rng(1)))
    res = gpu_handle.ws_from_seeds({}, [dict(input=x, seeds=s), ok])
    ref = O.ws_from_seeds({}, [dict(input=x, seeds=s), ok])
    assert res[0]['status'] == ref[0]['status'] == 4  # CTWS_BLOCK_FAILED: the reference asserts
    assert res[1]['status'] == 0
    with O.flood_model():
        model = O.ws_from_seeds({}, [ok])[0]
    np.testing.assert_array_equal(res[1]['output'], model['output'])


def test_from_seeds_empty_mask_writes_nothing(gpu_handle):
    x = boundary_map(SHAPE, seed=11)
    out = np.full(SHAPE, 5, np.uint64)
    b = dict(input=x, seeds=_seeds(SHAPE, 10, np.random.default_rng(2)), mask=np.zeros(SHAPE, np.uint8), out=out)
    res = gpu_handle.ws_from_seeds({}, [b])[0]
    assert res['status'] == 1 and (out == 5).all()


def test_from_seeds_batch_equals_single(gpu_handle):
    """Several blocks of different shapes in one call give the per-block results."""
    rng = np.random.default_rng(3)
    blocks = []
    for i, sh in enumerate([(16, 64, 64), (10, 50, 90), (24, 80, 72)]):
        blocks.append(dict(input=boundary_map(sh, seed=20 + i), seeds=_seeds(sh, 30, rng, blob=2)))
    together = gpu_handle.ws_from_seeds({'size_filter': 25}, blocks)
    for b, t in zip(blocks, together):
        single = gpu_handle.ws_from_seeds({'size_filter': 25}, [b])[0]
        np.testing.assert_array_equal(single['output'], t['output'])
