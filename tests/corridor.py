"""A serpentine corridor: hop distances on one equal-height plateau far beyond the packed flood
key's 12-bit d field (kDMax = 4095, cluster_tools_amd/csrc/ctws_dev.h).

Boundary walls (input 1) enclose two 9 x 9 rooms joined by a 1-voxel-wide corridor that winds
through the block row by row.  In `_ws_block` (watershed.py:139-207) the corridor's distance
transform is 1 everywhere, so its hmap is one exact plateau; the rooms' DT maxima are the only
seeds; the two floods enter the corridor at its ends and meet about 10,000 hops from each seed.
With d saturating at 4095 the packed key cannot order the voxels past that depth (a cycle of
equal keys can keep a stale label, ctws_dev.h): the GPU must detect the saturation and flood
those blocks on the wide keys (run_batch, BlockStat::dsat), reproducing the unbounded model.
WatershedFromSeeds (watershed_from_seeds.py:143-199) floods the corridor map itself with one
seed per room.  Reference semantics of the flood: utils/volume_utils.py:123-139.
"""
from collections import deque

import numpy as np

ROOM = 9


def corridor_map(ny=222, nx=200):
    """(1, ny, nx) float32 map: walls 1, rooms and corridor 0; the room centres (z, y, x)."""
    a = np.ones((1, ny, nx), np.float32)
    # room A top left, room B bottom left
    a[0, 1:1 + ROOM, 1:1 + ROOM] = 0
    yb = ny - 1 - ROOM
    a[0, yb:yb + ROOM, 1:1 + ROOM] = 0
    # serpentine rows between the rooms: y = y0, y0 + 2, ..., joined alternately at the right
    # and the left end
    y0, y1 = 1 + ROOM + 2, yb - 2
    rows = list(range(y0, y1 + 1, 2))
    for k, y in enumerate(rows):
        a[0, y, 1:nx - 1] = 0
        if k + 1 < len(rows):
            x = nx - 2 if k % 2 == 0 else 1
            a[0, y + 1, x] = 0
    # room A down to the first row (x = 1), the last row (an even count: it ends at x = 1) down
    # to room B
    assert len(rows) % 2 == 0, 'ny must give an even number of corridor rows'
    a[0, 1 + ROOM:y0, 1] = 0
    a[0, rows[-1] + 1:yb, 1] = 0
    c = ROOM // 2 + 1
    return a, [(0, c, c), (0, yb + ROOM // 2, c)]


def hop_distances(free, src):
    """BFS hop distance inside `free` (4-/6-neighbourhood) from the voxel `src`; -1 unreached."""
    d = np.full(free.shape, -1, np.int64)
    d[src] = 0
    q = deque([src])
    while q:
        p = q.popleft()
        for ax in range(free.ndim):
            for s in (-1, 1):
                n = list(p)
                n[ax] += s
                n = tuple(n)
                if 0 <= n[ax] < free.shape[ax] and free[n] and d[n] < 0:
                    d[n] = d[p] + 1
                    q.append(n)
    return d


def meeting_depth(labels, free, seeds):
    """The smallest hop distance from its own seed of a free voxel next to a voxel of the other
    seed's label: the depth at which the two floods meet on the plateau."""
    la, lb = labels[seeds[0]], labels[seeds[1]]
    assert la != lb and la and lb
    da, db = hop_distances(free, seeds[0]), hop_distances(free, seeds[1])
    best = None
    for ax in range(labels.ndim):
        sl0 = [slice(None)] * labels.ndim
        sl1 = [slice(None)] * labels.ndim
        sl0[ax], sl1[ax] = slice(0, -1), slice(1, None)
        a, b = labels[tuple(sl0)], labels[tuple(sl1)]
        f = free[tuple(sl0)] & free[tuple(sl1)] & (a != b)
        m = f & (a == la) & (b == lb)
        if m.any():
            v = int(min(da[tuple(sl0)][m].min(), db[tuple(sl1)][m].min()))
            best = v if best is None else min(best, v)
        m = f & (a == lb) & (b == la)
        if m.any():
            v = int(min(db[tuple(sl0)][m].min(), da[tuple(sl1)][m].min()))
            best = v if best is None else min(best, v)
    return best


BLOCK_SHAPE = (64, 256, 256)
_NOSMOOTH = dict(sigma_seeds=0., sigma_weights=0.)
_D3 = dict(apply_dt_2d=False, apply_ws_2d=False)


def _cases():
    a, seeds = corridor_map()
    free = a == 0
    # masked: the walls are masked out (the reference sets them to 1, watershed.py:299-303) over
    # noise, so the walls are the masked plateau the plateau fill handles (k_plateau.hip)
    am = np.where(free, a, np.random.default_rng(0).random(a.shape).astype(np.float32))
    m = free.astype(np.uint8)
    ws = {
        '2d': (dict(_NOSMOOTH), dict(input=a)),
        '2d_mask': (dict(_NOSMOOTH), dict(input=am, mask=m)),
        '3d': (dict(_NOSMOOTH, **_D3), dict(input=a)),
        '3d_mask': (dict(_NOSMOOTH, **_D3), dict(input=am, mask=m)),
        '2d_crop': (dict(_NOSMOOTH, halo=[0, 8, 8]),
                    dict(input=a, inner_begin=(0, 8, 8), inner_shape=(1, a.shape[1] - 16, a.shape[2] - 16),
                         crop_relabel=True)),
        '2d_sizefilter': (dict(_NOSMOOTH, size_filter=10 ** 9), dict(input=a)),
    }
    s = np.zeros(a.shape, np.uint64)
    s[seeds[0]], s[seeds[1]] = 5, 9
    fs = {
        'points': (dict(size_filter=0), dict(input=a, seeds=s)),
        'mask': (dict(size_filter=25), dict(input=am, seeds=s, mask=m)),
    }
    return ws, fs


CASES, FS_CASES = _cases()
_MODEL = {}


def run_model(name):
    from oracle import oracle as O
    if ('ws', name) not in _MODEL:
        cfg, blk = CASES[name]
        with O.flood_model():
            _MODEL[('ws', name)] = O.ws_blocks(cfg, BLOCK_SHAPE, [dict(blk, block_id=3)])[0]
    return _MODEL[('ws', name)]


def run_model_fs(name):
    from oracle import oracle as O
    if ('fs', name) not in _MODEL:
        cfg, blk = FS_CASES[name]
        with O.flood_model():
            _MODEL[('fs', name)] = O.ws_from_seeds(cfg, [blk])[0]
    return _MODEL[('fs', name)]
