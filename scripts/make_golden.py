"""Generate the golden fixtures in tests/golden/ from the CPU oracle.

Each fixture holds the inputs (outer block, optional mask), the task config, and the oracle's
results: the normalized input and seeds (exact), sha256 digests of the EDT and hmap, the uint32
watershed of the outer block and the final uint64 inner block.  The oracle itself is pinned
by scripts/crosscheck_py39.py (scikit-image / scipy) and tests/test_oracle_crosscheck.py.
Run:  python scripts/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cluster_tools_amd.synthetic import boundary_map, ellipsoid_mask  # noqa: E402
from oracle import oracle as O  # noqa: E402

SHAPE = (16, 40, 40)
BLOCK_SHAPE = (64, 256, 256)
D3 = dict(apply_dt_2d=False, apply_ws_2d=False)


def cases():
    x = boundary_map(SHAPE, seed=21, pitch=(8, 8, 8))
    m = ellipsoid_mask(SHAPE)
    x4 = np.stack([boundary_map(SHAPE, seed=s, pitch=(8, 8, 8)) for s in (22, 23)])
    xq = (np.round(boundary_map(SHAPE, seed=24, pitch=(8, 8, 8)) * 4) / 4).astype(np.float32)
    xe = x.copy()
    xe[3] = 0.0
    inner = dict(inner_begin=(2, 8, 8), inner_shape=(12, 24, 24), crop_relabel=True)
    return {
        '3d': (dict(D3), dict(input=x)),
        '2d': ({}, dict(input=x)),
        '2d_halo_testcfg': (dict(threshold=.25, sigma_weights=0.), dict(input=x, **inner)),
        '3d_aniso_halo': (dict(D3, sigma_seeds=(.5, 2., 2.), sigma_weights=(.5, 2., 2.)), dict(input=x, **inner)),
        '3d_pitch': (dict(D3, pixel_pitch=(10, 1, 1)), dict(input=x)),
        '3d_mask': (dict(D3), dict(input=x, mask=m)),
        '2d_mask_halo': ({}, dict(input=x, mask=m, **inner)),
        '4d_mean': (dict(D3), dict(input=x4)),
        '3d_invert_u8': (dict(D3, invert_inputs=True, threshold=.3),
                         dict(input=np.round(x * 255).astype(np.uint8))),
        '2d_plateaus_sigma0': (dict(sigma_seeds=0.), dict(input=xq)),
        '2d_empty_slice': ({}, dict(input=xe)),
        'empty_block': ({}, dict(input=np.full(SHAPE, .3, np.float32))),
    }


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    out_dir = os.path.join(ROOT, 'tests', 'golden')
    os.makedirs(out_dir, exist_ok=True)
    index = {}
    for name, (config, block) in cases().items():
        r = O.ws_blocks(config, BLOCK_SHAPE, [dict(block, block_id=3)], with_stages=True)[0]
        nd = 3 if not config.get('apply_ws_2d', True) else 2
        seeds = np.zeros(r['input'].shape, np.uint32)
        hm = np.zeros(r['input'].shape, np.float32)
        if r['status'] == 0:
            if nd == 3:
                seeds = O.make_seeds(r['dt'], config)
                hm = O.make_hmap(r['input'], r['dt'], config)
            else:
                for z in range(seeds.shape[0]):
                    seeds[z] = O.make_seeds(r['dt'][z], config)
                    hm[z] = O.make_hmap(r['input'][z], r['dt'][z], config)
        arrays = dict(input=block['input'], fin=r['input'], seeds=seeds, ws=r['ws'], output=r['output'])
        if block.get('mask') is not None:
            arrays['mask'] = block['mask']
        np.savez_compressed(os.path.join(out_dir, name + '.npz'), **arrays)
        index[name] = dict(config=config, block={k: (list(v) if isinstance(v, tuple) else v)
                                                 for k, v in block.items() if k not in ('input', 'mask')},
                           block_id=3, block_shape=list(BLOCK_SHAPE), status=r['status'],
                           max_label=r['max_label'], dt_sha256=sha(r['dt']), hmap_sha256=sha(hm))
    with open(os.path.join(out_dir, 'index.json'), 'w') as f:
        json.dump(index, f, indent=1, sort_keys=True)
    print('wrote %d fixtures' % len(index))


if __name__ == '__main__':
    main()
