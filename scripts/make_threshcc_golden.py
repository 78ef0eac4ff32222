"""Golden vectors for the BlockComponents labelling (k_threshcc.hip, oracle/threshcc.py).

Run with /opt/conda/bin/python3.9 (scikit-image 0.18.3, the labelling library the reference's
block_components.py imports).  Each case is a float32 block, a threshold, a mode, an optional
mask and whether the block is normalized first (the unmasked path of `_cc_block`) or compared
raw (`_cc_block_with_mask`, sigma 0); the expected labels are skimage.morphology.label of the
members (block_components.py:160-180 / :213-228).  Writes tests/golden/threshcc_label.npz.
"""
import os

import numpy as np
from skimage.morphology import label

CASES = [
    # name, shape, density-ish threshold, mode, masked, seed
    ('sparse_greater', (5, 17, 70), 0.78, 'greater', False, 1),
    ('dense_greater', (12, 9, 130), 0.45, 'greater', False, 2),
    ('less', (9, 16, 64), 0.3, 'less', False, 3),
    ('masked_raw', (10, 19, 66), 0.7, 'greater', True, 4),
    ('equal_u8', (8, 24, 72), 3.0, 'equal', True, 5),
    ('smooth_blobs', (16, 33, 129), 0.6, 'greater', False, 6),
    ('single_voxels', (3, 5, 7), 0.9, 'greater', False, 7),
    ('very_sparse', (10, 24, 140), 0.93, 'greater', False, 9),
    ('constant', (4, 8, 64), 0.5, 'greater', False, 8),
]


def _block(shape, seed, name):
    rng = np.random.default_rng(seed)
    if name == 'equal_u8':
        return rng.integers(0, 6, size=shape).astype('float32')
    if name == 'constant':
        return np.full(shape, 0.25, dtype='float32')
    x = rng.random(shape).astype('float32')
    if name == 'smooth_blobs':
        from scipy.ndimage import gaussian_filter
        x = gaussian_filter(x, 1.5).astype('float32')
    return x


def _normalize(x):
    x = x.astype('float32')
    x -= x.min()
    mx = x.max()
    if mx > 0:
        x /= mx
    return x


def main():
    out = {}
    for name, shape, thr, mode, masked, seed in CASES:
        x = _block(shape, seed, name)
        mask = None
        if masked:
            rng = np.random.default_rng(seed + 100)
            mask = np.zeros(shape, dtype='uint8')
            mask[:, 2:-3, 5:] = 1
            mask[rng.random(shape) < 0.05] = 0
        v = x if masked else _normalize(x)
        m = {'greater': v > thr, 'less': v < thr, 'equal': v == thr}[mode]
        if mask is not None:
            m[np.logical_not(mask.astype(bool))] = 0
        lab = label(m).astype('uint64') if m.sum() else np.zeros(shape, dtype='uint64')
        out[name + '__input'] = x
        out[name + '__labels'] = lab
        out[name + '__params'] = np.array([thr, ('greater', 'less', 'equal').index(mode), int(masked)])
        if mask is not None:
            out[name + '__mask'] = mask
        print(name, shape, int(lab.max()))
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests', 'golden', 'threshcc_label.npz')
    np.savez_compressed(path, **out)
    print('wrote', os.path.normpath(path))


if __name__ == '__main__':
    main()
