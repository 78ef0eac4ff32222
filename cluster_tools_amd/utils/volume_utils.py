"""Volume I/O, block lists and masks around the watershed path
(cluster_tools/utils/volume_utils.py:23-88, :91, :142-218; utils/volume_classes.py:155-232).
The numeric helpers of the reference module (filters, normalize, watershed, size filter) are
the GPU kernels of libctws.so and are not restated here."""
import json
import os
from math import ceil, floor

import numpy as np

from ..io import File
from .blocking import Blocking


def is_z5(path):
    return os.path.splitext(path)[1][1:].lower() in ('n5', 'zr', 'zarr')


def is_h5(path):
    return os.path.splitext(path)[1][1:].lower() in ('h5', 'hdf5', 'hdf', 'ilp')


def file_reader(path, mode='a'):
    if is_z5(path):
        return File(path, mode=mode)
    if is_h5(path):
        import h5py  # not installed in this image; kept for parity with the reference
        return h5py.File(path, mode=mode)
    raise RuntimeError("Invalid file format %s" % os.path.splitext(path)[1][1:].lower())


def get_shape(path, key):
    with file_reader(path, 'r') as f:
        return tuple(f[key].shape)


def blocks_in_volume(shape, block_shape, roi_begin=None, roi_end=None, block_list_path=None):
    assert len(shape) == len(block_shape), '%i; %i' % (len(shape), len(block_shape))
    assert (roi_begin is None) == (roi_end is None)
    have_roi = roi_begin is not None
    if block_list_path is not None:
        assert os.path.exists(block_list_path), block_list_path
    blocking_ = Blocking([0] * len(shape), list(shape), list(block_shape))
    if not have_roi and not block_list_path:
        return list(range(blocking_.numberOfBlocks))
    if have_roi:
        roi_end = [sh if re is None else re for re, sh in zip(roi_end, shape)]
        block_list = blocking_.getBlockIdsOverlappingBoundingBox(list(roi_begin), list(roi_end)).tolist()
        assert len(block_list) == len(set(block_list))
    if block_list_path:
        with open(block_list_path) as f:
            list_from_path = json.load(f)
        block_list = np.intersect1d(list_from_path, block_list).tolist() if have_roi else list_from_path
    return [int(b) for b in block_list]


def block_to_bb(block):
    return tuple(slice(b, e) for b, e in zip(block.begin, block.end))


def _checkerboard(blocking_, start, allowed):
    """Alternating DFS over upper neighbours from `start` (volume_utils.py:142-205), with an
    explicit stack so large grids do not hit Python's recursion limit; the visiting order (and
    therefore both lists) is that of the recursive reference."""
    blocks_a, blocks_b = [start], []
    seen = {start}
    lists = (blocks_a, blocks_b)
    # frame: (block, index of the list its neighbours go to, next dim)
    stack = [(start, 1, 0)]
    while stack:
        block, li, dim = stack.pop()
        if dim >= 3:
            continue
        stack.append((block, li, dim + 1))
        ngb = blocking_.getNeighborId(block, dim, False)
        if ngb != -1 and (allowed is None or ngb in allowed) and ngb not in seen:
            lists[li].append(ngb)
            seen.add(ngb)
            stack.append((ngb, 1 - li, 0))
    return blocks_a, blocks_b


def make_checkerboard_block_lists(blocking_, roi_begin=None, roi_end=None):
    assert (roi_begin is None) == (roi_end is None)
    if roi_begin is None:
        blocks_a, blocks_b = _checkerboard(blocking_, 0, None)
        expected = set(range(blocking_.numberOfBlocks))
    else:
        block0 = blocking_.coordinatesToBlockId(roi_begin)
        in_roi = set(int(b) for b in blocking_.getBlockIdsOverlappingBoundingBox(roi_begin, roi_end))
        assert block0 in in_roi
        blocks_a, blocks_b = _checkerboard(blocking_, block0, in_roi)
        expected = in_roi
    all_blocks = blocks_a + blocks_b
    assert len(all_blocks) == len(expected), "%i, %i" % (len(all_blocks), len(expected))
    assert len(set(all_blocks) - expected) == 0
    assert len(blocks_a) == len(blocks_b), "%i, %i" % (len(blocks_a), len(blocks_b))
    return blocks_a, blocks_b


def _resize_nearest(data, shape):
    """Order-0 resize (vigra.sampling.resize(order=0)): output i samples input
    round(i * (n_in - 1) / (n_out - 1)).  vigra is absent: parity unpinned."""
    out = data
    for ax, (n_in, n_out) in enumerate(zip(data.shape, shape)):
        if n_out == 1 or n_in == 1:
            idx = np.zeros(n_out, dtype=int)
        else:
            idx = np.floor(np.arange(n_out) * (n_in - 1) / (n_out - 1) + 0.5).astype(int)
        out = np.take(out, np.clip(idx, 0, n_in - 1), axis=ax)
    return out


class InterpolatedVolume:
    """Nearest-neighbour view of a low-resolution mask at full resolution
    (utils/volume_classes.py:155-232): each request reads the covering low-res crop and
    resizes it to the request shape."""

    def __init__(self, volume, output_shape, spline_order=0):
        assert len(output_shape) == volume.ndim == 3, "Only 3d supported"
        assert spline_order == 0
        self.volume = volume
        self.shape = tuple(output_shape)
        self.dtype = volume.dtype
        self.scale = [sh / float(fsh) for sh, fsh in zip(volume.shape, self.shape)]

    def __getitem__(self, index):
        index = tuple(slice(*ind.indices(sh)[:2]) for ind, sh in zip(index, self.shape))
        ret_shape = tuple(ind.stop - ind.start for ind in index)
        singletons = tuple(sh == 1 for sh in ret_shape)
        starts = tuple(int(floor(ind.start * sc)) for ind, sc in zip(index, self.scale))
        stops = tuple(sta + 1 if single else int(ceil(ind.stop * sc))
                      for ind, sc, sta, single in zip(index, self.scale, starts, singletons))
        # an axis that the low-res crop collapses to one voxel while the request is longer
        # reads one more voxel (volume_classes.py:207-212)
        stops = tuple(b + 1 if (b - a == 1 and not single) else b
                      for a, b, single in zip(starts, stops, singletons))
        data = self.volume[tuple(slice(a, b) for a, b in zip(starts, stops))]
        s = data.sum()
        if s == 0:
            return np.zeros(ret_shape, dtype=self.dtype)
        if s == data.size:
            return np.ones(ret_shape, dtype=self.dtype)
        return _resize_nearest(data, ret_shape).astype(self.dtype)


def load_mask(mask_path, mask_key, shape):
    with file_reader(mask_path, 'r') as f:
        mshape = f[mask_key].shape
    if tuple(mshape) == tuple(shape):
        return file_reader(mask_path, 'r')[mask_key]
    with file_reader(mask_path, 'r') as f:
        mask = f[mask_key][:].astype('bool')
    return InterpolatedVolume(mask, shape, spline_order=0)
