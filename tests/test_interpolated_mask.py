"""InterpolatedVolume / load_mask (utils/volume_classes.py:155-232, volume_utils.py:208-218):
the low-resolution mask path.  vigra.sampling.resize is absent, so the order-0 resize is the
restated formula (output i samples input round(i (n_in - 1) / (n_out - 1))): parity of the
interpolated values is unpinned; these tests pin the request arithmetic the reference code
fixes (crop bounds, the empty / full fast paths, singleton axes) and that the GPU path uses it."""
import numpy as np
import pytest

from cluster_tools_amd.utils import volume_utils as vu


def test_fast_paths_and_shapes():
    low = np.zeros((4, 8, 8), bool)
    low[:, 4:, :] = True
    iv = vu.InterpolatedVolume(low, (16, 32, 32))
    assert iv.shape == (16, 32, 32) and iv.dtype == np.bool_
    # a request whose low-res crop is all 0 / all 1 takes the fast paths (:213-217)
    assert not iv[0:16, 0:8, 0:32].any()
    assert iv[0:16, 24:32, 0:32].all()
    assert iv[3:9, 5:30, 1:2].shape == (6, 25, 1)


def test_request_bounds_follow_the_reference():
    """starts = floor(start * scale), stops = ceil(stop * scale) (+1 for a collapsed axis):
    the covering crop of a request is what the reference reads (volume_classes.py:196-212)."""
    low = np.arange(4 * 8 * 8).reshape(4, 8, 8) % 2 == 0
    iv = vu.InterpolatedVolume(low, (16, 32, 32))
    seen = []

    class Spy:
        shape, dtype, ndim = low.shape, low.dtype, 3

        def __getitem__(self, idx):
            seen.append(tuple((s.start, s.stop) for s in idx))
            return low[idx]

    iv.volume = Spy()
    iv[4:8, 8:16, 10:20]
    # scale 0.25: z 1..2 (collapsed to 1 voxel -> +1), y 2..4, x floor(2.5)=2 .. ceil(5)=5
    assert seen[-1] == ((1, 3), (2, 4), (2, 5))
    iv[5:6, 8:16, 10:20]  # singleton request axis: start .. start + 1
    assert seen[-1][0] == (1, 2)


def test_resize_nearest_formula():
    d = np.array([[[0, 1, 0]]], np.uint8)
    out = vu._resize_nearest(d, (1, 1, 5))
    # i * 2 / 4 = 0, .5, 1, 1.5, 2 -> round half up: 0, 1, 1, 2, 2
    np.testing.assert_array_equal(out[0, 0], [0, 1, 1, 0, 0])


def test_load_mask_full_and_low_res(tmp_path):
    path = str(tmp_path / 'm.n5')
    full = np.zeros((8, 16, 16), np.uint8)
    full[:, 4:12, 4:12] = 1
    with vu.file_reader(path) as f:
        f.create_dataset('full', data=full, chunks=(4, 8, 8))
        f.create_dataset('low', data=full[::2, ::2, ::2], chunks=(4, 8, 8))
    m = vu.load_mask(path, 'full', (8, 16, 16))
    np.testing.assert_array_equal(m[:], full)
    low = vu.load_mask(path, 'low', (8, 16, 16))
    assert isinstance(low, vu.InterpolatedVolume)
    got = low[0:8, 0:16, 0:16]
    assert got.dtype == np.bool_ and got.shape == (8, 16, 16)
    # the interior of the square survives the 2x nearest upsampling, the far corners stay out
    assert got[:, 6:10, 6:10].all() and not got[:, :2, :2].any()
