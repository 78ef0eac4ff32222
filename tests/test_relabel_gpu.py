"""GPU RelabelWorkflow primitives against numpy (relabel/find_uniques.py:93-159,
find_labeling.py:84-126, write/write.py:153-226): ctws_unique_u64 == np.unique for dense
watershed ids (bitmap path) and for sparse / huge ids (radix-sort path: ranges beyond 2^35, a
single 2^64 - 1 id), ctws_unique_counts_u64 == np.unique(return_counts=True), and the
assignment lookup == takeDict."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _cases():
    rng = np.random.default_rng(7)
    V = 64 * 256 * 256
    dense = (np.uint64(37 * V) + rng.integers(1, 5000, size=(32, 64, 64)).astype(np.uint64))
    dense[::3] = 0
    wide = rng.integers(0, 2 ** 63, size=200000, dtype=np.int64).view(np.uint64)
    wide[:1000] = 0
    span36 = np.concatenate([np.arange(1, 100, dtype=np.uint64), np.array([2 ** 36 + 5], np.uint64)])
    huge = np.array([0, 2 ** 64 - 1, 2 ** 64 - 1, 5, 0], dtype=np.uint64)
    single_huge = np.full(1000, 2 ** 64 - 1, dtype=np.uint64)
    zeros = np.zeros(4096, np.uint64)
    blocks = np.repeat(np.arange(1, 300, dtype=np.uint64) * np.uint64(V), 37)
    return dict(dense=dense, wide=wide, span36=span36, huge=huge, single_huge=single_huge, zeros=zeros,
                blocks=blocks)


CASES = _cases()


@pytest.mark.parametrize('name', sorted(CASES))
def test_unique_matches_numpy(gpu_handle, name):
    x = CASES[name]
    np.testing.assert_array_equal(gpu_handle.unique_u64(x), np.unique(x))


@pytest.mark.parametrize('name', sorted(CASES))
def test_unique_counts_matches_numpy(gpu_handle, name):
    x = CASES[name]
    u, c = gpu_handle.unique_counts_u64(x)
    ru, rc = np.unique(x.ravel(), return_counts=True)
    np.testing.assert_array_equal(u, ru)
    np.testing.assert_array_equal(c, rc.astype(np.uint64))


def test_lookup_is_take_dict(gpu_handle):
    x = CASES['dense'].copy()
    uniq = np.unique(x)
    vals = np.arange(len(uniq), dtype=np.uint64) * np.uint64(3) + np.uint64(11)
    exp = vals[np.searchsorted(uniq, x)]
    assert gpu_handle.lookup_u64(x, uniq, vals) == 0
    np.testing.assert_array_equal(x, exp)
    y = np.array([uniq[1], 123456789], dtype=np.uint64)  # 123456789 is not a key
    assert gpu_handle.lookup_u64(y, uniq, vals) == 1
    assert y[0] == vals[1] and y[1] == 123456789
