"""Pins the CPU oracle (test infrastructure) before it is used as the parity checker.

* scipy (this interpreter): EDT bit-exact incl. pixel pitch; Gaussian vs gaussian_filter;
* scikit-image 0.18 (conda python 3.9, scripts/crosscheck_py39.py): local maxima, seed
  numbering in vigra scan order, watershed -- the recorded results are asserted here and the
  script is re-run when that interpreter exists;
* an independent pure-Python restatement of vigra's seededWatersheds on top of a port of
  libstdc++'s push_heap / pop_heap (the heap vigra's PriorityQueue wraps) -- equal labels on
  tie-heavy inputs;
* the committed golden fixtures (tests/golden) are reproduced exactly.
vigra itself is not available here: parity at the vigra boundary is "partially pinned"
(DESIGN.md §4)."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest
import scipy.ndimage as ndi

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GDIR = os.path.join(ROOT, 'tests', 'golden')
PY39 = '/opt/conda/bin/python3.9'


@pytest.mark.parametrize('shape,pitch', [((20, 33, 41), None), ((12, 40, 30), (10, 1, 1)), ((50, 61), None),
                                         ((7, 9, 11), (2, 3, 1))])
def test_edt_bit_exact_vs_scipy(shape, pitch):
    rng = np.random.default_rng(sum(shape))
    fg = rng.random(shape) > 0.97
    dt = O.distance_transform(fg, pitch)
    ref = ndi.distance_transform_edt(~fg, sampling=pitch).astype(np.float32)
    assert np.array_equal(dt, ref)


def test_edt_no_foreground_is_sqrt_dmax():
    dt = O.distance_transform(np.zeros((4, 5, 6), bool))
    assert np.all(dt == np.float32(np.sqrt(np.ceil(16 + 25 + 36))))


@pytest.mark.parametrize('sigma', [0.5, 1.0, 2.0, 3.3])
def test_gaussian_vs_scipy(sigma):
    x = np.random.default_rng(1).random((20, 30, 25)).astype(np.float32)
    g = O.gaussian_smoothing(x, sigma)
    ref = ndi.gaussian_filter(x, sigma, mode='mirror', truncate=3.0)
    assert np.max(np.abs(g - ref) / np.maximum(np.abs(ref), 1e-6)) <= 2.4e-7


def test_gaussian_kernel_is_vigra_init_gaussian():
    k = O.gaussian_kernel(2.0)
    assert len(k) == 2 * int(3 * 2.0 + 0.5) + 1
    assert np.array_equal(k, k[::-1])
    assert abs(k.sum() - 1.0) < 1e-15
    assert len(O.gaussian_kernel(0.1)) == 3  # radius int(0.3 + 0.5) == 0 -> 1


def test_py39_crosscheck_results_recorded():
    rep = json.load(open(os.path.join(GDIR, 'crosscheck_py39.json')))
    assert len(rep) >= 10
    for name, r in rep.items():
        assert r['edt_bit_exact_vs_scipy'], name
        assert r['local_maxima_equal_skimage'], name
        assert r['seed_labels_equal_skimage_scan_order'], name
        assert r['gaussian_max_rel_diff_vs_scipy'] <= 2.4e-7, name
        if 'watershed_vi_vs_skimage' in r:
            assert r['watershed_vi_vs_skimage'] <= 0.01, name


@pytest.mark.skipif(not os.path.exists(PY39), reason='no conda python3.9 with scikit-image')
def test_py39_crosscheck_rerun(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    out = subprocess.run([PY39, os.path.join(ROOT, 'scripts', 'crosscheck_py39.py')], env=env,
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]


# ---- independent restatement of vigra's seededWatersheds with libstdc++'s heap ----------
def _push_heap(h, comp):
    hole = len(h) - 1
    val = h[hole]
    parent = (hole - 1) // 2
    while hole > 0 and comp(h[parent], val):
        h[hole] = h[parent]
        hole = parent
        parent = (hole - 1) // 2
    h[hole] = val


def _adjust_heap(h, hole, length, val, comp):
    top = hole
    child = hole
    while child < (length - 1) // 2:
        child = 2 * (child + 1)
        if comp(h[child], h[child - 1]):
            child -= 1
        h[hole] = h[child]
        hole = child
    if (length & 1) == 0 and child == (length - 2) // 2:
        child = 2 * (child + 1)
        h[hole] = h[child - 1]
        hole = child - 1
    parent = (hole - 1) // 2
    while hole > top and comp(h[parent], val):
        h[hole] = h[parent]
        hole = parent
        parent = (hole - 1) // 2
    h[hole] = val


def _pop_heap(h, comp):
    last = h[-1]
    h[-1] = h[0]
    _adjust_heap(h, 0, len(h) - 1, last, comp)
    return h.pop()


def _vigra_watershed_py(hmap, seeds):
    lab = seeds.copy()
    shape = lab.shape
    nd = lab.ndim
    # direct neighbourhood order of vigra's GridGraph: -e_{N-1} .. -e_0, +e_0 .. +e_{N-1}
    offs = [(k, -1) for k in range(nd - 1, -1, -1)] + [(k, 1) for k in range(nd)]
    comp = lambda a, b: a[1] > b[1]   # std::greater on the priority: min-heap

    def nbrs(idx):
        for k, s in offs:
            c = list(idx)
            c[k] += s
            if 0 <= c[k] < shape[k]:
                yield tuple(c)
    heap = []
    for flat in range(lab.size):   # scan order: dim 0 fastest
        idx = np.unravel_index(flat, shape, order='F')
        if lab[idx]:
            if any(lab[n] == 0 for n in nbrs(idx)):
                heap.append((idx, float(hmap[idx])))
                _push_heap(heap, comp)
    while heap:
        idx, cost = _pop_heap(heap, comp)
        for n in nbrs(idx):
            if lab[n] == 0:
                lab[n] = lab[idx]
                heap.append((n, max(float(hmap[n]), cost)))
                _push_heap(heap, comp)
    return lab


@pytest.mark.parametrize('seed', [0, 1, 2])
def test_oracle_watershed_matches_python_heap_restatement(seed):
    rng = np.random.default_rng(seed)
    h = (rng.integers(0, 4, size=(6, 9, 8)) / 4).astype(np.float32)   # many exact ties
    s = np.zeros(h.shape, np.uint32)
    for i, p in enumerate(rng.choice(h.size, 6, replace=False)):
        s.flat[p] = i + 1
    got, _ = O.watershed(h, s)
    assert np.array_equal(got, _vigra_watershed_py(h, s))


def test_label_numbering_first_occurrence_in_scan_order():
    x = np.zeros((3, 4, 5), np.uint8)
    x[2, 0, 0] = 1   # F-index 2
    x[0, 3, 0] = 1   # F-index 9
    x[0, 0, 4] = 1   # F-index 48
    lab, n = O.label_with_background(x)
    assert n == 3 and lab[2, 0, 0] == 1 and lab[0, 3, 0] == 2 and lab[0, 0, 4] == 3


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_oracle_reproduces_golden_fixtures():
    index = json.load(open(os.path.join(GDIR, 'index.json')))
    for name, meta in index.items():
        z = np.load(os.path.join(GDIR, name + '.npz'))
        b = dict(meta['block'], input=z['input'])
        if 'mask' in z.files:
            b['mask'] = z['mask']
        r = O.ws_blocks(meta['config'], meta['block_shape'], [dict(b, block_id=meta['block_id'])],
                        with_stages=True)[0]
        assert r['status'] == meta['status'], name
        assert np.array_equal(r['output'], z['output']), name
        if meta['status'] == 0:
            assert np.array_equal(r['input'], z['fin']), name
            assert np.array_equal(r['ws'], z['ws']), name
            assert _sha(r['dt']) == meta['dt_sha256'], name


def test_metrics_orientation_matches_reference():
    """validation_utils.py:60-76 with contigency_table(groundtruth, segmentation): a
    segmentation that splits every gt object has vi-split > 0 and vi-merge = 0."""
    from cluster_tools_amd.metrics import vi_scores
    gt = np.repeat(np.arange(4), 16).reshape(8, 8)
    seg = np.arange(64).reshape(8, 8) // 4
    vs, vm = vi_scores(seg, gt)
    assert vs > 0.5 and abs(vm) < 1e-12
    vs2, vm2 = vi_scores(gt, seg)
    assert abs(vs2) < 1e-12 and abs(vm2 - vs) < 1e-12
