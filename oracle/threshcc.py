"""TEST INFRASTRUCTURE ONLY — CPU oracle of ThresholdedComponentsWorkflow (numpy / scipy).

Restates, for the parity tests of k_threshcc.hip / ctws_ufd_find and the task chain:
  block_components   thresholded_components/block_components.py:143-230 (`_cc_block`,
                     `_cc_block_with_mask`) with utils/volume_utils.py:113-120 (normalize), the
                     sigma_prefilter Gaussian (vigra restatement of the C++ oracle) and
                     skimage.morphology.label (full 26-connectivity, background 0; labels in
                     order of first appearance in a C-order scan)
  merge_offsets      thresholded_components/merge_offsets.py:96-130
  block_faces        thresholded_components/block_faces.py:87-177 with
                     utils/volume_utils.py:221-270 (iterate_faces / get_face: axial faces only)
  boost_ufd_find     merge_assignments.py:125-130: nifty.ufd.boost_ufd -> boost::disjoint_sets
                     (boost/pending/detail/disjoint_sets.hpp link_sets: union by rank, at equal
                     ranks the first root goes under the second); nifty is absent here, so the
                     representatives are pinned by this restatement only
  thresholded_components   the workflow: the above + write/write.py:178-211 (offsets + take)

Parity pinning: block_components's labelling is checked against skimage 0.18.3 outputs
(tests/golden/threshcc_label.npz, made by scripts/make_threshcc_golden.py under
/opt/conda/bin/python3.9, the reference's own labelling library).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module.
"""
import numpy as np
from scipy import ndimage

MODES = ('greater', 'less', 'equal')


def normalize(x):
    """vu.normalize (volume_utils.py:113-120) in float32."""
    x = x.astype('float32')
    x -= x.min()
    mx = x.max()
    if mx > 0:
        x /= mx
    return x


def label26(members):
    """skimage.morphology.label(members) for a 3-D bool array: 26-connected components, numbered
    1.. by first appearance in C order (scipy labels, renumbered)."""
    lab, n = ndimage.label(members, structure=np.ones((3, 3, 3), dtype=bool))
    if n == 0:
        return lab.astype('uint64'), 0
    flat = lab.ravel()
    ids, first = np.unique(flat, return_index=True)
    keep = ids > 0
    ids, first = ids[keep], first[keep]
    order = np.argsort(first, kind='stable')
    new = np.zeros(n + 1, dtype='uint64')
    new[ids[order]] = np.arange(1, len(ids) + 1, dtype='uint64')
    return new[lab], int(len(ids))


def gaussian(x, sigma):
    """vu.apply_filter(x, 'gaussianSmoothing', sigma) with a scalar sigma: vigra's
    gaussianSmoothing (fastfilters is absent in the reference env, volume_utils.py:15-20) on the
    float32 values -- the oracle's C++ restatement (ctws_oracle.cpp gaussian_smoothing)."""
    from oracle import oracle as O
    return O.gaussian_smoothing(np.ascontiguousarray(x, dtype='float32'), float(sigma))


def members(block, threshold, mode='greater', mask=None, normalize_input=True, sigma=0.):
    """The thresholded block of `_cc_block` (block_components.py:150-171: the single-channel
    block normalized, a channel sum raw; with sigma the Gaussian and a normalize) and
    `_cc_block_with_mask` (:198-222: raw values; with sigma normalize, Gaussian, normalize).
    The comparison is the reference's `input_ > threshold` with a Python float, i.e. numpy's
    promotion: float32 values against the threshold as float32, float64 and integer values in
    float64."""
    x = block
    if mask is None:
        if normalize_input:
            x = normalize(x)
        if sigma > 0:
            x = normalize(gaussian(x, sigma))
    elif sigma > 0:
        x = normalize(gaussian(normalize(x), sigma))
    x = np.asarray(x)
    thr = float(threshold)
    if mode == 'greater':
        m = x > thr
    elif mode == 'less':
        m = x < thr
    elif mode == 'equal':
        m = x == thr
    else:
        raise RuntimeError("Thresholding Mode %s not supported" % mode)
    if mask is not None:
        m &= np.asarray(mask).astype(bool)
    return m


def block_components(block, threshold, mode='greater', mask=None, normalize_input=True, sigma=0.):
    """-> (uint64 labels, n_labels); n_labels 0 = no member (the reference returns offset 0 and
    writes nothing; the labels are all 0 here)."""
    m = members(block, threshold, mode, mask, normalize_input, sigma)
    if not m.any():
        return np.zeros(m.shape, dtype='uint64'), 0
    return label26(m)


def merge_offsets(counts):
    """counts[b] = block b's `max + 1` (0 if empty) -> (offsets, empty_blocks, n_labels)."""
    counts = np.asarray(counts, dtype='uint64')
    last = counts[-1]
    empty = np.where(counts == 0)[0].tolist()
    offs = np.roll(counts, 1)
    offs[0] = 0
    offs = np.cumsum(offs)
    return offs.tolist(), empty, int(offs[-1] + last + 1)


def block_faces(seg, blocking, offsets, empty_blocks, faces_jobs=1):
    """Unique (a, b) label pairs across every block's upper faces (block_faces.py:116-177), from
    `faces_jobs` BlockFaces jobs (block_list[j::n]): empty when one of the jobs found no pair --
    MergeAssignments then merges nothing (merge_assignments.py:116-123)."""
    empty = set(empty_blocks)
    n_jobs = max(1, min(blocking.numberOfBlocks, faces_jobs))
    jobs = []
    for j in range(n_jobs):
        out = []
        for bid in range(j, blocking.numberOfBlocks, n_jobs):
            if bid in empty:
                continue
            for axis in range(3):
                ngb = blocking.getNeighborId(bid, axis, False)
                if ngb == -1 or ngb in empty:
                    continue
                blk = blocking.getBlock(bid)
                face = tuple(slice(b, e) if d != axis else slice(e - 1, e + 1)
                             for d, (b, e) in enumerate(zip(blk.begin, blk.end)))
                f = seg[face]
                la = np.take(f, 0, axis=axis).ravel().astype('uint64')
                lb = np.take(f, 1, axis=axis).ravel().astype('uint64')
                have = (la != 0) & (lb != 0)
                la, lb = la[have] + np.uint64(offsets[bid]), lb[have] + np.uint64(offsets[ngb])
                if la.size:
                    out.append(np.unique(np.stack([la, lb], axis=1), axis=0))
        jobs.append(np.unique(np.concatenate(out, axis=0), axis=0) if out else np.zeros((0, 2), dtype='uint64'))
    if not all(p.size for p in jobs):
        return np.zeros((0, 2), dtype='uint64')
    return np.unique(np.concatenate(jobs, axis=0), axis=0)


def boost_ufd_find(n, pairs):
    """boost_ufd(n).merge(pairs); find(arange(n)) — pure-Python loops (small cases only)."""
    parent = list(range(n))
    rank = [0] * n

    def find(a):
        r = a
        while parent[r] != r:
            r = parent[r]
        while parent[a] != r:
            parent[a], a = r, parent[a]
        return r

    for a, b in np.asarray(pairs, dtype='uint64').reshape(-1, 2).tolist():
        i, j = find(a), find(b)
        if i == j:
            continue
        if rank[i] > rank[j]:
            parent[j] = i
        else:
            parent[i] = j
            if rank[i] == rank[j]:
                rank[j] += 1
    return np.array([find(i) for i in range(n)], dtype='uint64')


def thresholded_components(volume, blocking, threshold, mode='greater', mask=None, normalize_input=None, sigma=0.,
                           faces_jobs=1):
    """The whole workflow on an in-memory volume (one job per task, `faces_jobs` BlockFaces jobs):
    -> (segmentation uint64, assignments uint64, offsets dict).  normalize_input None: as the
    reference, normalize the unmasked blocks only; False: the summed channels of a 4-D input
    (block_components.py:152-158 compares them raw)."""
    seg = np.zeros(volume.shape, dtype='uint64')
    counts = []
    for bid in range(blocking.numberOfBlocks):
        blk = blocking.getBlock(bid)
        bb = tuple(slice(b, e) for b, e in zip(blk.begin, blk.end))
        if mask is not None:
            mb = np.asarray(mask[bb]).astype(bool)
            if not mb.any():
                counts.append(0)
                continue
            lab, n = block_components(volume[bb], threshold, mode, mb, normalize_input=False, sigma=sigma)
        else:
            lab, n = block_components(volume[bb], threshold, mode, None,
                                      normalize_input=True if normalize_input is None else normalize_input,
                                      sigma=sigma)
        if n:
            seg[bb] = lab
        counts.append(n + 1 if n else 0)
    offsets, empty, n_labels = merge_offsets(counts)
    pairs = block_faces(seg, blocking, offsets, empty, faces_jobs)
    assignments = boost_ufd_find(n_labels, pairs) if len(pairs) else np.arange(n_labels, dtype='uint64')
    out = np.zeros_like(seg)
    for bid in range(blocking.numberOfBlocks):
        if bid in set(empty):
            continue
        blk = blocking.getBlock(bid)
        bb = tuple(slice(b, e) for b, e in zip(blk.begin, blk.end))
        s = seg[bb].copy()
        nz = s != 0
        if not nz.any():
            continue
        s[nz] += np.uint64(offsets[bid])
        out[bb] = assignments[s]
    return out, assignments, {'offsets': offsets, 'empty_blocks': empty, 'n_labels': n_labels}
