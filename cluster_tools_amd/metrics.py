"""Segmentation comparison metrics with the reference's formulas.

VI (split, merge; log2) and adapted Rand error exactly as
cluster_tools/utils/validation_utils.py:60-76 (compute_vi_scores) and :178-198
(compute_rand_scores), with the contingency table of validation_utils.py:9-35 computed by a
vectorised numpy pair-count instead of nifty.ground_truth.overlap.  As in
variation_of_information (validation_utils.py:79-112: contigency_table(groundtruth,
segmentation)) and measures.py (overlaps of seg with gt), `gt` plays seg_a and `seg` plays
seg_b, so vi_split = H(seg | gt) and vi_merge = H(gt | seg); `ignore_gt` drops voxels whose gt
label is in the list (the evaluation workflow ignores gt label 0 by default,
evaluation/evaluation_workflow.py:53,60-67).  Host-side check for the tests; the GPU version
is ctws.Handle.evaluate (k_eval.hip).
"""
import numpy as np


def contingency(seg, gt, ignore_gt=None):
    """(a = gt counts, b = seg counts, pair gt index, pair seg index, pair counts, n)."""
    seg = np.asarray(seg).ravel()
    gt = np.asarray(gt).ravel()
    if ignore_gt is not None:
        keep = ~np.isin(gt, ignore_gt)
        seg, gt = seg[keep], gt[keep]
    n = float(seg.size)
    a_ids, a_inv, a_counts = np.unique(gt, return_inverse=True, return_counts=True)
    b_ids, b_inv, b_counts = np.unique(seg, return_inverse=True, return_counts=True)
    pair = a_inv.astype(np.int64) * len(b_ids) + b_inv.astype(np.int64)
    p_ids, p_counts = np.unique(pair, return_counts=True)
    pa, pb = p_ids // len(b_ids), p_ids % len(b_ids)
    return (a_counts.astype(np.float64), b_counts.astype(np.float64), pa, pb,
            p_counts.astype(np.float64), n)


def vi_scores(seg, gt, ignore_gt=None):
    """(vi_split, vi_merge) with log2, as compute_vi_scores(..., use_log2=True)."""
    a, b, pa, pb, pc, n = contingency(seg, gt, ignore_gt)
    if n == 0:
        return 0.0, 0.0
    sum_a = float(np.sum(-a / n * np.log2(a / n)))
    sum_b = float(np.sum(-b / n * np.log2(b / n)))
    sum_ab = float(np.sum(pc / n * np.log2(n * pc / (a[pa] * b[pb]))))
    return sum_b - sum_ab, sum_a - sum_ab


def rand_scores(seg, gt, ignore_gt=None):
    """(adapted_rand_error, rand_index) as compute_rand_scores."""
    a, b, pa, pb, pc, n = contingency(seg, gt, ignore_gt)
    sum_a = float(np.sum(a * a))
    sum_b = float(np.sum(b * b))
    sum_ab = float(np.sum(pc * pc))
    prec = sum_ab / sum_b
    rec = sum_ab / sum_a
    ari = (2 * prec * rec) / (prec + rec)
    ri = 1. - (sum_a + sum_b - 2 * sum_ab) / (n * n)
    return 1. - ari, ri
