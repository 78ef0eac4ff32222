"""Cross-check the CPU oracle against scipy / scikit-image (run with /opt/conda/bin/python3.9,
which has scikit-image 0.18.3 and scipy 1.7).  Writes tests/golden/crosscheck_py39.json.

What is checked on every golden fixture (tests/golden/*.npz):
* EDT: scipy.ndimage.distance_transform_edt of (fin <= threshold), per slice for apply_dt_2d,
  with `sampling=pixel_pitch` -- must be bit-exact (except slices without foreground, where
  vigra returns sqrt(dmax) and scipy inf / a different value; those slices are skipped);
* Gaussian: scipy.ndimage.gaussian_filter(mode='mirror', truncate=3.0), max relative diff
  (scipy folds symmetric taps, so the summation order differs: <= a few ulp);
* local maxima: skimage.morphology.local_maxima(connectivity=1 in 3-D / 2 in 2-D,
  allow_borders=True) -- must be identical;
* seed numbering: skimage.measure.label(connectivity=1) partition renumbered by first
  occurrence in F order (vigra scan order) -- must equal the oracle's seeds;
* watershed: skimage.segmentation.watershed(hmap, seeds) -- different tie order, VI recorded.
"""
import json
import os
import sys

import numpy as np
import scipy.ndimage as ndi
from skimage.measure import label as sk_label
from skimage.morphology import local_maxima as sk_local_maxima
from skimage.segmentation import watershed as sk_watershed

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402


def first_occurrence_relabel(lab):
    """Relabel a partition 1..k by first occurrence in F order (vigra scan order)."""
    flat = lab.ravel(order='F')
    ids, first = np.unique(flat, return_index=True)
    mapping = {}
    nxt = 1
    for i in np.argsort(first):
        if ids[i] == 0:
            continue
        mapping[ids[i]] = nxt
        nxt += 1
    out = np.zeros_like(lab, dtype=np.uint32)
    for k, v in mapping.items():
        out[lab == k] = v
    return out


def vi(a, b):
    a = a.ravel(); b = b.ravel(); n = float(a.size)
    _, ai, ac = np.unique(a, return_inverse=True, return_counts=True)
    _, bi, bc = np.unique(b, return_inverse=True, return_counts=True)
    p, pc = np.unique(ai.astype(np.int64) * len(bc) + bi, return_counts=True)
    pa, pb = p // len(bc), p % len(bc)
    h = lambda c: float(np.sum(-c / n * np.log2(c / n)))
    i = float(np.sum(pc / n * np.log2(n * pc / (ac[pa] * bc[pb]))))
    return h(ac) + h(bc) - 2 * i


def main():
    gdir = os.path.join(ROOT, 'tests', 'golden')
    index = json.load(open(os.path.join(gdir, 'index.json')))
    report = {}
    for name, meta in sorted(index.items()):
        if meta['status'] != 0:
            continue
        cfg = meta['config']
        z = np.load(os.path.join(gdir, name + '.npz'))
        fin = z['fin']
        thr = np.float32(cfg.get('threshold', .5))
        fg = fin > thr
        rep = {}
        # --- EDT
        dt2d = cfg.get('apply_dt_2d', True)
        pitch = cfg.get('pixel_pitch')
        if dt2d:
            dt = np.stack([O.distance_transform(fg[k]) for k in range(fg.shape[0])])
            ok = True
            for k in range(fg.shape[0]):
                if fg[k].any():
                    ref = ndi.distance_transform_edt(~fg[k]).astype(np.float32)
                    ok &= bool(np.array_equal(dt[k], ref))
        else:
            dt = O.distance_transform(fg, pitch)
            ref = ndi.distance_transform_edt(~fg, sampling=pitch).astype(np.float32)
            ok = bool(np.array_equal(dt, ref))
        rep['edt_bit_exact_vs_scipy'] = ok
        # --- seeds: Gaussian, local maxima, labels
        ws2d = cfg.get('apply_ws_2d', True)
        sig = cfg.get('sigma_seeds', 2.)
        slices = [dt[k] for k in range(dt.shape[0])] if ws2d else [dt]
        g_rel, lm_ok, lab_ok = 0.0, True, True
        for s in slices:
            if sig:
                sm = O.gaussian_smoothing(s, sig)
                sref = ndi.gaussian_filter(s, sig, mode='mirror', truncate=3.0)
                g_rel = max(g_rel, float(np.max(np.abs(sm - sref) / np.maximum(np.abs(sref), 1e-6))))
            else:
                sm = s
            mx = O.local_maxima(sm).astype(bool)
            if np.all(sm == sm.flat[0]):
                # constant image: vigra marks the whole plateau (hence the "all maxima -> ones"
                # branch of _make_seeds, watershed.py:195-197); skimage returns no maxima
                rep['constant_slices_skipped'] = rep.get('constant_slices_skipped', 0) + 1
                assert mx.all()
                continue
            skm = sk_local_maxima(sm, connectivity=1 if s.ndim == 3 else 2, allow_borders=True)
            lm_ok &= bool(np.array_equal(mx, skm.astype(bool)))
            ol, _ = O.label_with_background(mx.astype(np.uint8))
            sl = first_occurrence_relabel(sk_label(mx.astype(np.uint8), connectivity=1, background=0))
            lab_ok &= bool(np.array_equal(ol, sl))
        rep['gaussian_max_rel_diff_vs_scipy'] = g_rel
        rep['local_maxima_equal_skimage'] = lm_ok
        rep['seed_labels_equal_skimage_scan_order'] = lab_ok
        # --- watershed vs skimage (approximate: different tie order)
        seeds = z['seeds']
        if not ws2d:
            hm = O.make_hmap(fin, dt, cfg)
            wsk = sk_watershed(hm, seeds.astype(np.int64), connectivity=1)
            wo, _ = O.watershed(hm, seeds)
            rep['watershed_vi_vs_skimage'] = vi(wo, wsk)
        report[name] = rep
        print(name, rep)
    json.dump(report, open(os.path.join(gdir, 'crosscheck_py39.json'), 'w'), indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
