"""Shared parity cases: task configs x synthetic blocks (SURVEY.md §8(c) fixture list)."""
import numpy as np

from cluster_tools_amd.synthetic import boundary_map, ellipsoid_mask

SHAPE = (32, 96, 96)
BLOCK_SHAPE = (64, 256, 256)

D3 = dict(apply_dt_2d=False, apply_ws_2d=False)


def _x(seed=1, shape=SHAPE, dtype='float32'):
    return boundary_map(shape, seed=seed, dtype=dtype)


def make_cases():
    x = _x()
    m = ellipsoid_mask(SHAPE)
    x4 = np.stack([_x(seed=s) for s in (4, 5, 6)])
    inner = ((0, 16, 16), (32, 64, 64))
    inner3 = ((2, 16, 16), (28, 64, 64))
    # plateau-heavy input: quantized boundary map
    xq = (np.round(_x(seed=7) * 4) / 4).astype(np.float32)
    # a slice without any boundary (EDT = sqrt(dmax) there)
    xe = _x(seed=8).copy()
    xe[5] = 0.0
    # rows wider than 256 voxels: the x pass's register kernel at 8 and 16 voxels per lane, and
    # the ragged tail of a 1000-voxel row
    xw512 = _x(seed=10, shape=(8, 16, 512))
    xw600 = np.stack([_x(seed=s, shape=(3, 16, 600)) for s in (11, 12)])
    xw1000 = _x(seed=13, shape=(8, 12, 1000))
    # slices 0-3 of pure noise (only small segments) over a regular map: with size_filter 200
    # every segment of those slices is removed and vigra auto-seeds their regrow from the hmap
    # minima, while the other slices keep segments (volume_utils.py:131-139)
    xn = _x(seed=14).copy()
    rng = np.random.RandomState(5)
    xn[:4] = rng.rand(4, SHAPE[1], SHAPE[2]).astype(np.float32)
    # a few boundary voxels in a large empty volume: most EDT lines are far from (or without)
    # foreground, so the bounded search hands them to the lower-envelope pass (k_edt_col_fh)
    xs = np.zeros((12, 160, 144), np.float32)
    xs[3, 20, 30] = xs[3, 150, 100] = xs[9, 80, 5] = 1.0
    xs[6, :, 70] = 1.0
    # rows wider than a wave's registers (X > 1024: generic x-pass and row kernels), and a 2-D
    # dt with Y^2 + X^2 >= 2^24 (vigra's float arithmetic: k_edt_real_* with T = float)
    xw1100 = _x(seed=15, shape=(8, 10, 1100))
    xw4096 = _x(seed=16, shape=(2, 24, 4096))
    # 4096-voxel rows with a larger x radius than y: the x pass is the separate row kernel, whose
    # 1 KiB + 16 B per voxel of LDS is above 64 KiB (the opt-in launch)
    xw4096_3d = _x(seed=18, shape=(4, 12, 4096))
    # outer blocks beyond the round-5 caps (X <= 4096, Y, Z <= 2048): rows and
    # columns held whole in LDS above the 64 KiB default (the kernels' opt-in, up to 160 KiB)
    xw4200 = _x(seed=19, shape=(1, 64, 4200))
    xt2200 = _x(seed=20, shape=(1, 2200, 64))
    xd2200 = _x(seed=21, shape=(2200, 8, 32))
    # a mask of random blobs: the masked region is a non-convex plateau with holes, so the
    # plateau fill's run scans (k_plateau.hip) miss paths that the frontier has to correct
    rs = np.random.RandomState(17)
    from scipy.ndimage import gaussian_filter
    blobs = gaussian_filter(rs.rand(*SHAPE), (1.5, 4, 4)) > 0.5
    return {
        '3d_pitch_real': (dict(D3, pixel_pitch=(10.5, 1, 1)), dict(input=x)),
        '3d_pitch_frac': (dict(D3, pixel_pitch=(2.25, 0.75, 1.5)), dict(input=x)),
        '3d_pitch_bigdmax': (dict(D3, pixel_pitch=(600, 1, 1)), dict(input=x)),
        '2d_wide4096_bigdmax': ({}, dict(input=xw4096)),
        '3d_wide1100': (dict(D3), dict(input=xw1100)),
        '3d_wide4096_aniso': (dict(D3, sigma_seeds=(1., 1., 3.), sigma_weights=(1., 1., 3.)), dict(input=xw4096_3d)),
        '2d_sigma22': (dict(sigma_seeds=22.0), dict(input=x)),
        '2d_wide4200': ({}, dict(input=xw4200)),
        '2d_tall2200': (dict(sigma_weights=5.0), dict(input=xt2200)),
        '3d_deep2200': (dict(D3), dict(input=xd2200)),
        '3d_sparse_fg': (dict(D3), dict(input=xs)),
        '2d_sparse_fg': ({}, dict(input=xs)),
        '3d_sizefilter_all': (dict(D3, size_filter=10 ** 9), dict(input=x)),
        '2d_sizefilter_all': (dict(size_filter=10 ** 9), dict(input=x)),
        '2d_sizefilter_noise_slices': (dict(size_filter=200), dict(input=xn)),
        '2d_sizefilter_noise_halo': (dict(size_filter=200, halo=[0, 16, 16]),
                                     dict(input=xn, inner_begin=inner[0], inner_shape=inner[1], crop_relabel=True)),
        '3d_wide512_mask': (dict(D3), dict(input=xw512, mask=ellipsoid_mask(xw512.shape))),
        '2d_wide600_4d': ({}, dict(input=xw600)),
        '3d_wide1000': (dict(D3), dict(input=xw1000)),
        '3d_default': (dict(D3), dict(input=x)),
        '2d_default': ({}, dict(input=x)),
        '2d_test_cfg_halo': (dict(threshold=.25, sigma_weights=0., halo=[0, 32, 32]),
                             dict(input=x, inner_begin=inner[0], inner_shape=inner[1], crop_relabel=True)),
        '3d_aniso_halo': (dict(D3, sigma_seeds=(.5, 2., 2.), sigma_weights=(.5, 2., 2.), halo=[2, 32, 32]),
                          dict(input=x, inner_begin=inner3[0], inner_shape=inner3[1], crop_relabel=True)),
        '3d_pitch': (dict(D3, pixel_pitch=(10, 1, 1)), dict(input=x)),
        '3d_mask': (dict(D3), dict(input=x, mask=m)),
        '3d_mask_blobs': (dict(D3), dict(input=x, mask=blobs)),
        '2d_mask_blobs': ({}, dict(input=x, mask=blobs)),
        '2d_mask': ({}, dict(input=x, mask=m)),
        '3d_mask_halo': (dict(D3), dict(input=x, mask=m, inner_begin=inner3[0], inner_shape=inner3[1],
                                        crop_relabel=True)),
        '4d_mean': (dict(D3), dict(input=x4)),
        '4d_max_chan': (dict(D3, agglomerate_channels='max', channel_begin=1), dict(input=x4)),
        '2d_4d_min': (dict(agglomerate_channels='min'), dict(input=x4)),
        '3d_invert': (dict(D3, invert_inputs=True, threshold=.3), dict(input=x)),
        '3d_u8': (dict(D3), dict(input=_x(seed=9, dtype='uint8'))),
        '3d_f64': (dict(D3), dict(input=x.astype(np.float64))),
        '3d_plateaus': (dict(D3, sigma_seeds=0., sigma_weights=0.), dict(input=xq)),
        '2d_plateaus': (dict(sigma_seeds=0.), dict(input=xq)),
        '2d_empty_slice': ({}, dict(input=xe)),
        '3d_no_sizefilter': (dict(D3, size_filter=0), dict(input=x)),
        '3d_sigma0_alpha1': (dict(D3, sigma_seeds=0, alpha=1.0), dict(input=x)),
    }
