"""Deterministic synthetic boundary maps.

A jittered-grid Voronoi boundary map: one point per grid cell (jitter from
splitmix64(seed, cell)), b = clamp(1 - (d2 - d1) / 2.5, 0, 1) with d1/d2 the nearest and
second-nearest point distances over the 3x3x3 cell neighbourhood, plus uniform noise in
[-0.05, 0.05] from splitmix64(seed, voxel), clamped to [0, 1].  float32, or uint8 =
round(255 b).  The optional mask is the inscribed ellipsoid of the volume.

Used by bench.py and the tests; nothing here is on the product path.
"""
import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over='ignore'):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _u01(seed, idx):
    h = splitmix64(splitmix64(np.uint64(seed)) ^ np.asarray(idx, dtype=np.uint64))
    return (h >> np.uint64(40)).astype(np.float64) * (1.0 / (1 << 24))


def boundary_map(shape, seed=0, pitch=(24, 24, 24), noise=0.05, dtype='float32', z_chunk=16, origin=(0, 0, 0),
                 full_shape=None):
    """Voronoi boundary map of `shape` (Z, Y, X); with `full_shape`, the sub-volume
    [origin, origin + shape) of the map of `full_shape` (as boundary_map_torch)."""
    shape = tuple(int(s) for s in shape)
    full = tuple(int(s) for s in (full_shape or shape))
    gz0, gy0, gx0 = (int(o) for o in origin)
    pz, py, px = (float(p) for p in pitch)
    ncz, ncy, ncx = (int(np.ceil(s / p)) + 2 for s, p in zip(full, (pz, py, px)))
    # points for cells -1 .. nc-2 along each axis (one ring of padding cells)
    cz, cy, cx = np.meshgrid(np.arange(ncz), np.arange(ncy), np.arange(ncx), indexing='ij')
    cell = (cz * ncy + cy) * ncx + cx
    cell = cell.astype(np.uint64)
    jz = _u01(seed, cell * np.uint64(3))
    jy = _u01(seed, cell * np.uint64(3) + np.uint64(1))
    jx = _u01(seed, cell * np.uint64(3) + np.uint64(2))
    ptz = ((cz - 1) + 0.1 + 0.8 * jz) * pz
    pty = ((cy - 1) + 0.1 + 0.8 * jy) * py
    ptx = ((cx - 1) + 0.1 + 0.8 * jx) * px
    out = np.empty(shape, dtype=np.dtype(dtype))
    Y, X = shape[1], shape[2]
    FY, FX = full[1], full[2]
    yy, xx = np.meshgrid(gy0 + np.arange(Y, dtype=np.float64), gx0 + np.arange(X, dtype=np.float64), indexing='ij')
    icy = (yy // py).astype(np.int64) + 1
    icx = (xx // px).astype(np.int64) + 1
    for z0 in range(0, shape[0], z_chunk):
        z1 = min(shape[0], z0 + z_chunk)
        zz = np.arange(gz0 + z0, gz0 + z1, dtype=np.float64)[:, None, None]
        icz = (zz // pz).astype(np.int64) + 1
        d1 = np.full((z1 - z0, Y, X), np.inf)
        d2 = np.full((z1 - z0, Y, X), np.inf)
        for oz in (-1, 0, 1):
            for oy in (-1, 0, 1):
                for ox in (-1, 0, 1):
                    kz = icz + oz
                    ky = (icy + oy)[None]
                    kx = (icx + ox)[None]
                    d = np.sqrt((ptz[kz, ky, kx] - zz) ** 2 + (pty[kz, ky, kx] - yy[None]) ** 2 +
                                (ptx[kz, ky, kx] - xx[None]) ** 2)
                    closer = d < d1
                    d2 = np.where(closer, d1, np.minimum(d2, d))
                    d1 = np.where(closer, d, d1)
        b = np.clip(1.0 - (d2 - d1) / 2.5, 0.0, 1.0)
        vidx = (np.arange(gz0 + z0, gz0 + z1, dtype=np.uint64)[:, None, None] * np.uint64(FY) +
                np.arange(gy0, gy0 + Y, dtype=np.uint64)[None, :, None]) * np.uint64(FX) + \
            np.arange(gx0, gx0 + X, dtype=np.uint64)[None, None, :]
        b = b + noise * (2.0 * _u01(seed + 7919, vidx) - 1.0)
        b = np.clip(b, 0.0, 1.0)
        if out.dtype == np.uint8:
            out[z0:z1] = np.round(255.0 * b).astype(np.uint8)
        else:
            out[z0:z1] = b.astype(out.dtype)
    return out


def ellipsoid_mask_sub(shape, origin, full_shape):
    """`ellipsoid_mask(full_shape)[origin:origin + shape]` (numpy)."""
    ax = [((np.arange(o, o + s, dtype=np.float64) + 0.5) / f - 0.5) / 0.5
          for s, o, f in zip(shape, origin, full_shape)]
    r = ax[0][:, None, None] ** 2 + ax[1][None, :, None] ** 2 + ax[2][None, None, :] ** 2
    return (r <= 1.0).astype(np.uint8)


def ellipsoid_mask(shape):
    """uint8 mask of the inscribed ellipsoid (semi-axes 0.5*shape, centred)."""
    zz, yy, xx = (((np.arange(s, dtype=np.float64) + 0.5) / s - 0.5) / 0.5 for s in shape)
    r = zz[:, None, None] ** 2 + yy[None, :, None] ** 2 + xx[None, None, :] ** 2
    return (r <= 1.0).astype(np.uint8)


def boundary_map_torch(shape, seed=0, pitch=(24, 24, 24), noise=0.05, dtype='float32', device='cuda', z_chunk=32,
                       origin=(0, 0, 0), full_shape=None):
    """Same map as `boundary_map`, generated with torch (float64 arithmetic) on `device`.

    With `full_shape`, the sub-volume [origin, origin + shape) of the map of `full_shape`."""
    import torch
    shape = tuple(int(s) for s in shape)
    full = tuple(int(s) for s in (full_shape or shape))
    gz0, gy0, gx0 = (int(o) for o in origin)
    pz, py, px = (float(p) for p in pitch)
    ncz, ncy, ncx = (int(np.ceil(s / p)) + 2 for s, p in zip(full, (pz, py, px)))
    cz, cy, cx = np.meshgrid(np.arange(ncz), np.arange(ncy), np.arange(ncx), indexing='ij')
    cell = ((cz * ncy + cy) * ncx + cx).astype(np.uint64)
    pts = []
    for k, (c, p) in enumerate(((cz, pz), (cy, py), (cx, px))):
        j = _u01(seed, cell * np.uint64(3) + np.uint64(k))
        pts.append(torch.from_numpy(((c - 1) + 0.1 + 0.8 * j) * p).to(device))
    ptz, pty, ptx = pts
    Z, Y, X = shape
    FY, FX = full[1], full[2]
    out = torch.empty(shape, dtype=getattr(torch, dtype), device=device)
    yy = (gy0 + torch.arange(Y, dtype=torch.float64, device=device))[:, None].expand(Y, X)
    xx = (gx0 + torch.arange(X, dtype=torch.float64, device=device))[None, :].expand(Y, X)
    icy = torch.div(yy, py, rounding_mode='floor').long() + 1
    icx = torch.div(xx, px, rounding_mode='floor').long() + 1
    # per-voxel noise hash: splitmix64 in int64 arithmetic (wrapping)
    s0 = int(splitmix64(np.uint64(seed + 7919)))
    M = (1 << 64) - 1

    def to_i64(v):
        v &= M
        return v - (1 << 64) if v >= (1 << 63) else v

    def smix(x):
        x = x + to_i64(0x9E3779B97F4A7C15)
        x = (x ^ ((x >> 30) & ((1 << 34) - 1))) * to_i64(0xBF58476D1CE4E5B9)
        x = (x ^ ((x >> 27) & ((1 << 37) - 1))) * to_i64(0x94D049BB133111EB)
        return x ^ ((x >> 31) & ((1 << 33) - 1))

    for z0 in range(0, Z, z_chunk):
        z1 = min(Z, z0 + z_chunk)
        zz = torch.arange(gz0 + z0, gz0 + z1, dtype=torch.float64, device=device)[:, None, None]
        icz = torch.div(zz, pz, rounding_mode='floor').long() + 1
        d1 = torch.full((z1 - z0, Y, X), float('inf'), dtype=torch.float64, device=device)
        d2 = torch.full_like(d1, float('inf'))
        for oz in (-1, 0, 1):
            for oy in (-1, 0, 1):
                for ox in (-1, 0, 1):
                    kz = (icz + oz).expand(z1 - z0, Y, X)
                    ky = (icy + oy)[None].expand(z1 - z0, Y, X)
                    kx = (icx + ox)[None].expand(z1 - z0, Y, X)
                    d = torch.sqrt((ptz[kz, ky, kx] - zz) ** 2 + (pty[kz, ky, kx] - yy[None]) ** 2 +
                                   (ptx[kz, ky, kx] - xx[None]) ** 2)
                    closer = d < d1
                    d2 = torch.where(closer, d1, torch.minimum(d2, d))
                    d1 = torch.where(closer, d, d1)
        b = torch.clamp(1.0 - (d2 - d1) / 2.5, 0.0, 1.0)
        gz = torch.arange(gz0 + z0, gz0 + z1, dtype=torch.int64, device=device)[:, None, None]
        gy = torch.arange(gy0, gy0 + Y, dtype=torch.int64, device=device)[None, :, None]
        gx = torch.arange(gx0, gx0 + X, dtype=torch.int64, device=device)[None, None, :]
        vidx = (gz * FY + gy) * FX + gx
        h = smix(vidx ^ to_i64(s0))
        u = ((h >> 40) & ((1 << 24) - 1)).to(torch.float64) * (1.0 / (1 << 24))
        b = torch.clamp(b + noise * (2.0 * u - 1.0), 0.0, 1.0)
        if dtype == 'uint8':
            out[z0:z1] = torch.round(255.0 * b).to(torch.uint8)
        else:
            out[z0:z1] = b.to(out.dtype)
    return out


def ellipsoid_mask_torch(shape, origin=(0, 0, 0), full_shape=None, device='cuda'):
    """`ellipsoid_mask(full_shape)[origin:origin + shape]` as a uint8 torch tensor on `device`."""
    import torch
    full = tuple(int(s) for s in (full_shape or shape))
    ax = []
    for s, o, f in zip(shape, origin, full):
        c = torch.arange(o, o + s, dtype=torch.float64, device=device)
        ax.append(((c + 0.5) / f - 0.5) / 0.5)
    zz, yy, xx = ax
    r = zz[:, None, None] ** 2 + yy[None, :, None] ** 2 + xx[None, None, :] ** 2
    return (r <= 1.0).to(torch.uint8)
