"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU oracle (libctws_oracle.so).

The oracle restates cluster_tools' `_ws_block` / `_ws_pass2` and the vigra algorithms
they call (see ctws_oracle.cpp for the file:line map).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may use it; it is the checker,
never the product.

Parity status: vigra (the library holding the reference's arithmetic) is absent here, so
the restatement is pinned by cross-checks against scipy / scikit-image
(tests/test_oracle_crosscheck.py) — "partially pinned", see DESIGN.md.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from cluster_tools_amd._abi import CtwsBlock, make_cfg, dtype_code

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, 'libctws_oracle.so')
_lib = None


class OrcStages(C.Structure):
    _fields_ = [('input', C.c_void_p), ('dt', C.c_void_p), ('ws', C.c_void_p)]


def build():
    src = os.path.join(_HERE, 'ctws_oracle.cpp')
    if (not os.path.exists(_LIB_PATH)) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(['make', '-s', '-C', _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = C.CDLL(_LIB_PATH)
        _lib.orc_last_error.restype = C.c_char_p
        for name in ('orc_label_u8', 'orc_label_u32', 'orc_watershed', 'orc_make_seeds'):
            getattr(_lib, name).restype = C.c_int64
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _shape(a):
    return (C.c_int64 * a.ndim)(*a.shape)


def _check(ret):
    if ret < 0:
        raise RuntimeError(lib().orc_last_error().decode())
    return ret


class flood_model:
    """Context manager: run the oracle's floods with the GPU's tie-break model."""

    def __enter__(self):
        lib().orc_set_flood_model(1)

    def __exit__(self, *a):
        lib().orc_set_flood_model(0)


def distance_transform(fg, pixel_pitch=None):
    """vigra.filters.distanceTransform(fg) (background=True); fg != 0 has distance 0."""
    fg = np.ascontiguousarray(fg != 0, dtype=np.uint8)
    out = np.empty(fg.shape, dtype=np.float32)
    pitch = None if pixel_pitch is None else (C.c_double * 3)(*[float(p) for p in pixel_pitch])
    _check(lib().orc_distance_transform(_p(fg), fg.ndim, _shape(fg), pitch, _p(out)))
    return out


def gaussian_kernel(sigma):
    taps = (C.c_double * 512)()
    n = _check(lib().orc_gaussian_kernel(C.c_double(sigma), taps, 512))
    return np.array(taps[:n])


def gaussian_smoothing(x, sigma):
    x = np.ascontiguousarray(x, dtype=np.float32)
    sig = list(sigma) if isinstance(sigma, (list, tuple)) else [sigma] * x.ndim
    out = np.empty_like(x)
    _check(lib().orc_gaussian_smoothing(_p(x), x.ndim, _shape(x), (C.c_double * 3)(*sig, *([0.] * (3 - len(sig)))), _p(out)))
    return out


def local_maxima(x):
    """Plateau-aware local maxima (8-nbhd 2-D, 6-nbhd 3-D, border allowed) as uint8 mask."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty(x.shape, dtype=np.uint8)
    lib().orc_local_maxima(_p(x), x.ndim, _shape(x), _p(out))
    return out


def label_with_background(x):
    """labelMultiArrayWithBackground / labelVolumeWithBackground, direct nbhd."""
    out = np.empty(x.shape, dtype=np.uint32)
    if x.dtype == np.uint8 or x.dtype == np.bool_:
        x = np.ascontiguousarray(x, dtype=np.uint8)
        n = lib().orc_label_u8(_p(x), x.ndim, _shape(x), _p(out))
    else:
        x = np.ascontiguousarray(x, dtype=np.uint32)
        n = lib().orc_label_u32(_p(x), x.ndim, _shape(x), _p(out))
    return out, int(n)


def watershed(hmap, seeds):
    """vigra.analysis.watershedsNew(hmap, seeds=seeds) -> (labels, maxRegionLabel)."""
    h = np.ascontiguousarray(hmap, dtype=np.float32)
    lab = np.ascontiguousarray(seeds, dtype=np.uint32).copy()
    m = lib().orc_watershed(_p(h), h.ndim, _shape(h), _p(lab))
    return lab, int(m)


def make_seeds(dt, config):
    dt = np.ascontiguousarray(dt, dtype=np.float32)
    cfg = make_cfg(config, (1, 1, 1))
    out = np.empty(dt.shape, dtype=np.uint32)
    _check(lib().orc_make_seeds(_p(dt), dt.ndim, _shape(dt), C.byref(cfg), _p(out)))
    return out


def make_hmap(input_, dt, config):
    input_ = np.ascontiguousarray(input_, dtype=np.float32)
    dt = np.ascontiguousarray(dt, dtype=np.float32)
    cfg = make_cfg(config, (1, 1, 1))
    out = np.empty(dt.shape, dtype=np.float32)
    _check(lib().orc_make_hmap(_p(input_), _p(dt), dt.ndim, _shape(dt), C.byref(cfg), _p(out)))
    return out


def ws_blocks(config, block_shape, blocks, pass_id=0, with_stages=False):
    """Run `_ws_block` (pass_id 0) or `_ws_pass2` (pass_id 1) on a list of blocks.

    Each block is a dict: input (outer block ndarray, 3-D or 4-D C,Z,Y,X), mask (outer
    uint8/bool or None), inner_begin, inner_shape, crop_relabel (bool), block_id,
    initial_seeds (outer uint64, pass 2).  Returns a list of dicts with
    output (inner uint64), status, max_label and (optionally) input/dt/ws stages.
    """
    cfg = make_cfg(config, block_shape, pass_id)
    n = len(blocks)
    arr = (CtwsBlock * n)()
    keep = []
    results = []
    stages = (OrcStages * n)() if with_stages else None
    for i, b in enumerate(blocks):
        inp = np.ascontiguousarray(b['input'])
        keep.append(inp)
        c = arr[i]
        c.input = inp.ctypes.data
        c.input_dtype = dtype_code(inp.dtype)
        if inp.ndim == 4:
            c.n_channels = inp.shape[0]
            c.outer_shape[:] = inp.shape[1:]
        else:
            c.n_channels = 0
            c.outer_shape[:] = inp.shape
        oshape = tuple(c.outer_shape)
        if b.get('mask') is not None:
            m = np.ascontiguousarray(b['mask'], dtype=np.uint8)
            keep.append(m)
            c.mask = m.ctypes.data
        c.inner_begin[:] = list(b.get('inner_begin', (0, 0, 0)))
        ishape = tuple(b.get('inner_shape', oshape))
        c.inner_shape[:] = list(ishape)
        c.crop_relabel = int(bool(b.get('crop_relabel', False)))
        c.block_id = int(b.get('block_id', 0))
        if b.get('initial_seeds') is not None:
            s = np.ascontiguousarray(b['initial_seeds'], dtype=np.uint64)
            keep.append(s)
            c.initial_seeds = s.ctypes.data
        out = np.zeros(ishape, dtype=np.uint64)
        keep.append(out)
        c.output = out.ctypes.data
        res = {'output': out}
        if with_stages:
            st = {'input': np.zeros(oshape, np.float32), 'dt': np.zeros(oshape, np.float32),
                  'ws': np.zeros(oshape, np.uint32)}
            keep.extend(st.values())
            stages[i].input = st['input'].ctypes.data
            stages[i].dt = st['dt'].ctypes.data
            stages[i].ws = st['ws'].ctypes.data
            res.update(st)
        results.append(res)
    _check(lib().orc_ws_blocks(C.byref(cfg), arr, n, stages))
    for i, r in enumerate(results):
        r['status'] = int(arr[i].status)
        r['max_label'] = int(arr[i].max_label)
    return results


def ws_from_seeds(config, blocks):
    """WatershedFromSeeds `_ws_block[_masked]` (watershed/watershed_from_seeds.py:143-199) on a
    list of blocks: dicts with input (block ndarray, 3-D or 4-D C,Z,Y,X), seeds (block-shaped,
    uint64 as read from ds_seeds), mask (uint8/bool or None).  Returns dicts with output
    (uint64, block-shaped), status and max_label."""
    cfg = make_cfg(config, (1, 1, 1), 0)
    n = len(blocks)
    arr = (CtwsBlock * n)()
    keep, results = [], []
    for i, b in enumerate(blocks):
        inp = np.ascontiguousarray(b['input'])
        c = arr[i]
        c.input = inp.ctypes.data
        c.input_dtype = dtype_code(inp.dtype)
        c.n_channels = inp.shape[0] if inp.ndim == 4 else 0
        c.outer_shape[:] = inp.shape[-3:]
        c.inner_shape[:] = inp.shape[-3:]
        s = np.ascontiguousarray(b['seeds'], dtype=np.uint64)
        c.initial_seeds = s.ctypes.data
        keep += [inp, s]
        if b.get('mask') is not None:
            m = np.ascontiguousarray(b['mask'], dtype=np.uint8)
            keep.append(m)
            c.mask = m.ctypes.data
        out = np.zeros(inp.shape[-3:], dtype=np.uint64)
        keep.append(out)
        c.output = out.ctypes.data
        results.append({'output': out})
    _check(lib().orc_ws_from_seeds(C.byref(cfg), arr, n))
    for i, r in enumerate(results):
        r['status'] = int(arr[i].status)
        r['max_label'] = int(arr[i].max_label)
    return results
