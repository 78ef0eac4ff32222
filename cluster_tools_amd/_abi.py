"""ctypes mirror of include/ctws.h (the C-ABI of libctws.so).

Pure data definitions: the ctws_cfg / ctws_block structs and the helpers that fill
them from a watershed task config (watershed.py:50-60 keys, with the inline
``config.get`` defaults the job code applies) and from numpy blocks.
"""
import ctypes as C

import numpy as np

CTWS_OK = 0
CTWS_U8, CTWS_U16, CTWS_F32, CTWS_F64 = 1, 2, 3, 4
CTWS_AGG = {'mean': 0, 'max': 1, 'min': 2}
CTWS_BLOCK_WRITTEN, CTWS_BLOCK_SKIPPED_MASK, CTWS_BLOCK_EMPTY, CTWS_BLOCK_EMPTY_PASS2, CTWS_BLOCK_FAILED = 0, 1, 2, 3, 4

_DTYPE_CODES = {np.dtype('uint8'): CTWS_U8, np.dtype('uint16'): CTWS_U16,
                np.dtype('float32'): CTWS_F32, np.dtype('float64'): CTWS_F64}
# ctws_threshold_components_ex also takes the integer dtypes (include/ctws.h CTWS_I8 .. CTWS_U64)
TC_DTYPE_CODES = dict(_DTYPE_CODES)
TC_DTYPE_CODES.update({np.dtype('int8'): 5, np.dtype('int16'): 6, np.dtype('int32'): 7, np.dtype('uint32'): 8,
                       np.dtype('int64'): 9, np.dtype('uint64'): 10})


class CtwsCfg(C.Structure):
    _fields_ = [('threshold', C.c_double),
                ('alpha', C.c_double),
                ('sigma_seeds', C.c_double * 3),
                ('sigma_seeds_is_list', C.c_int32),
                ('sigma_weights', C.c_double * 3),
                ('sigma_weights_is_list', C.c_int32),
                ('size_filter', C.c_int32),
                ('apply_dt_2d', C.c_int32),
                ('apply_ws_2d', C.c_int32),
                ('has_pixel_pitch', C.c_int32),
                ('pixel_pitch', C.c_double * 3),
                ('invert_inputs', C.c_int32),
                ('channel_begin', C.c_int32),
                ('channel_end', C.c_int32),
                ('agglomerate_channels', C.c_int32),
                ('non_maximum_suppression', C.c_int32),
                ('pass_id', C.c_int32),
                ('block_shape', C.c_int64 * 3)]


class CtwsBlock(C.Structure):
    _fields_ = [('input', C.c_void_p),
                ('input_dtype', C.c_int32),
                ('n_channels', C.c_int32),
                ('outer_shape', C.c_int64 * 3),
                ('mask', C.c_void_p),
                ('inner_begin', C.c_int64 * 3),
                ('inner_shape', C.c_int64 * 3),
                ('crop_relabel', C.c_int32),
                ('_pad0', C.c_int32),
                ('block_id', C.c_int64),
                ('initial_seeds', C.c_void_p),
                ('output', C.c_void_p),
                ('max_label', C.c_uint64),
                ('status', C.c_int32),
                ('n_ids', C.c_int32)]


def _sigma(value):
    """(values[3], is_list) for a sigma config entry (scalar or per-axis list)."""
    if isinstance(value, (list, tuple)):
        vals = [float(v) for v in value]
        if len(vals) != 3:
            # apply_filter asserts len(sigma) == input_.ndim (volume_utils.py:97-98)
            raise ValueError("per-axis sigma must have 3 entries, got %r" % (value,))
        return vals, 1
    return [float(value or 0.0)] * 3, 0


def make_cfg(config, block_shape, pass_id=0):
    """Fill a CtwsCfg from a watershed task/job config dict.

    Defaults are the inline ``config.get`` defaults of the reference job code
    (watershed.py:141,152-153,180-181,212-215, :269-281), which can differ from
    ``default_task_config`` (e.g. ``non_maximum_suppression``: True inline).
    """
    cfg = CtwsCfg()
    cfg.threshold = float(config.get('threshold', .5))
    cfg.alpha = float(config.get('alpha', 0.8))
    vals, is_list = _sigma(config.get('sigma_seeds', 2.))
    cfg.sigma_seeds[:] = vals
    cfg.sigma_seeds_is_list = is_list
    vals, is_list = _sigma(config.get('sigma_weights', 2.))
    cfg.sigma_weights[:] = vals
    cfg.sigma_weights_is_list = is_list
    cfg.size_filter = int(config.get('size_filter', 25))
    cfg.apply_dt_2d = int(bool(config.get('apply_dt_2d', True)))
    cfg.apply_ws_2d = int(bool(config.get('apply_ws_2d', True)))
    pitch = config.get('pixel_pitch', None)
    if pitch is not None:
        cfg.has_pixel_pitch = 1
        cfg.pixel_pitch[:] = [float(p) for p in pitch]
    else:
        cfg.pixel_pitch[:] = [1., 1., 1.]
    cfg.invert_inputs = int(bool(config.get('invert_inputs', False)))
    cfg.channel_begin = int(config.get('channel_begin', 0))
    ce = config.get('channel_end', None)
    cfg.channel_end = -1 if ce is None else int(ce)
    agg = config.get('agglomerate_channels', 'mean')
    assert agg in ('mean', 'max', 'min')
    cfg.agglomerate_channels = CTWS_AGG[agg]
    # NMS needs nifty.filters.nonMaximumDistanceSuppression, which is not available;
    # the reference then logs and continues without it (watershed.py:180-184).
    cfg.non_maximum_suppression = 0
    cfg.pass_id = int(pass_id)
    cfg.block_shape[:] = [int(b) for b in block_shape]
    return cfg


def dtype_code(dtype):
    try:
        return _DTYPE_CODES[np.dtype(dtype)]
    except KeyError:
        raise ValueError("unsupported input dtype %s" % dtype)
