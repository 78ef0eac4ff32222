"""ctypes binding of libctws.so (include/ctws.h) — the MI355X watershed kernels.

This is the product path: there is no CPU fallback.  If the HIP library is missing or no
GPU is visible, every call raises.  Build the library with ``python __graft_entry__.py`` or
``make -C cluster_tools_amd/csrc``.
"""
import ctypes as C
import os
import threading

import numpy as np

from ._abi import CtwsBlock, make_cfg, dtype_code, CTWS_OK, CTWS_BLOCK_FAILED, CTWS_BLOCK_WRITTEN  # noqa: F401

_HERE = os.path.dirname(os.path.abspath(__file__))
# CTWS_LIB: another build of the library (A/B of build variants in one process tree)
LIB_PATH = os.environ.get('CTWS_LIB') or os.path.join(_HERE, 'libctws.so')

_lib = None
_lock = threading.Lock()


def lib():
    """Load libctws.so (raises OSError if it was not built).

    If torch is importable it is imported first: its bundled libamdhip64 then satisfies
    libctws.so's HIP dependency, so the process has ONE HIP runtime and device pointers,
    streams and contexts are shared with torch.
    """
    global _lib
    with _lock:
        if _lib is None:
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
            if not os.path.exists(LIB_PATH):
                raise OSError("libctws.so not found at %s: build it with `make -C %s/csrc`"
                              % (LIB_PATH, _HERE))
            L = C.CDLL(LIB_PATH)
            L.ctws_abi_version.restype = C.c_int
            if L.ctws_abi_version() != ABI_VERSION:
                raise OSError("libctws.so ABI version %d, expected %d (include/ctws.h): rebuild it"
                              % (L.ctws_abi_version(), ABI_VERSION))
            L.ctws_open.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
            L.ctws_close.argtypes = [C.c_void_p]
            L.ctws_close.restype = None
            L.ctws_last_error.argtypes = [C.c_void_p]
            L.ctws_last_error.restype = C.c_char_p
            for fn in ('ctws_ws_blocks', 'ctws_ws_blocks_device', 'ctws_ws_from_seeds', 'ctws_ws_from_seeds_device',
                    'ctws_eval_begin', 'ctws_eval_add', 'ctws_eval_end', 'ctws_threshold_components',
                    'ctws_threshold_components_ex', 'ctws_ufd_find'):
                getattr(L, fn).argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
            L.ctws_last_timings.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
            L.ctws_unique_u64.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_int64,
                                          C.POINTER(C.c_int64)]
            L.ctws_unique_counts_u64.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p,
                                                 C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
            L.ctws_lookup_u64.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_void_p,
                                          C.c_int64, C.POINTER(C.c_int64)]
            L.ctws_set_table_u64.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]
            L.ctws_ufd_find.argtypes = [C.c_int64, C.c_void_p, C.c_int64, C.c_void_p]
            L.ctws_threshold_components.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int64,
                                                    C.c_int64, C.c_int, C.c_int, C.c_double, C.c_int, C.c_void_p,
                                                    C.POINTER(C.c_int64)]
            L.ctws_threshold_components_ex.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int64,
                                                       C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_double, C.c_int,
                                                       C.c_double, C.c_void_p, C.POINTER(C.c_int64)]
            L.ctws_eval_begin.argtypes = [C.c_void_p, C.c_int64, C.c_int64]
            L.ctws_eval_add.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_int]
            L.ctws_eval_end.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int64)]
            L.ctws_debug_set_stop.argtypes = [C.c_void_p, C.c_int]
            L.ctws_debug_read.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_void_p, C.c_int64]
            L.ctws_debug_sqrt_int.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
            _lib = L
        return _lib


# include/ctws.h CTWS_ABI_VERSION (2: the library's own RCCL communicator entry points removed)
ABI_VERSION = 2

EXPORTED_SYMBOLS = ('ctws_abi_version', 'ctws_open', 'ctws_close', 'ctws_last_error', 'ctws_ws_blocks',
                    'ctws_ws_blocks_device', 'ctws_last_timings', 'ctws_unique_u64', 'ctws_unique_counts_u64', 'ctws_set_table_u64', 'ctws_lookup_u64',
                    'ctws_debug_set_stop', 'ctws_debug_read', 'ctws_debug_sqrt_int', 'ctws_ws_from_seeds', 'ctws_ws_from_seeds_device',
                    'ctws_eval_begin', 'ctws_eval_add', 'ctws_eval_end', 'ctws_threshold_components',
                    'ctws_threshold_components_ex', 'ctws_ufd_find')


def ufd_find(n_labels, pairs):
    """nifty.ufd.boost_ufd(n_labels).merge(pairs); .find(arange(n_labels)) in libctws.so (host
    code, no GPU handle): the representative of every label, uint64."""
    pairs = np.ascontiguousarray(np.asarray(pairs, dtype=np.uint64).reshape(-1, 2))
    out = np.empty(int(n_labels), dtype=np.uint64)
    ret = lib().ctws_ufd_find(int(n_labels), pairs.ctypes.data if pairs.size else None, len(pairs),
                              out.ctypes.data)
    if ret != CTWS_OK:
        raise CtwsError("ctws_ufd_find failed (%i): labels out of range" % ret)
    return out


class CtwsError(RuntimeError):
    pass


class Handle:
    """One library handle = one GPU, one HIP stream, one device workspace."""

    def __init__(self, device=0):
        self._h = C.c_void_p()
        ret = lib().ctws_open(int(device), C.byref(self._h))
        if ret != CTWS_OK:
            raise CtwsError("ctws_open(device=%i) failed with %i (no HIP device?)" % (device, ret))
        self.device = device

    def close(self):
        if self._h:
            lib().ctws_close(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *args):
        self.close()

    def _check(self, ret, what):
        if ret != CTWS_OK:
            msg = lib().ctws_last_error(self._h)
            raise CtwsError("%s failed (%i): %s" % (what, ret, msg.decode() if msg else ''))

    def last_error(self):
        """Message of the last call (also set, with status CTWS_BLOCK_FAILED, for failed blocks)."""
        msg = lib().ctws_last_error(self._h)
        return msg.decode() if msg else ''

    def timings(self):
        n = lib().ctws_last_timings(self._h, None, None, 0)
        names = (C.c_char_p * n)()
        ms = (C.c_float * n)()
        lib().ctws_last_timings(self._h, names, ms, n)
        return {names[i].decode(): float(ms[i]) for i in range(n)}

    # ---- test hooks ----------------------------------------------------------------------
    def debug_set_stop(self, stage):
        self._check(lib().ctws_debug_set_stop(self._h, int(stage)), 'ctws_debug_set_stop')

    def debug_read(self, array, block, shape):
        dt = {'fin': np.float32, 'dt': np.float32, 'seedmap': np.float32, 'hmap': np.float32,
              'labels': np.uint32, 'cls': np.uint8}[array]
        out = np.empty(shape, dtype=dt)
        self._check(lib().ctws_debug_read(self._h, array.encode(), int(block), out.ctypes.data, out.nbytes),
                    'ctws_debug_read')
        return out

    def debug_sqrt_int(self, n0, count):
        """The EDT's integer sqrt (k_edt.hip sqrt_rn_int) of n0 .. n0 + count - 1, as float32."""
        out = np.empty(int(count), dtype=np.float32)
        self._check(lib().ctws_debug_sqrt_int(self._h, int(n0), int(count), out.ctypes.data), 'ctws_debug_sqrt_int')
        return out

    # ---- host (numpy) blocks ------------------------------------------------------------
    def ws_blocks(self, config, block_shape, blocks, pass_id=0):
        """Run `_ws_block` on numpy blocks (see oracle.ws_blocks for the dict layout).

        Returns [{'output': inner uint64, 'status': int, 'max_label': int}, ...].
        """
        cfg = make_cfg(config, block_shape, pass_id)
        n = len(blocks)
        arr = (CtwsBlock * n)()
        keep, results = [], []
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
            out = b.get('out')
            if out is None:
                out = np.empty(ishape, dtype=np.uint64)  # (every voxel of a written block is set)
            assert out.dtype == np.uint64 and out.flags.c_contiguous and out.shape == ishape
            keep.append(out)
            c.output = out.ctypes.data
            results.append({'output': out})
        self._check(lib().ctws_ws_blocks(self._h, C.byref(cfg), arr, n), 'ctws_ws_blocks')
        for i, r in enumerate(results):
            r['status'] = int(arr[i].status)
            r['max_label'] = int(arr[i].max_label)
            r['n_ids'] = int(arr[i].n_ids)
        return results

    # ---- device (torch) blocks ----------------------------------------------------------
    def ws_blocks_device(self, config, block_shape, blocks, pass_id=0):
        """Same with torch tensors resident on this GPU: blocks[i] has 'input' (outer tensor),
        'output' (inner uint64/int64 tensor), optional 'mask' (uint8 tensor), 'initial_seeds'
        (outer int64 tensor, pass 2), 'inner_begin', 'crop_relabel', 'block_id'.
        Returns [(status, max_label, n_ids)]."""
        import torch
        cfg = make_cfg(config, block_shape, pass_id)
        n = len(blocks)
        arr = (CtwsBlock * n)()
        # the library runs on its own stream: make torch's pending writes visible first (torch's
        # stream only: other handles' streams on this device keep running)
        torch.cuda.current_stream(blocks[0]['input'].device if blocks else None).synchronize()
        codes = {'torch.uint8': 1, 'torch.uint16': 2, 'torch.float32': 3, 'torch.float64': 4}
        for i, b in enumerate(blocks):
            inp = b['input']
            assert inp.is_contiguous() and inp.is_cuda
            c = arr[i]
            c.input = inp.data_ptr()
            c.input_dtype = codes[str(inp.dtype)]
            if inp.dim() == 4:
                c.n_channels = inp.shape[0]
                c.outer_shape[:] = list(inp.shape[1:])
            else:
                c.n_channels = 0
                c.outer_shape[:] = list(inp.shape)
            if b.get('mask') is not None:
                assert b['mask'].is_contiguous() and b['mask'].element_size() == 1
                c.mask = b['mask'].data_ptr()
            if b.get('initial_seeds') is not None:
                s = b['initial_seeds']
                assert s.is_contiguous() and s.element_size() == 8 and tuple(s.shape) == tuple(c.outer_shape)
                c.initial_seeds = s.data_ptr()
            out = b['output']
            assert out.is_contiguous() and out.element_size() == 8
            c.inner_begin[:] = list(b.get('inner_begin', (0, 0, 0)))
            c.inner_shape[:] = list(out.shape)
            c.crop_relabel = int(bool(b.get('crop_relabel', False)))
            c.block_id = int(b.get('block_id', 0))
            c.output = out.data_ptr()
        self._check(lib().ctws_ws_blocks_device(self._h, C.byref(cfg), arr, n), 'ctws_ws_blocks_device')
        return [(int(arr[i].status), int(arr[i].max_label), int(arr[i].n_ids)) for i in range(n)]

    # ---- WatershedFromSeeds --------------------------------------------------------------
    def ws_from_seeds(self, config, blocks):
        """WatershedFromSeeds `_ws_block[_masked]` (watershed_from_seeds.py:143-199) on numpy
        blocks: dicts with 'input' (block, 3-D or 4-D C,Z,Y,X), 'seeds' (block-shaped ids, as
        ds_seeds[bb] returns them), optional 'mask' and 'out' (uint64, block-shaped).
        Returns [{'output', 'status', 'max_label'}, ...]."""
        cfg = make_cfg(config, (1, 1, 1), 0)
        n = len(blocks)
        arr = (CtwsBlock * n)()
        keep, results = [], []
        for i, b in enumerate(blocks):
            inp = np.ascontiguousarray(b['input'])
            shape = tuple(inp.shape[-3:])
            c = arr[i]
            c.input = inp.ctypes.data
            c.input_dtype = dtype_code(inp.dtype)
            c.n_channels = inp.shape[0] if inp.ndim == 4 else 0
            c.outer_shape[:] = list(shape)
            c.inner_shape[:] = list(shape)
            seeds = np.ascontiguousarray(b['seeds'], dtype=np.uint64)
            assert seeds.shape == shape
            c.initial_seeds = seeds.ctypes.data
            keep += [inp, seeds]
            if b.get('mask') is not None:
                m = np.ascontiguousarray(b['mask'], dtype=np.uint8)
                keep.append(m)
                c.mask = m.ctypes.data
            out = b.get('out')
            if out is None:
                out = np.zeros(shape, dtype=np.uint64)
            assert out.dtype == np.uint64 and out.flags.c_contiguous and out.shape == shape
            keep.append(out)
            c.output = out.ctypes.data
            results.append({'output': out})
        self._check(lib().ctws_ws_from_seeds(self._h, C.byref(cfg), arr, n), 'ctws_ws_from_seeds')
        for i, r in enumerate(results):
            r['status'] = int(arr[i].status)
            r['max_label'] = int(arr[i].max_label)
        return results

    # ---- evaluation (VI / Rand) ---------------------------------------------------------
    def eval_begin(self, cap_labels, cap_pairs):
        """Start a contingency table for at most cap_labels distinct ids per side and
        cap_pairs distinct (gt, seg) pairs."""
        self._check(lib().ctws_eval_begin(self._h, int(cap_labels), int(cap_pairs)), 'ctws_eval_begin')

    def eval_add(self, seg, gt, ignore_gt_zero=False):
        """Add a block: numpy uint64 arrays, or torch tensors (int64 / uint64) on this GPU."""
        on_dev = hasattr(seg, 'data_ptr')
        if on_dev:
            assert seg.is_contiguous() and gt.is_contiguous() and seg.numel() == gt.numel()
            assert seg.element_size() == 8 and gt.element_size() == 8
            import torch
            torch.cuda.current_stream(seg.device).synchronize()
            ps, pg, n = seg.data_ptr(), gt.data_ptr(), seg.numel()
        else:
            seg = np.ascontiguousarray(seg, dtype=np.uint64)
            gt = np.ascontiguousarray(gt, dtype=np.uint64)
            assert seg.size == gt.size
            ps, pg, n = seg.ctypes.data, gt.ctypes.data, seg.size
        self._check(lib().ctws_eval_add(self._h, ps, pg, int(n), int(on_dev), int(bool(ignore_gt_zero))),
                    'ctws_eval_add')

    def eval_end(self):
        """{'vi-split', 'vi-merge', 'adapted-rand-error', 'rand-index', 'n_points'}."""
        sc = (C.c_double * 4)()
        npts = C.c_int64()
        self._check(lib().ctws_eval_end(self._h, sc, C.byref(npts)), 'ctws_eval_end')
        return {'vi-split': sc[0], 'vi-merge': sc[1], 'adapted-rand-error': sc[2], 'rand-index': sc[3],
                'n_points': int(npts.value)}

    def evaluate(self, seg, gt, ignore_gt_zero=False, cap_labels=None, cap_pairs=None):
        """VI / Rand of one segmentation against one groundtruth in a single table.  Without
        capacities the table is sized for the worst case (every voxel its own id), capped."""
        n = int(np.prod(seg.shape))
        cap = min(n, 1 << 26)
        self.eval_begin(cap_labels or cap, cap_pairs or cap)
        self.eval_add(seg, gt, ignore_gt_zero)
        return self.eval_end()

    # ---- RelabelWorkflow kernels ---------------------------------------------------------
    def unique_u64(self, labels):
        """np.unique of a uint64 label array on the GPU (sorted).  numpy in, numpy out."""
        lab = np.ascontiguousarray(labels, dtype=np.uint64).ravel()
        n = C.c_int64(0)
        cap = 1024
        while True:
            out = np.empty(cap, dtype=np.uint64)
            ret = lib().ctws_unique_u64(self._h, lab.ctypes.data, lab.size, 0, out.ctypes.data, cap, C.byref(n))
            if ret == -1 and n.value > cap:
                cap = n.value
                continue
            self._check(ret, 'ctws_unique_u64')
            return out[:n.value]

    def unique_counts_u64(self, labels):
        """np.unique(labels, return_counts=True) on the GPU (radix sort + run-length encoding):
        (sorted uniques uint64, counts uint64)."""
        lab = np.ascontiguousarray(labels, dtype=np.uint64).ravel()
        n = C.c_int64(0)
        cap = 1024
        while True:
            out = np.empty(cap, dtype=np.uint64)
            cnt = np.empty(cap, dtype=np.uint64)
            ret = lib().ctws_unique_counts_u64(self._h, lab.ctypes.data, lab.size, 0, out.ctypes.data,
                                               cnt.ctypes.data, cap, C.byref(n))
            if ret == -1 and n.value > cap:
                cap = n.value
                continue
            self._check(ret, 'ctws_unique_counts_u64')
            return out[:n.value], cnt[:n.value]

    def set_table_u64(self, keys, values):
        """Upload an assignment table (keys ascending) and keep it resident on the GPU."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        values = np.ascontiguousarray(values, dtype=np.uint64)
        assert keys.shape == values.shape and keys.ndim == 1
        self._check(lib().ctws_set_table_u64(self._h, keys.ctypes.data, values.ctypes.data, keys.size),
                    'ctws_set_table_u64')

    def lookup_u64(self, labels, keys=None, values=None):
        """takeDict: labels (uint64 ndarray, modified in place) through the table keys -> values
        (keys ascending; None: the resident table).  Returns the number of labels absent from
        the table (they are left unchanged)."""
        assert labels.dtype == np.uint64 and labels.flags.c_contiguous
        kp = vp = None
        nt = 0
        if keys is not None:
            keys = np.ascontiguousarray(keys, dtype=np.uint64)
            values = np.ascontiguousarray(values, dtype=np.uint64)
            kp, vp, nt = keys.ctypes.data, values.ctypes.data, keys.size
        miss = C.c_int64(0)
        self._check(lib().ctws_lookup_u64(self._h, labels.ctypes.data, labels.size, 0, kp, vp, nt, C.byref(miss)),
                    'ctws_lookup_u64')
        return int(miss.value)

    # ---- ThresholdedComponentsWorkflow kernels --------------------------------------------
    THRESHOLD_MODES = ('greater', 'less', 'equal')

    def threshold_components(self, block, threshold, mode='greater', mask=None, normalize=True, sigma=0.):
        """BlockComponents of one 3-D block on the GPU (block_components.py:143-230): members =
        block `mode` threshold inside the mask, their 26-connected components numbered 1.. in
        C-order of first appearance (skimage.morphology.label).  `block` is the dataset's values
        in its own dtype (float32 / float64 / any 8-64 bit integer): normalize = vu.normalize
        first (float32); sigma > 0 = vu.normalize(gaussianSmoothing(float32 x, sigma)); raw
        values are compared as numpy compares them with a Python float (include/ctws.h
        ctws_threshold_components_ex).  -> (uint64 labels, n_labels); n_labels 0 = no member
        (the labels are then all 0)."""
        from ._abi import TC_DTYPE_CODES
        block = np.ascontiguousarray(block)
        if block.dtype not in TC_DTYPE_CODES:
            raise ValueError("threshold_components: unsupported dtype %s" % block.dtype)
        assert block.ndim == 3, block.shape
        if mode not in self.THRESHOLD_MODES:
            raise RuntimeError("Thresholding Mode %s not supported" % mode)
        mp = None
        if mask is not None:
            mask = np.ascontiguousarray(mask).astype(np.bool_, copy=False).view(np.uint8)
            assert mask.shape == block.shape, (mask.shape, block.shape)
            mp = mask.ctypes.data
        out = np.zeros(block.shape, dtype=np.uint64)
        n = C.c_int64(0)
        self._check(lib().ctws_threshold_components_ex(self._h, block.ctypes.data, TC_DTYPE_CODES[block.dtype], mp,
                                                       *block.shape, 0, self.THRESHOLD_MODES.index(mode),
                                                       float(threshold), 1 if normalize else 0, float(sigma),
                                                       out.ctypes.data, C.byref(n)),
                    'ctws_threshold_components_ex')
        return out, int(n.value)

    def threshold_components_device(self, block, threshold, mode='greater', mask=None, normalize=True, out=None):
        """threshold_components on torch tensors on this GPU: block float32 (Z, Y, X), mask uint8
        or None, out int64 (uint64 bits; allocated if None) -> (out, n_labels).  Nothing crosses
        PCIe but the member flag and the label count; out is left unwritten when n_labels is 0."""
        import torch
        assert block.is_cuda and block.is_contiguous() and block.dtype == torch.float32 and block.dim() == 3
        if mode not in self.THRESHOLD_MODES:
            raise RuntimeError("Thresholding Mode %s not supported" % mode)
        if out is None:
            out = torch.empty(block.shape, dtype=torch.int64, device=block.device)
        assert out.is_contiguous() and out.element_size() == 8 and tuple(out.shape) == tuple(block.shape)
        mp = None
        if mask is not None:
            assert mask.is_cuda and mask.is_contiguous() and mask.dtype == torch.uint8
            assert tuple(mask.shape) == tuple(block.shape)
            mp = mask.data_ptr()
        torch.cuda.current_stream(block.device).synchronize()
        n = C.c_int64(0)
        self._check(lib().ctws_threshold_components(self._h, block.data_ptr(), mp, *block.shape, 1,
                                                    self.THRESHOLD_MODES.index(mode), float(threshold),
                                                    1 if normalize else 0, out.data_ptr(), C.byref(n)),
                    'ctws_threshold_components')
        return out, int(n.value)

    def unique_u64_device(self, labels):
        """np.unique of a uint64 (or int64) torch tensor on this GPU: the sorted uniques as a
        numpy uint64 array (the labels stay in HBM; only the uniques cross PCIe)."""
        import torch
        assert labels.is_cuda and labels.is_contiguous() and labels.element_size() == 8
        torch.cuda.current_stream(labels.device).synchronize()
        n = C.c_int64(0)
        cap = 1024
        while True:
            out = torch.empty(cap, dtype=torch.int64, device=labels.device)
            ret = lib().ctws_unique_u64(self._h, labels.data_ptr(), labels.numel(), 1, out.data_ptr(), cap,
                                        C.byref(n))
            if ret == -1 and n.value > cap:
                cap = n.value
                continue
            self._check(ret, 'ctws_unique_u64')
            return out[:n.value].cpu().numpy().view(np.uint64)

    def lookup_u64_device(self, labels, keys, values):
        """lookup_u64 on a uint64 / int64 torch tensor on this GPU (in place) with a numpy
        table; returns the number of labels absent from it."""
        import torch
        assert labels.is_cuda and labels.is_contiguous() and labels.element_size() == 8
        kd = torch.from_numpy(np.ascontiguousarray(keys, dtype=np.uint64).view(np.int64)).to(labels.device)
        vd = torch.from_numpy(np.ascontiguousarray(values, dtype=np.uint64).view(np.int64)).to(labels.device)
        torch.cuda.current_stream(labels.device).synchronize()
        miss = C.c_int64(0)
        self._check(lib().ctws_lookup_u64(self._h, labels.data_ptr(), labels.numel(), 1, kd.data_ptr(), vd.data_ptr(),
                                          kd.numel(), C.byref(miss)), 'ctws_lookup_u64')
        return int(miss.value)

    # ---- multi-GPU label-count exchange (RCCL) ------------------------------------------
