"""gzip / zlib chunk codec on libdeflate (the image's /lib/x86_64-linux-gnu/libdeflate.so.0),
through ctypes, with Python's zlib as the fallback.

The chunk payloads are DEFLATE streams in a gzip (n5 "gzip", zarr "gzip") or zlib (zarr
"zlib") wrapper, whatever library wrote them; any conforming decoder reads them, so the choice
of codec changes speed, not the data.  On the synthetic EM volumes libdeflate inflates float32
chunks 2.5x and deflates uint64 label chunks 1.8x faster than zlib 1.2.11 at the same level
(scripts/codec_probe.py).  ctypes drops the GIL for the call, so the dataset's chunk thread pool
runs the codecs in parallel; libdeflate's (de)compressor objects are not thread safe, so every
thread allocates its own (threading.local, freed when the thread ends).
"""
import ctypes as C
import threading
import zlib

import numpy as np

_lib = None
_tls = threading.local()


def _load():
    global _lib
    if _lib is None:
        try:
            L = C.CDLL('libdeflate.so.0')
        except OSError:
            _lib = False
            return _lib
        L.libdeflate_alloc_decompressor.restype = C.c_void_p
        L.libdeflate_alloc_compressor.restype = C.c_void_p
        L.libdeflate_alloc_compressor.argtypes = [C.c_int]
        for fn in ('libdeflate_gzip_decompress', 'libdeflate_zlib_decompress'):
            getattr(L, fn).argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                       C.POINTER(C.c_size_t)]
            getattr(L, fn).restype = C.c_int
        for fn in ('libdeflate_gzip_compress', 'libdeflate_zlib_compress'):
            getattr(L, fn).argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
            getattr(L, fn).restype = C.c_size_t
        L.libdeflate_free_decompressor.argtypes = [C.c_void_p]
        L.libdeflate_free_compressor.argtypes = [C.c_void_p]
        for fn in ('libdeflate_gzip_compress_bound', 'libdeflate_zlib_compress_bound'):
            getattr(L, fn).argtypes = [C.c_void_p, C.c_size_t]
            getattr(L, fn).restype = C.c_size_t
        _lib = L
    return _lib


def available():
    return bool(_load())


class _Codecs:
    """One thread's decompressor and per-level compressors; freed with the thread's locals."""

    def __init__(self, L):
        self.L = L
        self.dec = None
        self.comp = {}

    def decompressor(self):
        if self.dec is None:
            self.dec = self.L.libdeflate_alloc_decompressor()
            if not self.dec:
                raise MemoryError("libdeflate_alloc_decompressor")
        return self.dec

    def compressor(self, level):
        c = self.comp.get(level)
        if c is None:
            c = self.L.libdeflate_alloc_compressor(int(level))
            if not c:
                raise MemoryError("libdeflate_alloc_compressor(%i)" % level)
            self.comp[level] = c
        return c

    def __del__(self):
        if self.dec:
            self.L.libdeflate_free_decompressor(self.dec)
        for c in self.comp.values():
            self.L.libdeflate_free_compressor(c)


def _codecs(L):
    cs = getattr(_tls, 'codecs', None)
    if cs is None:
        cs = _tls.codecs = _Codecs(L)
    return cs


def inflate(data, nbytes):
    """Decompress one gzip- or zlib-wrapped stream whose decompressed size is `nbytes` into a
    fresh uint8 array (zlib, which also takes multi-member gzip, when libdeflate is absent or
    refuses the stream)."""
    L = _load()
    if L and len(data) >= 2:
        out = np.empty(nbytes, np.uint8)
        n = C.c_size_t(0)
        gz = data[0] == 0x1f and data[1] == 0x8b
        fn = L.libdeflate_gzip_decompress if gz else L.libdeflate_zlib_decompress
        if fn(_codecs(L).decompressor(), data, len(data), out.ctypes.data, nbytes, C.byref(n)) == 0 and n.value == nbytes:
            return out
    return np.frombuffer(zlib.decompress(data, 47), np.uint8)


def deflate(arr, wrapper, level):
    """Compress the bytes of the C-contiguous array `arr` in a 'gzip' or 'zlib' wrapper."""
    L = _load()
    if not L:
        if wrapper == 'gzip':
            c = zlib.compressobj(level, zlib.DEFLATED, 31)
            return c.compress(arr) + c.flush()
        return zlib.compress(arr, level)
    c = _codecs(L).compressor(level)
    src = np.ascontiguousarray(arr).reshape(-1).view(np.uint8)
    bound = (L.libdeflate_gzip_compress_bound if wrapper == 'gzip' else L.libdeflate_zlib_compress_bound)(c, src.size)
    buf = np.empty(bound, np.uint8)
    fn = L.libdeflate_gzip_compress if wrapper == 'gzip' else L.libdeflate_zlib_compress
    m = fn(c, src.ctypes.data, src.size, buf.ctypes.data, bound)
    if m == 0:
        raise RuntimeError("libdeflate: %s compression of %i bytes failed" % (wrapper, src.size))
    return buf[:m].tobytes()
