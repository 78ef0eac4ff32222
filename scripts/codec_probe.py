"""zlib vs libdeflate (cluster_tools_amd/io/deflate.py) on a synthetic float32 boundary chunk and a
uint64 label chunk: compression ratio, compress and inflate MB/s per thread."""
import sys, time, zlib, ctypes as C, numpy as np
sys.path.insert(0, '/root/repo')
from cluster_tools_amd.synthetic import boundary_map
L = C.CDLL('libdeflate.so.0')
L.libdeflate_alloc_decompressor.restype = C.c_void_p
L.libdeflate_alloc_compressor.restype = C.c_void_p
L.libdeflate_alloc_compressor.argtypes = [C.c_int]
L.libdeflate_gzip_decompress.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
L.libdeflate_gzip_compress.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
L.libdeflate_gzip_compress.restype = C.c_size_t
L.libdeflate_gzip_compress_bound.argtypes = [C.c_void_p, C.c_size_t]
L.libdeflate_gzip_compress_bound.restype = C.c_size_t
x = boundary_map((32, 256, 256), seed=1).astype(np.float32)
lab = (np.arange(32*256*256, dtype=np.uint64) // 700 + 123456789).reshape(32,256,256)
for name, arr in (('float', x), ('labels', lab)):
    raw = arr.astype(arr.dtype.newbyteorder('>')).tobytes()
    co = zlib.compressobj(5, zlib.DEFLATED, 31); t = time.perf_counter(); g = co.compress(raw) + co.flush(); tz = time.perf_counter() - t
    t = time.perf_counter(); d = zlib.decompress(g, 47); tzd = time.perf_counter() - t
    d = L.libdeflate_alloc_decompressor(); out = np.empty(len(raw), np.uint8); n = C.c_size_t()
    t = time.perf_counter()
    for _ in range(5): r = L.libdeflate_gzip_decompress(d, g, len(g), out.ctypes.data, len(raw), C.byref(n))
    tld = (time.perf_counter() - t) / 5
    assert r == 0 and n.value == len(raw) and out.tobytes() == raw
    for lvl in (1, 5, 6):
        c = L.libdeflate_alloc_compressor(lvl); cap = L.libdeflate_gzip_compress_bound(c, len(raw)); buf = np.empty(cap, np.uint8)
        t = time.perf_counter(); m = L.libdeflate_gzip_compress(c, raw, len(raw), buf.ctypes.data, cap); tlc = time.perf_counter() - t
        assert zlib.decompress(buf[:m].tobytes(), 47) == raw
        print(name, 'libdeflate level', lvl, 'ratio %.2f' % (len(raw) / m), 'compress %.0f MB/s' % (len(raw) / tlc / 1e6))
    print(name, 'zlib5 ratio %.2f compress %.0f MB/s inflate %.0f MB/s; libdeflate inflate %.0f MB/s' % (len(raw)/len(g), len(raw)/tz/1e6, len(raw)/tzd/1e6, len(raw)/tld/1e6))
