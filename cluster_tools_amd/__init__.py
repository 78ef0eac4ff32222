"""MI355X-native blockwise DT watershed with the cluster_tools task surface.

The hot path (k-dominik/cluster_tools ``watershed/watershed.py:_ws_block``) runs as
hand-written HIP kernels for gfx950 in ``libctws.so`` (C-ABI: ``include/ctws.h``),
loaded by ``cluster_tools_amd.ctws`` via ctypes.
"""
__version__ = '0.1.0'
