"""Debug: bench block 0, descent flood without fallback vs the oracle flood model."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ['CTWS_TRACE'] = '1'
os.environ['CTWS_NO_FALLBACK'] = '1'
import torch
from cluster_tools_amd import ctws
from cluster_tools_amd.synthetic import boundary_map_torch
from oracle import oracle as O
vol = boundary_map_torch((512, 512, 512), seed=0, device="cuda")[:64, :256, :256].contiguous()
x = vol.cpu().numpy()
cfg = dict(apply_dt_2d=False, apply_ws_2d=False, size_filter=0)
with ctws.Handle(0) as h:
    h.debug_set_stop(2)  # after the flood
    h.ws_blocks(cfg, (64, 256, 256), [dict(input=x, block_id=1)])
    lab = h.debug_read('labels', 0, x.shape) & np.uint32(0x7FFFFFFF)
    hm = h.debug_read('hmap', 0, x.shape)
with O.flood_model():
    r = O.ws_blocks(cfg, (64, 256, 256), [dict(input=x, block_id=1)], with_stages=True)[0]
ref = r['ws']
d = np.argwhere(lab != ref)
print('differ', len(d))
seeds = O.make_seeds(r['dt'], cfg)
for z, y, xx in d[:6]:
    print((z, y, xx), 'gpu', lab[z, y, xx], 'ref', ref[z, y, xx], 'h', repr(hm[z, y, xx]), 'seed', seeds[z, y, xx])
    for dz, dy, dx in ((-1, 0, 0), (1, 0, 0), (0, -1, 0), (0, 1, 0), (0, 0, -1), (0, 0, 1)):
        a, b, c = z + dz, y + dy, xx + dx
        if 0 <= a < 64 and 0 <= b < 256 and 0 <= c < 256:
            print('   nb', (dz, dy, dx), 'h', repr(hm[a, b, c]), 'gpu', lab[a, b, c], 'ref', ref[a, b, c], 'seed', seeds[a, b, c])
