"""Debug: flood labels of config-4 blocks run alone vs in one batch (CTWS_VERIFY=0)."""
import os, sys
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
os.environ['CTWS_VERIFY'] = '0'
import numpy as np
from bench import CONFIGS, volume_geometry
from cluster_tools_amd import ctws
from cluster_tools_amd.synthetic import boundary_map
cfg = CONFIGS[4]
geo = volume_geometry(cfg)
ids = [int(a) for a in sys.argv[1].split(',')]
blocks = []
for b in geo['blocks']:
    if b['block_id'] not in ids:
        continue
    osh = [e - s for s, e in zip(b['obeg'], b['oend'])]
    x = boundary_map(osh, seed=cfg['seed'], origin=b['obeg'], full_shape=geo['full'])
    blocks.append(dict(input=x, block_id=b['block_id'], inner_begin=[s - o for s, o in zip(b['beg'], b['obeg'])],
                       inner_shape=[e - s for s, e in zip(b['beg'], b['end'])], crop_relabel=True))
with ctws.Handle(0) as h:
    h.debug_set_stop(2)
    h.ws_blocks(cfg['task'], cfg['block_shape'], blocks)
    together = [h.debug_read('labels', i, b['input'].shape) for i, b in enumerate(blocks)]
    print('batch timings', {k: v for k, v in h.timings().items() if 'iters' in k})
    for i, b in enumerate(blocks):
        h.ws_blocks(cfg['task'], cfg['block_shape'], [b])
        alone = h.debug_read('labels', 0, b['input'].shape)
        d = np.argwhere(alone != together[i])
        print('block', b['block_id'], b['input'].shape, 'diff voxels', len(d), d[:5].tolist(),
              {k: v for k, v in h.timings().items() if 'iters' in k})
