"""Debug: pass 2 on the wide keys (CTWS_FORCE_WIDE=1) vs the flood model."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..', 'tests'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
from oracle import oracle as O
from pass2_cases import scenario
from cluster_tools_amd import ctws

os.environ['CTWS_FORCE_WIDE'] = '1'
hw = ctws.Handle(0)
os.environ.pop('CTWS_FORCE_WIDE')
for name in sys.argv[1:]:
    config, bs, blocks = scenario(name)
    for sf in (None, 0):
        cfg = dict(config) if sf is None else dict(config, size_filter=sf)
        with O.flood_model():
            ref = O.ws_blocks(cfg, bs, blocks, pass_id=1)
        res = hw.ws_blocks(cfg, bs, blocks, pass_id=1)
        t = hw.timings()
        bad = [int((g['output'] != r['output']).sum()) for g, r in zip(res, ref)]
        print(name, 'sf', sf, 'diffs', bad, 'status', [g['status'] for g in res], [r['status'] for r in ref],
              {k: v for k, v in t.items() if 'rerun' in k or 'fallback' in k or 'auto' in k}, flush=True)
        for g, r in zip(res, ref):
            d = g['output'] != r['output']
            if d.any():
                z = np.argwhere(d)[:, 0]
                print('   slices', np.unique(z).tolist()[:20], 'gpu ids', np.unique(g['output'][d])[:8].tolist(),
                      'ref ids', np.unique(r['output'][d])[:8].tolist(), flush=True)
