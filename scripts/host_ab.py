#!/usr/bin/env python
"""A/B of the host-pointer path (ctws_ws_blocks: numpy in -> numpy uint64 out) on a BASELINE
config: one JSON line per environment setting (the library reads CTWS_* when a handle opens).
Usage: python scripts/host_ab.py [--config 3] 'CTWS_HOST_THREADS=4' 'CTWS_HOST_THREADS=8 CTWS_D2H_WGS=0' ..."""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=3)
    ap.add_argument('--reps', type=int, default=2)
    ap.add_argument('settings', nargs='*')
    a = ap.parse_args()
    import torch
    import bench
    from cluster_tools_amd import ctws
    from cluster_tools_amd.synthetic import boundary_map_torch, ellipsoid_mask_torch
    cfg = bench.CONFIGS[a.config]
    geo = bench.volume_geometry(cfg)
    dev = torch.device('cuda', 0)
    vol = torch.empty(geo['gshape'], dtype=torch.uint8 if cfg.get('dtype') == 'uint8' else torch.float32, device=dev)
    for z0 in range(0, geo['gshape'][0], 32):
        z1 = min(geo['gshape'][0], z0 + 32)
        vol[z0:z1] = boundary_map_torch((z1 - z0,) + tuple(geo['gshape'][1:]), seed=cfg['seed'], device=dev,
                                        dtype=cfg.get('dtype', 'float32'), pitch=cfg.get('pitch', (24, 24, 24)),
                                        origin=(geo['g0'] + z0, 0, 0), full_shape=geo['full'])
    mvol = ellipsoid_mask_torch(geo['gshape'], (geo['g0'], 0, 0), geo['full'], device=dev) if cfg.get('mask') else None
    hb, inner = [], 0
    for b in geo['blocks']:
        osl = tuple(slice(s, e) for s, e in zip(b['obeg'], b['oend']))
        ishape = [e - s for s, e in zip(b['beg'], b['end'])]
        m = mvol[osl].cpu().numpy() if mvol is not None else None
        if m is not None:
            isl = tuple(slice(s - o, e - o) for s, e, o in zip(b['beg'], b['end'], b['obeg']))
            if not m[isl].any():
                continue
        hb.append(dict(input=vol[osl].cpu().numpy(), inner_begin=[s - o for s, o in zip(b['beg'], b['obeg'])],
                       inner_shape=ishape, block_id=b['block_id'], mask=m,
                       crop_relabel=list(b['obeg']) != list(b['beg']) or list(b['oend']) != list(b['end']),
                       out=np.empty(ishape, dtype=np.uint64)))
        inner += int(np.prod(ishape))
    del vol
    torch.cuda.synchronize()
    for setting in (a.settings or ['']):
        env = dict(kv.split('=', 1) for kv in setting.split())
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        h = ctws.Handle(0)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        h.ws_blocks(cfg['task'], cfg['block_shape'], hb)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            h.ws_blocks(cfg['task'], cfg['block_shape'], hb)
            ts.append(time.perf_counter() - t0)
        ph = {k: round(v, 1) for k, v in h.timings().items() if k.startswith('host_')}
        h.close()
        print(json.dumps({'setting': setting, 'gvox_s': round(inner / min(ts) / 1e9, 3),
                          'ms': [round(t * 1e3, 1) for t in ts], 'phases': ph}), flush=True)


if __name__ == '__main__':
    main()
