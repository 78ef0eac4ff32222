"""Debug: one batch of bench config-4 blocks through the device path with the flood
fixpoint check fused (default) and unfused (CTWS_VERIFY_UNFUSED=1): which one flags?"""
import os, sys, subprocess
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
if len(sys.argv) > 1:
    import torch, numpy as np
    from bench import CONFIGS, volume_geometry
    from cluster_tools_amd import ctws
    from cluster_tools_amd.synthetic import boundary_map_torch
    cfg = CONFIGS[int(sys.argv[2])]
    nblk = int(sys.argv[3])
    geo = volume_geometry(cfg)
    dev = torch.device('cuda', 0)
    vol = boundary_map_torch(geo['gshape'], seed=cfg['seed'], device=dev, pitch=cfg.get('pitch', (24, 24, 24)),
                             origin=(geo['g0'], 0, 0), full_shape=geo['full'])
    blocks = []
    for b in geo['blocks'][:nblk]:
        osl = tuple(slice(a, c) for a, c in zip(b['obeg'], b['oend']))
        ish = [e - s for s, e in zip(b['beg'], b['end'])]
        blocks.append(dict(input=vol[osl].contiguous(), output=torch.empty(ish, dtype=torch.int64, device=dev),
                           inner_begin=[s - o for s, o in zip(b['beg'], b['obeg'])], block_id=b['block_id'],
                           crop_relabel=list(b['obeg']) != list(b['beg']) or list(b['oend']) != list(b['end'])))
    with ctws.Handle(0) as h:
        try:
            r = h.ws_blocks_device(cfg['task'], cfg['block_shape'], blocks)
            print(sys.argv[1], 'ok', h.timings().get('flood_fallback'))
        except Exception as e:
            print(sys.argv[1], 'ERROR', e)
    sys.exit(0)
for mode in ('fused', 'unfused'):
    for cfgid, n in ((4, 1), (4, 8), (4, 64), (2, 32)):
        env = dict(os.environ, CTWS_VERIFY='2', CTWS_TRACE='1')
        if mode == 'unfused':
            env['CTWS_VERIFY_UNFUSED'] = '1'
        out = subprocess.run([sys.executable, __file__, mode, str(cfgid), str(n)], env=env, capture_output=True,
                             text=True, timeout=300)
        print(cfgid, n, out.stdout.strip()[-300:], [l for l in out.stderr.splitlines() if 'verify' in l][:2])
