#!/usr/bin/env python
"""Benchmark: blockwise DT watershed throughput (Gvoxel/s) on MI355X.

Workload (BASELINE.json configs[1]): synthetic 512^3 float32
boundary map, 64x256x256 blocks, no halo, 3-D DT watershed (apply_dt_2d = apply_ws_2d =
False), reference defaults otherwise (threshold .5, sigma_seeds 2, sigma_weights 2,
alpha .8, size_filter 25).  One step = the watershed of every block of the volume (the
`_ws_block` loop of one job), inputs resident in HBM, uint64 outputs written to HBM.

Multi-GPU (torchrun, one process per GPU): weak scaling — every rank processes its own
512^3 volume; after each step the per-block label counts are all-gathered over RCCL (the
exchange that assigns compact global id offsets).  value = voxels of all
ranks / max-over-ranks time.

The CPU baseline (rank 0, N = 1) is the oracle (C++ restatement of the reference path,
oracle/) on a bounded sample, run like LocalTask: one single-threaded process per block.
It runs before any GPU initialisation so that no process is forked from a GPU process.
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

# BASELINE.json configs; the driver's line is config 2 (configs[1]).  The
# others run with --config N as single-GPU shares (config 5: the central z-slab of 8).
D3 = dict(apply_dt_2d=False, apply_ws_2d=False)
CONFIGS = {
    2: dict(shape=(512, 512, 512), block_shape=(64, 256, 256), halo=(0, 0, 0), task=dict(D3),
            workload='config2: synthetic 512^3 f32 boundary map, 64x256x256 blocks, halo 0, 3-D DT watershed, '
                     'size_filter 25'),
    3: dict(shape=(256, 2048, 2048), block_shape=(64, 512, 512), halo=(0, 32, 32), pitch=(3, 24, 24),
            task=dict(apply_dt_2d=True, apply_ws_2d=True),
            workload='config3: synthetic anisotropic 256x2048x2048 f32, 64x512x512 blocks, halo [0,32,32], '
                     'apply_dt_2d + apply_ws_2d'),
    4: dict(shape=(1024, 1024, 1024), block_shape=(64, 256, 256), halo=(8, 32, 32), task=dict(D3),
            workload='config4 (1 GPU): synthetic 1024^3 f32, 64x256x256 blocks, halo [8,32,32], 3-D'),
    5: dict(shape=(256, 2048, 2048), full_shape=(2048, 2048, 2048), slab=3, block_shape=(64, 256, 256),
            halo=(8, 32, 32), dtype='uint8', mask=True, two_pass=True,
            task=dict(D3, size_filter=25, non_maximum_suppression=False),
            workload='config5 (1 GPU share): z-slab 3 of 8 (256x2048x2048) of a synthetic 2048^3 uint8 map '
                     'with ellipsoid mask, 64x256x256 blocks, halo [8,32,32], 3-D two-pass'),
}
CONFIG2 = CONFIGS[2]

# Algorithmic HBM bytes per OUTER voxel of each pipeline stage, 3-D f32:
STAGE_BYTES = {'prep_edt_x': 12, 'edt_yz': 20, 'smooth_seeds': 24, 'hmap': 28, 'seeds': 16,
               'flood': 12, 'size_filter': 16}
INNER_BYTES = 12  # crop / CC / offset / uint64 write, per inner voxel
# library timing marks (HIP events on the library's stream) -> pipeline stages
STAGE_PARTS = {'flood': ('descent_tile', 'flood_descent', 'flood_relax', 'flood'),
               'output': ('finalize', 'crop_cc', 'output')}
STAGE_KERNELS = {'prep_edt_x': 'k_input_minmax + k_prep_edt_x', 'edt_yz': 'k_edt_col (y, z)',
                 'smooth_seeds': 'k_gauss_col_r (z, y) + k_gauss_row_r', 'hmap': 'k_gauss_col_r + k_gauss_row_r',
                 'seeds': 'k_localmax ... k_root_label', 'flood': 'k_descent_tile + k_descent_init + k_frontier',
                 'size_filter': 'k_hist + k_size_filter + regrow flood', 'output': 'k_finalize_ws + k_output'}
HBM_PEAK_GBS = 8000.0


def _cpu_job(args):
    block, task, block_shape = args
    from oracle import oracle as O
    t0 = time.time()
    O.ws_blocks(task, block_shape, [dict(input=block, block_id=1)])
    return time.time() - t0


def cpu_baseline(cfg, n_jobs=16):
    """Oracle on a bounded sample: n_jobs blocks, one process each (LocalTask model)."""
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor
    from cluster_tools_amd.synthetic import boundary_map
    from oracle import oracle as O
    O.build()
    bz, by, bx = cfg['block_shape']
    blocks = [boundary_map((bz, by, bx), seed=s, dtype=cfg.get('dtype', 'float32')) for s in (11, 12)]
    cores = min(n_jobs, len(os.sched_getaffinity(0)))
    jobs = [(blocks[i % 2], cfg['task'], cfg['block_shape']) for i in range(n_jobs)]
    t0 = time.time()
    with ProcessPoolExecutor(cores, mp_context=mp.get_context('fork')) as pool:
        per_job = list(pool.map(_cpu_job, jobs))
    wall = time.time() - t0
    vox = n_jobs * bz * by * bx
    return {'value': vox / wall / 1e9, 'unit': 'Gvoxel/s', 'cores': cores, 'kind': 'port',
            'sample': '%d oracle jobs (one %dx%dx%d block each, single-threaded, %d processes like '
                      'LocalTask); %.1f s wall, %.2f s per block' % (n_jobs, bz, by, bx, cores, wall,
                                                                   float(np.mean(per_job)))}


def blocking(shape, block_shape, halo):
    """Block list in nifty C-order with outer/inner bbs (watershed.py:252-264)."""
    grid = [(s + b - 1) // b for s, b in zip(shape, block_shape)]
    out = []
    for bid in range(grid[0] * grid[1] * grid[2]):
        c = (bid // (grid[1] * grid[2]), (bid // grid[2]) % grid[1], bid % grid[2])
        beg = [ci * b for ci, b in zip(c, block_shape)]
        end = [min(s, bb + b) for s, bb, b in zip(shape, beg, block_shape)]
        obeg = [max(0, bb - h) for bb, h in zip(beg, halo)]
        oend = [min(s, e + h) for s, e, h in zip(shape, end, halo)]
        out.append(dict(block_id=bid, beg=beg, end=end, obeg=obeg, oend=oend))
    return out


def alg_bytes(cfg, outer_vox, inner_vox, pass2_outer):
    """Algorithmic HBM bytes of one step."""
    two_d = cfg['task'].get('apply_ws_2d', True)
    per_outer = 104 if two_d else 128
    if cfg.get('dtype', 'float32') == 'uint8':
        per_outer -= 9
    per_inner = INNER_BYTES
    if cfg.get('mask'):
        per_outer += 1
        per_inner += 1
    return per_outer * outer_vox + 8 * pass2_outer + per_inner * inner_vox


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--config', type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-jobs', type=int, default=16)
    ap.add_argument('--streams', type=int, default=3,
                    help='library handles (one HIP stream each) per GPU, driven from host threads; '
                         'the blocks are split between them so their launch-bound phases overlap')
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    cfg = CONFIGS[args.config]
    two_pass = cfg.get('two_pass', False)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, args.cpu_jobs)

    import torch
    import torch.distributed as dist
    from cluster_tools_amd import ctws
    from cluster_tools_amd.synthetic import boundary_map_torch, ellipsoid_mask_torch

    torch.cuda.set_device(local_rank)
    dev = torch.device('cuda', local_rank)
    if world > 1:
        dist.init_process_group('nccl', device_id=dev)

    shape = tuple(cfg['shape'])
    origin = (0, 0, 0)
    full = cfg.get('full_shape', shape)
    if 'slab' in cfg:
        origin = (((cfg['slab'] + rank) % (full[0] // shape[0])) * shape[0], 0, 0)
    gen = dict(seed=rank if 'full_shape' not in cfg else 0, device=dev, dtype=cfg.get('dtype', 'float32'),
               pitch=cfg.get('pitch', (24, 24, 24)), origin=origin, full_shape=full)
    vol = boundary_map_torch(shape, **gen)
    mvol = ellipsoid_mask_torch(shape, origin, full, device=dev) if cfg.get('mask') else None
    blist = blocking(shape, cfg['block_shape'], cfg['halo'])
    out_vol = torch.zeros(shape, dtype=torch.int64, device=dev) if two_pass else None

    def sl(beg, end):
        return tuple(slice(a, b) for a, b in zip(beg, end))

    blocks = {}
    inner_vox = outer_vox = pass2_outer = 0
    for b in blist:
        ob, oe = b['obeg'], b['oend']
        isl = sl(b['beg'], b['end'])
        if mvol is not None and not bool(mvol[isl].any()):
            continue  # empty inner mask: nothing to do, nothing written (watershed.py:295-297)
        inp = vol[sl(ob, oe)].contiguous()
        ishape = [e - s for s, e in zip(b['beg'], b['end'])]
        ibeg = [s - o for s, o in zip(b['beg'], ob)]
        d = dict(input=inp, output=torch.empty(ishape, dtype=torch.int64, device=dev), inner_begin=ibeg,
                 crop_relabel=list(ob) != list(b['beg']) or list(oe) != list(b['end']), block_id=b['block_id'],
                 isl=isl, osl=sl(ob, oe))
        if mvol is not None:
            d['mask'] = mvol[sl(ob, oe)].contiguous()
        blocks[b['block_id']] = d
        inner_vox += int(np.prod(ishape))
        outer_vox += int(inp.numel())
    del vol
    if two_pass:
        from cluster_tools_amd.utils.blocking import Blocking
        from cluster_tools_amd.utils import volume_utils as vu
        lists = vu.make_checkerboard_block_lists(Blocking([0, 0, 0], list(shape), list(cfg['block_shape'])))
        passes = [[blocks[i] for i in lst if i in blocks] for lst in lists]
        for b in passes[1]:
            b['crop_relabel'] = False
            b['initial_seeds'] = torch.empty(tuple(b['input'].shape[-3:]), dtype=torch.int64, device=dev)
            pass2_outer += int(b['input'].numel())
    else:
        passes = [list(blocks.values())]
    torch.cuda.synchronize()

    nstreams = max(1, min(args.streams, min(len(p) for p in passes)))
    handles = [ctws.Handle(local_rank) for _ in range(nstreams)]
    pool = ThreadPoolExecutor(nstreams) if nstreams > 1 else None
    nblocks = len(blocks)
    counts = torch.zeros(nblocks, dtype=torch.int64, device=dev)
    gathered = torch.zeros(nblocks * world, dtype=torch.int64, device=dev)
    stage_ms = {}

    def step(record, ns=None, into=None):
        ns = nstreams if ns is None else ns
        into = stage_ms if into is None else into
        res = []
        for pid, pblocks in enumerate(passes):
            if pid == 1:
                for b in pblocks:  # initial_seeds = ds_out[input_bb] (two_pass_watershed.py:228)
                    b['initial_seeds'].copy_(out_vol[b['osl']])
            # contiguous shares of the pass's blocks, one per handle (stream)
            parts = [pblocks[len(pblocks) * i // ns:len(pblocks) * (i + 1) // ns] for i in range(ns)]

            def run(i):
                return handles[i].ws_blocks_device(cfg['task'], cfg['block_shape'], parts[i], pass_id=pid)

            rs = list(pool.map(run, range(ns))) if ns > 1 else [run(0)]
            r = [x for part in rs for x in part]
            if record:
                # stage times summed over the handles (overlapping streams: an upper bound)
                for hh in handles[:ns]:
                    for k, v in hh.timings().items():
                        into[k] = into.get(k, 0.0) + v
            if two_pass:
                for b, (st, _) in zip(pblocks, r):
                    if st in (0, 2):
                        out_vol[b['isl']] = b['output']
            res += r
        if world > 1:
            counts.copy_(torch.tensor([m for _, m in res], dtype=torch.int64))
            dist.all_gather_into_tensor(gathered, counts)
        return res

    for _ in range(args.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    stage_ms = {k: v / args.steps for k, v in stage_ms.items()}
    # roofline durations: one more, untimed step with every block on ONE stream, so that no
    # other stream's kernels share the chip while a launch runs (with concurrent streams the
    # HIP-event duration of a launch includes the time it shares)
    stage_1 = {}
    if nstreams > 1:
        step(True, ns=1, into=stage_1)
        torch.cuda.synchronize()
    else:
        stage_1 = stage_ms

    total_vox = inner_vox * world * args.steps
    value = total_vox / dt / 1e9
    ms_per_step = dt / args.steps * 1e3

    def per_stage(sm):
        st = {}
        for k in STAGE_BYTES:
            st[k] = sum(sm.get(p, 0.0) for p in STAGE_PARTS.get(k, (k,)))
        st['output'] = sum(sm.get(p, 0.0) for p in STAGE_PARTS['output'])
        return st

    stages = per_stage(stage_1)
    stage_gbs = {}
    for k, ms in stages.items():
        b = STAGE_BYTES[k] * outer_vox if k in STAGE_BYTES else INNER_BYTES * inner_vox
        stage_gbs[k] = round(b / (ms * 1e-3) / 1e9, 1) if ms > 0 else None
    # roofline of the dominant stage by time (algorithmic bytes / its single-stream HIP-event time)
    dom = max(STAGE_BYTES, key=lambda k: stages[k])
    dom_ms = stages[dom]
    achieved = STAGE_BYTES[dom] * outer_vox / (dom_ms * 1e-3) / 1e9
    alg_total = alg_bytes(cfg, outer_vox, inner_vox, pass2_outer)
    pipe = alg_total / (ms_per_step * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(HERE, 'profiles', 'pmc_traffic.json')
    if args.config == 2 and os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get(dom)

    if rank == 0:
        line = {
            'metric': 'Gvoxel/s DT-watershed (node, 1/2/4/8 GPU) + % HBM roofline; VI vs ref',
            'value': round(value, 4), 'unit': 'Gvoxel/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 3), 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': cfg.get('dtype', 'float32').replace('float', 'f'),
            'data': 'synthetic',
            'config': {'workload': cfg['workload'], 'volume': list(shape), 'block_shape': list(cfg['block_shape']),
                       'halo': list(cfg['halo']), 'blocks_per_gpu': nblocks, 'passes': len(passes),
                       'streams_per_gpu': nstreams,
                       'parallelism': 'blocks sharded, %d GPU(s)' % world},
            'roofline': {'bound': 'hbm', 'kernel': '%s (%s)' % (dom, STAGE_KERNELS[dom]),
                         'ms_per_step': round(dom_ms, 3), 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 4), 'traffic': traffic,
                         'alg_bytes_per_outer_voxel': STAGE_BYTES[dom],
                         'timing': 'HIP events on the library stream, one untimed step with all blocks on 1 stream',
                         'traffic_unit': 'HBM bytes per step of the stage (profiles/pmc_traffic.json)'},
            'pipeline_roofline': {'alg_bytes_per_inner_voxel': round(alg_total / inner_vox, 1),
                                  'achieved': round(pipe, 1), 'unit': 'GB/s',
                                  'frac': round(pipe / HBM_PEAK_GBS, 4)},
            'stage_ms': {k: round(v, 3) for k, v in stage_ms.items()},
            'stage_ms_1stream': {k: round(v, 3) for k, v in stage_1.items()},
            'stage_gbs': stage_gbs,
            'cpu_baseline': cpu,
        }
        print(json.dumps(line), flush=True)
    for hh in handles:
        hh.close()
    if pool:
        pool.shutdown()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
