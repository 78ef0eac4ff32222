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

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

CONFIG2 = dict(shape=(512, 512, 512), block_shape=(64, 256, 256), halo=(0, 0, 0),
               task=dict(apply_dt_2d=False, apply_ws_2d=False))

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
    blocks = [boundary_map((bz, by, bx), seed=s) for s in (11, 12)]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-jobs', type=int, default=16)
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    cfg = CONFIG2

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, args.cpu_jobs)

    import torch
    import torch.distributed as dist
    from cluster_tools_amd import ctws
    from cluster_tools_amd.synthetic import boundary_map_torch

    torch.cuda.set_device(local_rank)
    dev = torch.device('cuda', local_rank)
    if world > 1:
        dist.init_process_group('nccl', device_id=dev)

    vol = boundary_map_torch(cfg['shape'], seed=rank, device=dev)
    blist = blocking(cfg['shape'], cfg['block_shape'], cfg['halo'])
    blocks = []
    inner_vox = 0
    outer_vox = 0
    for b in blist:
        ob, oe = b['obeg'], b['oend']
        inp = vol[ob[0]:oe[0], ob[1]:oe[1], ob[2]:oe[2]].contiguous()
        ishape = [e - s for s, e in zip(b['beg'], b['end'])]
        ibeg = [s - o for s, o in zip(b['beg'], ob)]
        out = torch.empty(ishape, dtype=torch.int64, device=dev)
        crop = ob != b['beg'] or oe != b['end']
        blocks.append(dict(input=inp, output=out, inner_begin=ibeg, crop_relabel=crop, block_id=b['block_id']))
        inner_vox += int(np.prod(ishape))
        outer_vox += int(inp.numel())
    del vol
    torch.cuda.synchronize()

    h = ctws.Handle(local_rank)
    counts = torch.zeros(len(blocks), dtype=torch.int64, device=dev)
    gathered = torch.zeros(len(blocks) * world, dtype=torch.int64, device=dev)

    def step():
        res = h.ws_blocks_device(cfg['task'], cfg['block_shape'], blocks)
        if world > 1:
            counts.copy_(torch.tensor([m for _, m in res], dtype=torch.int64))
            dist.all_gather_into_tensor(gathered, counts)
        return res

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stage_ms = {}
    for _ in range(args.steps):
        step()
        for k, v in h.timings().items():
            stage_ms[k] = stage_ms.get(k, 0.0) + v
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    stage_ms = {k: v / args.steps for k, v in stage_ms.items()}

    total_vox = inner_vox * world * args.steps
    value = total_vox / dt / 1e9
    ms_per_step = dt / args.steps * 1e3

    # roofline of the dominant kernel (by time, HIP events inside the library)
    stages = {}
    for k in STAGE_BYTES:
        stages[k] = sum(stage_ms.get(p, 0.0) for p in STAGE_PARTS.get(k, (k,)))
    stages['output'] = sum(stage_ms.get(p, 0.0) for p in STAGE_PARTS['output'])
    stage_bytes = dict(STAGE_BYTES)
    stage_gbs = {}
    for k, ms in stages.items():
        b = stage_bytes[k] * outer_vox if k in stage_bytes else INNER_BYTES * inner_vox
        stage_gbs[k] = round(b / (ms * 1e-3) / 1e9, 1) if ms > 0 else None
    # roofline of the dominant stage by time (algorithmic bytes / its HIP-event time)
    dom = max(STAGE_BYTES, key=lambda k: stages[k])
    dom_ms = stages[dom]
    achieved = STAGE_BYTES[dom] * outer_vox / (dom_ms * 1e-3) / 1e9
    alg_total = sum(STAGE_BYTES.values()) * outer_vox + INNER_BYTES * inner_vox
    pipe = alg_total / (ms_per_step * 1e-3) / 1e9

    if rank == 0:
        line = {
            'metric': 'Gvoxel/s DT-watershed (node, 1/2/4/8 GPU) + % HBM roofline; VI vs ref',
            'value': round(value, 4), 'unit': 'Gvoxel/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 3), 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32', 'data': 'synthetic',
            'config': {'workload': 'config2: synthetic 512^3 f32 boundary map, 64x256x256 blocks, halo 0, '
                                   '3-D DT watershed, size_filter 25',
                       'volume': list(cfg['shape']), 'block_shape': list(cfg['block_shape']),
                       'blocks_per_gpu': len(blocks), 'parallelism': 'blocks sharded, %d GPU(s)' % world},
            'roofline': {'bound': 'hbm', 'kernel': '%s (%s)' % (dom, STAGE_KERNELS[dom]),
                         'ms_per_step': round(dom_ms, 3), 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 4), 'traffic': None,
                         'alg_bytes_per_outer_voxel': STAGE_BYTES[dom]},
            'pipeline_roofline': {'alg_bytes_per_inner_voxel': round(alg_total / inner_vox, 1),
                                  'achieved': round(pipe, 1), 'unit': 'GB/s',
                                  'frac': round(pipe / HBM_PEAK_GBS, 4)},
            'stage_ms': {k: round(v, 3) for k, v in stage_ms.items()},
            'stage_gbs': stage_gbs,
            'cpu_baseline': cpu,
        }
        print(json.dumps(line), flush=True)
    h.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
