#!/usr/bin/env python
"""Benchmark: blockwise DT watershed throughput (Gvoxel/s) on MI355X.

Default workload (BASELINE.json configs[2], SURVEY.md §8(d) config 3 — the largest single-GPU
configuration): a synthetic anisotropic 256x2048x2048 float32 boundary map (cells of 3x24x24
voxels), 64x512x512 blocks with halo [0, 32, 32] (outer blocks 64x576x576), apply_dt_2d +
apply_ws_2d, reference defaults otherwise (threshold .5, sigma_seeds 2, sigma_weights 2,
alpha .8, size_filter 25).  One step = the `_ws_block` of every block of the volume: read the
outer block, EDT, seeds, hmap, flood, size filter + regrow, halo crop +
labelVolumeWithBackground, uint64 output with the block id offset.  `value` counts inner
(output) voxels; inputs are resident in HBM when the timed region starts and the uint64
outputs are written to HBM.  The PCIe-inclusive rate (host numpy input -> host numpy uint64
output through ctws_ws_blocks) is reported beside it as `host_resident`.

`--config N` runs the other BASELINE configs on one GPU (config 2: 512^3 3-D; config 4: 1024^3
with halo [8,32,32]; config 5: one z-slab share of the 2048^3 uint8 two-pass run).

Multi-GPU, one process per GPU: `--gpus N` starts the N ranks itself (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR / MASTER_PORT in each child's environment, before anything in the
parent touches a GPU; the parent waits and fails when a rank fails), or runs as one rank of a
torchrun launch when WORLD_SIZE is set.  Weak scaling (`value`): every rank processes its own
z-slab volume of the config; after each step the per-block label counts are all-gathered over
RCCL and exclusively scanned into compact global id offsets (the exchange of
relabel/find_labeling.py:104-116).  value = inner voxels of all ranks / max-over-ranks time.
`strong_config4` (every run): config 4's whole 1024^3 volume cut into N z-slabs of the block grid
(BASELINE.json configs[3]: "blocks sharded over 8 MI355X, RCCL label-offset scan").
Ranks that share a GPU (a rehearsal on a 1-GPU box) use a gloo group instead of RCCL.

The CPU baseline (rank 0, N = 1) is the oracle (oracle/, the C++ restatement of the
reference path) on a bounded sample of the same workload, driven like LocalTask: one
single-threaded process per block, n_jobs = min(n_blocks, cores).  It runs before any GPU
initialisation so that no process is forked from a GPU process.  Worker 0's oracle output
is compared with the GPU output of the same block (VI, adapted Rand).
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

# BASELINE.json configs.  The single-GPU headline is config 3.
D3 = dict(apply_dt_2d=False, apply_ws_2d=False)
CONFIGS = {
    2: dict(shape=(512, 512, 512), block_shape=(64, 256, 256), halo=(0, 0, 0), task=dict(D3), seed=0,
            workload='config2: synthetic 512^3 f32 boundary map, 64x256x256 blocks, halo 0, 3-D DT watershed, '
                     'size_filter 25'),
    3: dict(shape=(256, 2048, 2048), block_shape=(64, 512, 512), halo=(0, 32, 32), pitch=(3, 24, 24), seed=1,
            task=dict(apply_dt_2d=True, apply_ws_2d=True, halo=[0, 32, 32]),
            workload='config3: synthetic anisotropic 256x2048x2048 f32 EM-like boundary map, 64x512x512 blocks, '
                     'halo [0,32,32], apply_dt_2d + apply_ws_2d, size_filter 25'),
    4: dict(shape=(1024, 1024, 1024), block_shape=(64, 256, 256), halo=(8, 32, 32), task=dict(D3, halo=[8, 32, 32]),
            seed=2,
            workload='config4 (1 GPU): synthetic 1024^3 f32, 64x256x256 blocks, halo [8,32,32], 3-D'),
    5: dict(shape=(256, 2048, 2048), full_shape=(2048, 2048, 2048), slab=3, block_shape=(64, 256, 256),
            halo=(8, 32, 32), dtype='uint8', mask=True, two_pass=True, seed=3,
            task=dict(D3, size_filter=25, non_maximum_suppression=False, halo=[8, 32, 32]),
            workload='config5 (1 GPU share): z-slab 3 of 8 (256x2048x2048) of a synthetic 2048^3 uint8 map '
                     'with ellipsoid mask, 64x256x256 blocks, halo [8,32,32], 3-D two-pass'),
}
DEFAULT_CONFIG = 3

# Algorithmic HBM bytes per OUTER voxel of each stage: the minimal
# one-read / one-write traffic; iterative kernels count once.
STAGE_BYTES_3D = {'prep_edt_x': 12, 'edt_yz': 20, 'smooth_seeds': 24, 'hmap': 28, 'seeds': 16, 'flood': 12,
                  'size_filter': 16}
STAGE_BYTES_2D = {'prep_edt_x': 12, 'edt_yz': 12, 'smooth_seeds': 16, 'hmap': 20, 'seeds': 16, 'flood': 12,
                  'size_filter': 16}
# per INNER voxel: crop CC (labels read) and the uint64 output write
INNER_STAGE_BYTES = {'crop_cc': 4, 'output': 8}
# library timing marks (HIP events on the library's stream) -> stages
STAGE_PARTS = {'flood': ('descent_tile', 'flood_descent', 'flood_relax', 'flood_verify', 'flood'),
               'crop_cc': ('finalize', 'crop_cc'), 'output': ('output',)}
STAGE_KERNELS = {'prep_edt_x': 'k_input_minmax + k_prep_edt_x_reg', 'edt_yz': 'k_edt_col (y[, z])',
                 'smooth_seeds': 'k_gauss_col_r + k_gauss_row_r', 'hmap': 'k_gauss_col_r + k_gauss_row_r',
                 'seeds': 'k_localmax + k_tile_cc/k_tile_merge + bitmap rank',
                 'flood': 'k_descent_tile + k_descent_init + k_frontier + k_flood_verify',
                 'size_filter': 'k_hist2d/k_hist + k_regrow_init + k_frontier',
                 'crop_cc': 'k_tile_cc<CROP> + k_tile_merge + k_flatten_roots + bitmap rank',
                 'output': 'k_output'}
HBM_PEAK_GBS = 8000.0


def stage_bytes(cfg):
    """{stage: (bytes per unit, 'outer' | 'inner')} for the config."""
    two_d = cfg['task'].get('apply_ws_2d', True)
    sb = {k: [v, 'outer'] for k, v in (STAGE_BYTES_2D if two_d else STAGE_BYTES_3D).items()}
    if cfg.get('dtype', 'float32') == 'uint8':
        sb['prep_edt_x'][0] -= 6   # min/max and EDT-x reads of the raw input: 1 B instead of 4
        sb['hmap'][0] -= 3
    if cfg.get('mask'):
        sb['prep_edt_x'][0] += 1
    for k, v in INNER_STAGE_BYTES.items():
        sb[k] = [v + (1 if (cfg.get('mask') and k == 'output') else 0), 'inner']
    return sb


def alg_bytes(cfg, outer_vox, inner_vox, pass2_outer):
    """Algorithmic HBM bytes of one step."""
    tot = 0
    for k, (b, unit) in stage_bytes(cfg).items():
        tot += b * (outer_vox if unit == 'outer' else inner_vox)
    return tot + 8 * pass2_outer


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


def volume_geometry(cfg, rank=0, world=1, scaling='weak'):
    """The rank's share of the workload.

    weak (the per-GPU work is fixed): every rank owns a z-slab of cfg['shape'] of one volume:
    config 5's slabs are those of the 2048^3 volume (slab cfg['slab'] on one GPU, slab `rank`
    on N); the other configs stack N slabs into an (N * Z, Y, X) volume of the same map.
    strong (the volume is fixed): the config's whole volume (cfg['full_shape'] or
    cfg['shape']: config 4's 1024^3, config 5's 2048^3) is cut into N z-slabs along the block
    grid, each rank a contiguous range of block rows (SURVEY.md §8(e) partitioning).
    A rank processes the blocks of the volume's global block grid whose inner block lies in
    its slab, with their full halos (a halo that reaches into a neighbouring slab is generated
    from the same map), and global block ids.  Returns full (volume shape), z0 (slab start),
    g0 / gshape (the generated region: slab + z halos) and the blocks with bounding boxes in
    region coordinates.
    """
    Z, Y, X = cfg['shape']
    if scaling == 'strong':
        full = tuple(cfg.get('full_shape', cfg['shape']))
        bz = cfg['block_shape'][0]
        nzb = (full[0] + bz - 1) // bz
        r0, r1 = nzb * rank // world, nzb * (rank + 1) // world
        z0, z1 = r0 * bz, min(full[0], r1 * bz)
    else:
        if 'full_shape' in cfg:
            full = tuple(cfg['full_shape'])
            slab = cfg['slab'] if world == 1 else rank % (full[0] // Z)
        else:
            full = (Z * world, Y, X)
            slab = rank
        z0, z1 = slab * Z, slab * Z + Z
    Z = z1 - z0
    hz = cfg['halo'][0]
    g0, g1 = max(0, z0 - hz), min(full[0], z0 + Z + hz)
    blocks = []
    for b in blocking(full, cfg['block_shape'], cfg['halo']):
        if not z0 <= b['beg'][0] < z0 + Z:
            continue
        d = dict(b)
        for k in ('beg', 'end', 'obeg', 'oend'):
            d[k] = [d[k][0] - g0] + list(d[k][1:])
        blocks.append(d)
    return dict(full=full, z0=z0, g0=g0, gshape=(g1 - g0, Y, X), lo=z0 - g0, hi=g1 - (z0 + Z), blocks=blocks)


# ---- CPU baseline (oracle) -----------------------------------------------------------------
_BARRIER = None


def _cpu_init(barrier):
    global _BARRIER
    _BARRIER = barrier


def _cpu_job(args):
    """One LocalTask-like job: generate its block (untimed), wait for all jobs, run the oracle."""
    cfg_id, b, want_output = args
    from oracle import oracle as O
    from cluster_tools_amd.synthetic import boundary_map, ellipsoid_mask_sub
    cfg = CONFIGS[cfg_id]
    geo = volume_geometry(cfg)
    full = geo['full']
    ob = [b['obeg'][0] + geo['g0']] + list(b['obeg'][1:])
    oshape = [e - s for s, e in zip(b['obeg'], b['oend'])]
    x = boundary_map(oshape, seed=cfg['seed'], pitch=cfg.get('pitch', (24, 24, 24)),
                     dtype=cfg.get('dtype', 'float32'), origin=ob, full_shape=full)
    blk = dict(input=x, block_id=b['block_id'], inner_begin=[s - o for s, o in zip(b['beg'], b['obeg'])],
               inner_shape=[e - s for s, e in zip(b['beg'], b['end'])],
               crop_relabel=list(b['obeg']) != list(b['beg']) or list(b['oend']) != list(b['end']))
    if cfg.get('mask'):
        blk['mask'] = ellipsoid_mask_sub(oshape, ob, full)
    _BARRIER.wait()
    t0 = time.time()
    res = O.ws_blocks(cfg['task'], cfg['block_shape'], [blk])[0]
    t1 = time.time()
    return t0, t1, (res['output'] if want_output else None)


def block_colour(cfg, geo, b):
    """Checkerboard colour of a block: 0 for the list of block 0 (make_checkerboard_block_lists,
    volume_utils.py:142-205: even coordinate sum)."""
    c = [(bb + (geo['g0'] if k == 0 else 0)) // s for k, (bb, s) in enumerate(zip(b['beg'], cfg['block_shape']))]
    return sum(c) % 2


def cpu_model():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def effective_cores():
    """CPUs this process may use: the affinity mask, capped by the cgroup CPU quota (a GPU box
    shares a large host: nproc shows all of its CPUs, the quota is this job's share)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            quota, period = f.read().split()[:2]
        if quota != 'max':
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(cfg_id, max_cores=None):
    """Oracle over the first n_jobs = min(n_blocks, cores) blocks, one process per block
    (LocalTask: n_jobs = min(n_blocks, max_jobs), cluster_tasks.py:500,524-529, with max_jobs =
    the CPUs this job may use)."""
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor
    from oracle import oracle as O
    O.build()
    cfg = CONFIGS[cfg_id]
    geo = volume_geometry(cfg)
    blist = geo['blocks']
    if cfg.get('two_pass'):
        blist = [b for b in blist if block_colour(cfg, geo, b) == 0]   # pass-1 blocks (_ws_block)
    cores = effective_cores() if not max_cores else min(max_cores, effective_cores())
    n_jobs = min(len(blist), cores)
    ctx = mp.get_context('fork')
    barrier = ctx.Barrier(n_jobs)
    jobs = [(cfg_id, blist[i], i == 0) for i in range(n_jobs)]
    with ProcessPoolExecutor(n_jobs, mp_context=ctx, initializer=_cpu_init, initargs=(barrier,)) as pool:
        res = list(pool.map(_cpu_job, jobs))
    wall = max(r[1] for r in res) - min(r[0] for r in res)
    inner = sum(int(np.prod([e - s for s, e in zip(b['beg'], b['end'])])) for b in blist[:n_jobs])
    per = [r[1] - r[0] for r in res]
    out = {'value': inner / wall / 1e9, 'unit': 'Gvoxel/s', 'cores': n_jobs, 'kind': 'port',
           'cpu': cpu_model(),
           'sample': '%d of the config\'s %d blocks, one single-threaded oracle process per block (LocalTask '
                     'model, n_jobs = min(n_blocks, %d usable cores: affinity and cgroup quota, %d online)); '
                     '%.1f s wall, %.1f s mean per block'
                     % (n_jobs, len(blist), cores, os.cpu_count() or 0, wall, float(np.mean(per)))}
    return out, (blist[0]['block_id'], res[0][2])


def pcie_rates(dev, nbytes=1 << 30, reps=4):
    """Pinned host <-> HBM copy rates (GB/s) of this box: each direction alone, and both at once on
    two streams (full duplex: the host path's uploads and downloads overlap)."""
    import torch
    hin = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    hout = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    din = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dout = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def run(h2d, d2h):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            if h2d:
                with torch.cuda.stream(s1):
                    din.copy_(hin, non_blocking=True)
            if d2h:
                with torch.cuda.stream(s2):
                    hout.copy_(dout, non_blocking=True)
        torch.cuda.synchronize()
        return nbytes * reps / (time.perf_counter() - t0) / 1e9

    run(True, True)
    out = {'h2d_gbs': round(run(True, False), 1), 'd2h_gbs': round(run(False, True), 1),
           'duplex_each_gbs': round(run(True, True), 1), 'bytes_per_copy': nbytes}
    del hin, hout, din, dout
    return out


def threshcc_leg(dev, shape=(128, 512, 512), reps=10):
    """BlockComponents of ThresholdedComponentsWorkflow (k_threshcc.hip) on
    one synthetic block of smooth blobs (uniform noise, two 5^3 box filters on the GPU),
    normalized and thresholded at 0.5, input and labels in HBM.  The CPU oracle
    (oracle/threshcc.py: scipy ndimage.label, one core) runs on the first quarter in z, which
    is also checked bit-exact against the GPU."""
    import torch
    import torch.nn.functional as F
    from cluster_tools_amd import ctws
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand((1, 1) + tuple(shape), generator=g, device=dev)
    for _ in range(2):
        x = F.avg_pool3d(x, 5, stride=1, padding=2, count_include_pad=False)
    x = x[0, 0].contiguous()
    n_vox = x.numel()
    with ctws.Handle(dev.index or 0) as h:
        out = torch.empty(shape, dtype=torch.int64, device=dev)
        for _ in range(2):
            h.threshold_components_device(x, .5, 'greater', out=out)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            _, n = h.threshold_components_device(x, .5, 'greater', out=out)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        sub = x[:shape[0] // 4].contiguous()
        lab, _ = h.threshold_components_device(sub, .5, 'greater')
        lab = lab.cpu().numpy().view(np.uint64)
    from oracle import threshcc as T
    xs = sub.cpu().numpy()
    t0 = time.perf_counter()
    ref, _ = T.block_components(xs, .5, 'greater')
    t_cpu = time.perf_counter() - t0
    traffic = None
    pmc = os.path.join(HERE, 'profiles', 'pmc_traffic_threshcc.json')
    if os.path.exists(pmc) and tuple(shape) == (128, 512, 512):
        with open(pmc) as f:
            traffic = json.load(f).get('total_bytes_per_call')
    return {'workload': 'BlockComponents, %s smooth blobs, normalize + threshold 0.5, 26-connected' % 'x'.join(map(str, shape)),
            'value': round(n_vox / dt / 1e9, 3), 'unit': 'Gvoxel/s', 'ms_per_block': round(dt * 1e3, 3),
            'n_labels': n, 'alg_bytes_per_voxel': 28,
            'roofline': {'bound': 'hbm', 'achieved': round(28 * n_vox / dt / 1e9, 1), 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': round(28 * n_vox / dt / 1e9 / HBM_PEAK_GBS, 4), 'traffic': traffic,
                         'traffic_unit': 'HBM bytes per block call, rocprofv3 FETCH_SIZE x2 + WRITE_SIZE on the same '
                                         'block shape (profiles/pmc_traffic_threshcc.json)'},
            'cpu_baseline': {'value': round(xs.size / t_cpu / 1e9, 4), 'unit': 'Gvoxel/s', 'cores': 1, 'kind': 'port',
                             'sample': 'first %d z-slices of the block' % xs.shape[0]},
            'bit_exact_vs_oracle_on_sample': bool(np.array_equal(lab, ref))}


def end_to_end(cfg_id, dev, z_extent=None, max_jobs=4, threads=4):
    """The product path from file to file: WatershedWorkflow
    (target 'local', GPU jobs, the relabel inside the watershed jobs) from an n5 gzip input to the
    relabelled n5 uint64 output with its assignment table and maxId, on the whole config volume
    (z_extent slices of it when given, or when the temp file system cannot hold the uncompressed
    leg: 64).  Run twice: with the datasets gzip-compressed (n5 default, watershed.py:80-83) and
    uncompressed; the difference is the gzip share.  The input file is written before the timed
    region."""
    import json as _json
    import shutil
    import subprocess
    import tempfile
    import torch
    from cluster_tools_amd.synthetic import boundary_map_torch
    from cluster_tools_amd.utils import volume_utils as vu
    cfg = CONFIGS[cfg_id]
    if z_extent is None:
        # the raw leg holds the float32 input and the uint64 output uncompressed
        raw_bytes = 12 * int(np.prod(cfg['shape']))
        z_extent = cfg['shape'][0] if shutil.disk_usage(tempfile.gettempdir()).free > 3 * raw_bytes else 64
    shape = (min(z_extent, cfg['shape'][0]),) + tuple(cfg['shape'][1:])
    x = boundary_map_torch(shape, seed=cfg['seed'], device=dev, dtype=cfg.get('dtype', 'float32'),
                           pitch=cfg.get('pitch', (24, 24, 24))).cpu().numpy()
    out = {'volume': list(shape), 'block_shape': list(cfg['block_shape']), 'max_jobs': max_jobs,
           'threads_per_job': threads,
           'workflow': 'WatershedWorkflow(target=local), GPU jobs, relabel in the jobs (relabel_in_job)'}
    root = tempfile.mkdtemp(prefix='ctws_e2e_')
    try:
        for comp in ('gzip', 'raw'):
            d = os.path.join(root, comp)
            os.makedirs(os.path.join(d, 'configs'))
            env = dict(os.environ, CTWS_N5_COMPRESSION=comp)
            inp = os.path.join(d, 'data.n5')
            os.environ['CTWS_N5_COMPRESSION'] = comp
            with vu.file_reader(inp) as f:
                ds = f.create_dataset('boundaries', shape=shape, dtype=x.dtype,
                                      chunks=tuple(b // 2 for b in cfg['block_shape']))
                ds.n_threads = 16
                ds[...] = x
            os.environ.pop('CTWS_N5_COMPRESSION', None)
            glob = {'block_shape': list(cfg['block_shape']), 'shebang': '#! ' + sys.executable,
                    'roi_begin': None, 'roi_end': None, 'max_num_retries': 0, 'block_list_path': None}
            with open(os.path.join(d, 'configs', 'global.config'), 'w') as f:
                _json.dump(glob, f)
            from cluster_tools_amd.watershed.watershed import WatershedLocal
            tc = WatershedLocal.default_task_config()
            tc.update(cfg['task'])
            tc['threads_per_job'] = threads
            with open(os.path.join(d, 'configs', 'watershed.config'), 'w') as f:
                _json.dump(tc, f)
            for name in ('find_uniques', 'find_labeling', 'write'):
                with open(os.path.join(d, 'configs', name + '.config'), 'w') as f:
                    _json.dump({'threads_per_job': threads}, f)
            code = ('import sys; sys.path.insert(0, %r)\n'
                    'from cluster_tools_amd import luigi_compat as luigi\n'
                    'from cluster_tools_amd.watershed import WatershedWorkflow\n'
                    'wf = WatershedWorkflow(input_path=%r, input_key="boundaries", output_path=%r, output_key="ws", '
                    'config_dir=%r, tmp_folder=%r, target="local", max_jobs=%d)\n'
                    'sys.exit(0 if luigi.build([wf], local_scheduler=True) else 1)\n'
                    % (HERE, inp, os.path.join(d, 'ws.n5'), os.path.join(d, 'configs'), os.path.join(d, 'tmp'),
                       max_jobs))
            t0 = time.perf_counter()
            rc = subprocess.call([sys.executable, '-c', code], env=env, stdout=subprocess.DEVNULL,
                                 stderr=subprocess.DEVNULL)
            t = time.perf_counter() - t0
            if rc != 0:
                out['error_' + comp] = 'workflow failed (rc %d)' % rc
                continue
            n = int(np.prod(shape))
            out[comp] = {'s': round(t, 2), 'gvoxel_s': round(n / t / 1e9, 4),
                         'input_bytes_on_disk': int(sum(os.path.getsize(os.path.join(dp, fn))
                                                        for dp, _, fs in os.walk(inp) for fn in fs)),
                         'output_bytes_on_disk': int(sum(os.path.getsize(os.path.join(dp, fn))
                                                         for dp, _, fs in os.walk(os.path.join(d, 'ws.n5'))
                                                         for fn in fs))}
            shutil.rmtree(d, ignore_errors=True)
        if 'gzip' in out and 'raw' in out:
            out['gzip_share'] = round(1.0 - out['raw']['s'] / out['gzip']['s'], 3)
            out['value'] = out['gzip']['gvoxel_s']
            out['unit'] = 'Gvoxel/s'
    finally:
        shutil.rmtree(root, ignore_errors=True)
    return out


def progress(msg):
    """A line on stderr per phase: long profiler passes show they are alive."""
    print('[bench %.1fs] %s' % (time.time() - _T0, msg), file=sys.stderr, flush=True)


_T0 = time.time()


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`--gpus N` without a launcher: start N ranks of this script (one process per GPU) and wait.

    Runs before anything in this process touches a GPU (no exec from a GPU process).  Children
    get the torchrun environment; rank 0 prints the JSON line.  A failing rank ends the others
    (their exact PIDs) and the parent exits with its code."""
    import subprocess
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), CTWS_BENCH_CHILD='1')
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            code = p.poll()
            if code is None:
                continue
            alive.remove(p)
            if code != 0 and rc == 0:
                rc = code
                print('[bench] rank %d exited with %d: stopping the other ranks' % (procs.index(p), code),
                      file=sys.stderr, flush=True)
                for q in alive:
                    q.terminate()
        time.sleep(0.2)
    return rc


def dist_env():
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', str(rank)))
    return world, rank, local_rank


def launch_check():
    """--launch-check: the process group of the ranks, no GPU (tests/test_bench_launch.py)."""
    import torch
    import torch.distributed as dist
    world, rank, local_rank = dist_env()
    if os.environ.get('CTWS_BENCH_FAIL_RANK') == str(rank):
        sys.exit(3)  # test hook: a rank that dies before joining the group
    dist.init_process_group('gloo', rank=rank, world_size=world)
    t = torch.tensor([rank, local_rank, world], dtype=torch.int64)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    if rank == 0:
        print(json.dumps({'launch_check': True, 'world_size': dist.get_world_size(),
                          'ranks': [p.tolist() for p in parts]}), flush=True)
    dist.destroy_process_group()


def run_workload(cfg_id, scaling, rank, world, dev, steps, warmup, nstreams_req, host_pass=False,
                 keep_block=None, keep_volume=False):
    """Stage one workload in HBM, run `warmup` + timed `steps` steps, and measure it.

    A step = the `_ws_block` (and `_ws_pass2`) of every block of the rank's share, then the RCCL
    offset scan.  Returns the timing, the per-stage HIP-event times of one extra single-stream
    step, the algorithmic bytes, and (host_pass, rank 0) the PCIe-inclusive rate."""
    import torch
    from cluster_tools_amd import ctws
    from cluster_tools_amd.synthetic import boundary_map_torch, ellipsoid_mask_torch
    from cluster_tools_amd.watershed import sharded
    import torch.distributed as dist
    cfg = CONFIGS[cfg_id]
    two_pass = cfg.get('two_pass', False)
    geo = volume_geometry(cfg, rank, world, scaling)
    full = geo['full']
    origin = (geo['g0'], 0, 0)
    gen = dict(seed=cfg['seed'], device=dev, dtype=cfg.get('dtype', 'float32'), pitch=cfg.get('pitch', (24, 24, 24)),
               origin=origin, full_shape=full)
    # generated slab by slab (per-voxel deterministic: identical to one call), with progress
    vol = torch.empty(geo['gshape'], dtype=torch.uint8 if cfg.get('dtype') == 'uint8' else torch.float32, device=dev)
    zs = 32
    for z0 in range(0, geo['gshape'][0], zs):
        z1 = min(geo['gshape'][0], z0 + zs)
        vol[z0:z1] = boundary_map_torch((z1 - z0,) + tuple(geo['gshape'][1:]),
                                        **dict(gen, origin=(origin[0] + z0, 0, 0)))
    progress('config %d (%s): synthetic input of rank %d generated, %s' % (cfg_id, scaling, rank, geo['gshape']))
    mvol = ellipsoid_mask_torch(geo['gshape'], origin, full, device=dev) if cfg.get('mask') else None
    blist = geo['blocks']
    # two-pass: the pass-1 labels of the region (own slab + z halos from the neighbour ranks)
    out_vol = torch.zeros(geo['gshape'], dtype=torch.int64, device=dev) if two_pass else None

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
        colour = {b['block_id']: block_colour(cfg, geo, b) for b in blist}
        p1 = [blocks[i] for i in sorted(blocks) if colour[i] == 0]
        p2 = [blocks[i] for i in sorted(blocks) if colour[i] == 1]
        for b in p2:
            b['crop_relabel'] = False
            b['initial_seeds'] = torch.empty(tuple(b['input'].shape[-3:]), dtype=torch.int64, device=dev)
            pass2_outer += int(b['input'].numel())
        # pass 2 in the workflow's schedule (watershed.make_batches): dependency levels of the
        # sequential loop over the pass-2 blocks of ALL ranks (the ones that write: non-empty
        # inner mask), each level reading ds_out after the levels before it wrote -- on this rank
        # or, through the z halos, on a neighbour.  The z halos are exchanged before level 0 (the
        # pass-1 labels) and after every level that wrote rows another rank's halo reads
        # (sharded.pass2_rank_schedule)
        writers = set(sharded.all_gather_ints([b['block_id'] for b in p2], device=dev)) if world > 1 else \
            set(b['block_id'] for b in p2)
        geos = [volume_geometry(cfg, r, world, scaling) for r in range(world)] if world > 1 else [geo]
        slabs = [(g['z0'], g['z0'] + g['gshape'][0] - g['lo'] - g['hi']) for g in geos]

        def gsl(g, beg, end):
            return sl([beg[0] + g['g0']] + list(beg[1:]), [end[0] + g['g0']] + list(end[1:]))
        glist = sorted((b['block_id'], r, gsl(g, b['obeg'], b['oend']), gsl(g, b['beg'], b['end']))
                       for r, g in enumerate(geos) for b in g['blocks'] if b['block_id'] in writers)
        lv, exch, xboxes = sharded.pass2_rank_schedule([x[1:] for x in glist], slabs, cfg['halo'][0], boxes=True)
        level = {x[0]: l for x, l in zip(glist, lv)}
        # level 0: the whole halo rows (pass 1 wrote everywhere); later levels: only the (y, x)
        # footprints of the blocks that wrote next to a slab boundary since
        groups = [(0, p1, False)] + [(1, [b for b in p2 if level[b['block_id']] == k],
                                      True if k == 0 else (xboxes[k] if exch[k] else False))
                                     for k in range(len(exch))]
    else:
        groups = [(0, list(blocks.values()), False)]
    # (empty pass-2 levels stay: every rank exchanges at the same levels)
    groups = [(pid, g, x) for pid, g, x in groups if g or x]
    torch.cuda.synchronize()

    nstreams = max(1, min(nstreams_req, max(len(g) for _, g, _ in groups)))
    handles = [ctws.Handle(dev.index) for _ in range(nstreams)]
    pool = ThreadPoolExecutor(nstreams) if nstreams > 1 else None
    stage_ms = {}
    offsets = {}

    def step(record, ns=None, into=None):
        ns = nstreams if ns is None else ns
        into = stage_ms if into is None else into
        res = []
        for pid, gblocks, exch in groups:
            if pid == 1:
                if exch is True:
                    # the neighbour slabs' labels in the z halos (point-to-point)
                    sharded.exchange_z_halos(out_vol, geo['lo'], geo['hi'])
                elif exch:
                    sharded.exchange_z_halo_boxes(out_vol, geo['lo'], geo['hi'], exch.get((rank, 'lo'), []),
                                                  exch.get((rank, 'hi'), []), exch.get((rank - 1, 'hi'), []),
                                                  exch.get((rank + 1, 'lo'), []))
                for b in gblocks:  # initial_seeds = ds_out[input_bb] (two_pass_watershed.py:228)
                    b['initial_seeds'].copy_(out_vol[b['osl']])
            if not gblocks:
                continue
            nsg = max(1, min(ns, len(gblocks)))
            # contiguous shares of the group's blocks, one per handle (stream)
            parts = [gblocks[len(gblocks) * i // nsg:len(gblocks) * (i + 1) // nsg] for i in range(nsg)]

            def run(i):
                return handles[i].ws_blocks_device(cfg['task'], cfg['block_shape'], parts[i], pass_id=pid)

            rs = list(pool.map(run, range(nsg))) if nsg > 1 else [run(0)]
            r = [x for part in rs for x in part]
            if record:
                # stage times summed over the handles (overlapping streams: an upper bound)
                for hh in handles[:nsg]:
                    for k, v in hh.timings().items():
                        into[k] = into.get(k, 0.0) + v
            if two_pass:
                for b, (st, _, _) in zip(gblocks, r):
                    if st in (0, 2):
                        out_vol[b['isl']] = b['output']
            res += r
        if not two_pass:
            # compact global id offsets: exclusive scan of the per-block distinct-id counts of
            # all ranks (relabel/find_labeling.py:104-116 over RCCL instead of .npy files)
            allc = sharded.gather_counts([k for _, _, k in res], device=dev)
            offsets['scan'], offsets['n_ids'] = sharded.compact_offsets(allc)
        return res

    for k in range(warmup):
        step(False)
        progress('config %d warmup step %d' % (cfg_id, k))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(True)
        progress('config %d step %d' % (cfg_id, k))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt_rank = time.perf_counter() - t0
    dt = sharded.all_reduce_max(dt_rank, device=dev)
    ms_ranks = [round(t / steps * 1e3, 3) for t in sharded.all_gather_float(dt_rank, device=dev)]
    stage_ms = {k: v / steps for k, v in stage_ms.items()}
    # roofline durations: one more, untimed step with every block on ONE stream, so that no
    # other stream's kernels share the chip while a launch runs (with concurrent streams the
    # HIP-event duration of a launch includes the time it shares)
    stage_1 = {}
    if nstreams > 1:
        step(True, ns=1, into=stage_1)
        torch.cuda.synchronize()
    else:
        stage_1 = stage_ms
    inner_all = sharded.all_reduce_sum_int(inner_vox, device=dev)

    host = None
    if host_pass and rank == 0 and not two_pass:
        hb = []
        for b in groups[0][1]:
            hb.append(dict(input=b['input'].cpu().numpy(), inner_begin=b['inner_begin'],
                           inner_shape=list(b['output'].shape), crop_relabel=b['crop_relabel'],
                           block_id=b['block_id'],
                           mask=b['mask'].cpu().numpy() if b.get('mask') is not None else None,
                           out=np.empty(tuple(b['output'].shape), dtype=np.uint64)))
        handles[0].ws_blocks(cfg['task'], cfg['block_shape'], hb)  # warm the staging buffers
        ths = []
        for _ in range(max(1, min(3, steps))):
            t0 = time.perf_counter()
            handles[0].ws_blocks(cfg['task'], cfg['block_shape'], hb)
            ths.append(time.perf_counter() - t0)
        th = min(ths)
        phases = {k: round(v, 2) for k, v in handles[0].timings().items() if k.startswith('host_')}
        same = all(np.array_equal(h_['out'], b['output'].cpu().numpy().view(np.uint64))
                   for h_, b in zip(hb, groups[0][1]))
        h2d = int(sum(x['input'].nbytes + (x['mask'].nbytes if x['mask'] is not None else 0) for x in hb))
        host = {'value': round(inner_vox / th / 1e9, 4), 'unit': 'Gvoxel/s', 'ms_per_step': round(th * 1e3, 3),
                'runs_ms': [round(t * 1e3, 1) for t in ths],
                'path': 'ctws_ws_blocks: host numpy input -> pinned staging -> HBM -> uint32 local labels -> '
                        'pinned -> widened with the block id offset into the host numpy uint64 output, one handle',
                'h2d_bytes': h2d, 'd2h_bytes': int(inner_vox * 4), 'host_output_bytes': int(inner_vox * 8),
                'phases_ms': phases, 'pcie': pcie_rates(dev), 'matches_device_path': bool(same),
                'method': 'its own leg after the config-5 leg (round 5 on): the best of %d calls of '
                          'ctws_ws_blocks over the whole workload on one handle (one stream), after one '
                          'warm-up call; not comparable with the round-4 field, which came from the '
                          'headline run' % len(ths), 'calls': len(ths), 'streams': 1}
        del hb
    kept = None
    if keep_block is not None and keep_block in blocks:
        kept = blocks[keep_block]['output'].cpu().numpy().view(np.uint64)
    kept_volume = None
    if keep_volume and two_pass:
        # the rank's own slab rows of the labels (tests/test_bench_two_pass_ranks.py)
        kept_volume = out_vol[geo['lo']:geo['gshape'][0] - geo['hi']].cpu().numpy().view(np.uint64)
    for hh in handles:
        hh.close()
    if pool:
        pool.shutdown()
    out = dict(cfg_id=cfg_id, geo=geo, full=full, dt=dt, ms_ranks=ms_ranks, steps=steps,
               inner_vox=inner_vox, outer_vox=outer_vox, pass2_outer=pass2_outer, inner_all=inner_all,
               nblocks=len(blocks), npass=2 if two_pass else 1, ngroups=len(groups), nstreams=nstreams,
               stage_ms=stage_ms, stage_1=stage_1, n_ids=offsets.get('n_ids'), host=host, kept=kept,
               kept_volume=kept_volume, n_exchanges=sum(1 for pid, _, x in groups if pid == 1 and x))
    del blocks, groups, out_vol, mvol
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def roofline_of(cfg, m):
    """Per-stage GB/s, the dominant stage's roofline and the pipeline roofline of a measurement."""
    def per_stage(sm):
        return {k: sum(sm.get(p, 0.0) for p in STAGE_PARTS.get(k, (k,))) for k in stage_bytes(cfg)}
    sbytes = stage_bytes(cfg)
    stages = per_stage(m['stage_1'])
    stage_gbs = {}
    for k, ms in stages.items():
        b, unit = sbytes[k]
        nbytes = b * (m['outer_vox'] if unit == 'outer' else m['inner_vox'])
        stage_gbs[k] = round(nbytes / (ms * 1e-3) / 1e9, 1) if ms > 0 else None
    # roofline of the dominant stage by time (algorithmic bytes / its single-stream HIP-event time)
    dom = max(stages, key=lambda k: stages[k])
    dom_ms = stages[dom]
    b_unit, unit = sbytes[dom]
    dom_bytes = b_unit * (m['outer_vox'] if unit == 'outer' else m['inner_vox'])
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    ms_per_step = m['dt'] / m['steps'] * 1e3
    alg_total = alg_bytes(cfg, m['outer_vox'], m['inner_vox'], m['pass2_outer'])
    pipe = alg_total / (ms_per_step * 1e-3) / 1e9
    return dict(dom=dom, dom_ms=dom_ms, dom_bytes=dom_bytes, b_unit=b_unit, unit=unit, achieved=achieved,
                stage_gbs=stage_gbs, alg_total=alg_total, pipe=pipe, ms_per_step=ms_per_step)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--config', type=int, default=DEFAULT_CONFIG, choices=sorted(CONFIGS))
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-host', action='store_true', help='skip the host-resident (PCIe-inclusive) pass')
    ap.add_argument('--no-e2e', action='store_true', help='skip the end-to-end n5 workflow run')
    ap.add_argument('--no-strong', action='store_true', help='skip the strong-scaling config 4 run')
    ap.add_argument('--no-threshcc', action='store_true', help='skip the thresholded-components block leg')
    ap.add_argument('--no-config5', action='store_true',
                    help='skip the config-5 leg (one GPU\'s z-slab of the 2048^3 uint8 two-pass workload)')
    ap.add_argument('--config5-steps', type=int, default=3)
    ap.add_argument('--strong-steps', type=int, default=3)
    ap.add_argument('--e2e-z', type=int, default=None,
                    help='z extent of the end-to-end volume (default: the whole config volume)')
    ap.add_argument('--cpu-cores', type=int, default=0, help='cap on the CPU baseline jobs (0: usable cores)')
    ap.add_argument('--scaling', choices=('weak', 'strong'), default='weak',
                    help='weak: every rank runs the config\'s single-GPU workload (default); strong: the '
                         'config\'s whole volume (config 4: 1024^3, config 5: 2048^3) in z-slabs over the ranks')
    ap.add_argument('--streams', type=int, default=3,
                    help='library handles (one HIP stream each) per GPU, driven from host threads; '
                         'the blocks are split between them so their launch-bound phases overlap')
    ap.add_argument('--launch-check', action='store_true',
                    help='start the ranks and their process group only (no GPU): a launcher test')
    args = ap.parse_args()

    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        # no launcher around us: start the ranks ourselves (nothing here has touched a GPU)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world, rank, local_rank = dist_env()
    if args.launch_check:
        launch_check()
        return
    if world != args.gpus:
        progress('WORLD_SIZE %d overrides --gpus %d' % (world, args.gpus))
    cfg = CONFIGS[args.config]
    two_pass = cfg.get('two_pass', False)

    cpu, ref_block = None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, ref_block = cpu_baseline(args.config, args.cpu_cores)

    import torch
    import torch.distributed as dist

    ndev = torch.cuda.device_count()  # (does not initialise the GPU)
    dev_index = local_rank % max(1, ndev)
    torch.cuda.set_device(dev_index)
    dev = torch.device('cuda', dev_index)
    backend = None
    if world > 1:
        # RCCL needs one device per rank; ranks sharing a GPU (a rehearsal) use gloo
        backend = os.environ.get('CTWS_DIST_BACKEND') or ('nccl' if ndev >= world else 'gloo')
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group('gloo')
    devices = sorted(set(int(x) for x in (sharded_gather_devices(dev_index, dev) if world > 1 else [dev_index])))

    m = run_workload(args.config, args.scaling, rank, world, dev, args.steps, args.warmup, args.streams,
                     host_pass=False, keep_block=ref_block[0] if ref_block else None)
    rf = roofline_of(cfg, m)
    value = m['inner_all'] * args.steps / m['dt'] / 1e9

    # ---- config 5: one rank's z-slab of the 2048^3 uint8 masked volume through
    # the workflow's two-pass schedule (pass 1, the z-halo exchange, pass 2 in the dependency
    # levels of the sequential loop) -- BASELINE.json's heaviest config, beside the headline
    c5 = None
    if not args.no_config5 and args.config != 5:
        progress('config 5 leg')
        torch.cuda.empty_cache()
        s5 = run_workload(5, 'weak', rank, world, dev, args.config5_steps, 2, args.streams)
        r5 = roofline_of(CONFIGS[5], s5)
        fl5 = sum(s5['stage_1'].get(p, 0.0) for p in STAGE_PARTS['flood'])
        c5 = {'value': round(s5['inner_all'] * s5['steps'] / s5['dt'] / 1e9, 4), 'unit': 'Gvoxel/s',
              'ms_per_step': round(r5['ms_per_step'], 3), 'ms_per_step_ranks': s5['ms_ranks'],
              'steps': s5['steps'], 'n_gpus': world, 'scaling': 'weak', 'workload': CONFIGS[5]['workload'],
              'blocks_per_gpu': s5['nblocks'], 'inner_voxels_per_gpu': s5['inner_vox'],
              'outer_voxels_per_gpu': s5['outer_vox'], 'pass2_outer_voxels': s5['pass2_outer'],
              'launch_groups': s5['ngroups'], 'z_halo_exchanges': s5['n_exchanges'],
              'pipeline_roofline': {'alg_bytes_per_inner_voxel': round(r5['alg_total'] / s5['inner_vox'], 1),
                                    'achieved': round(r5['pipe'], 1), 'unit': 'GB/s',
                                    'frac': round(r5['pipe'] / HBM_PEAK_GBS, 4)},
              'flood_ms_1stream': round(fl5, 3),
              'flood_frac': round(12 * s5['outer_vox'] / (fl5 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if fl5 > 0 else None,
              'stage_ms_1stream': {k: round(v, 3) for k, v in s5['stage_1'].items() if v >= 0.05}}

    # ---- the host-pointer path (PCIe-inclusive rate) of the main config, after the config-5
    # leg: run before it, its pinned staging and host pools left that leg's host-bound two-pass
    # schedule 179 ms per step instead of 157 (profiles/r05/config5/leg_after_host.json)
    host = None
    if not args.no_host:
        progress('host path leg')
        mh = run_workload(args.config, args.scaling, rank, world, dev, 1, 1, 1, host_pass=True)
        host = mh['host']

    # ---- strong scaling of config 4: the 1024^3 volume in z-slabs over the ranks -------------
    strong = None
    if not args.no_strong and not (args.config == 4 and args.scaling == 'strong'):
        s = run_workload(4, 'strong', rank, world, dev, args.strong_steps, 1, args.streams)
        srf = roofline_of(CONFIGS[4], s)
        strong = {'value': round(s['inner_all'] * s['steps'] / s['dt'] / 1e9, 4), 'unit': 'Gvoxel/s',
                  'ms_per_step': round(s['dt'] / s['steps'] * 1e3, 3), 'ms_per_step_ranks': s['ms_ranks'],
                  'steps': s['steps'], 'n_gpus': world, 'scaling': 'strong',
                  'volume': list(s['full']), 'block_shape': list(CONFIGS[4]['block_shape']),
                  'halo': list(CONFIGS[4]['halo']), 'blocks_this_rank': s['nblocks'],
                  'inner_voxels_all_gpus': s['inner_all'], 'global_ids': s['n_ids'],
                  'pipeline_roofline_frac_per_gpu': round(srf['pipe'] / HBM_PEAK_GBS, 4),
                  'flood_ms_1stream_rank0': round(sum(s['stage_1'].get(p, 0.0) for p in STAGE_PARTS['flood']), 3),
                  'offset_scan': 'per step: all-gather of the per-block distinct-id counts (%s) + exclusive scan'
                                 % (backend or 'single process')}

    # ---- end to end: n5 gzip in -> WatershedWorkflow (GPU jobs) + relabel -> n5 out --------
    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e and not two_pass:
        progress('end-to-end workflow run')
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        try:
            e2e = end_to_end(args.config, dev, z_extent=args.e2e_z)
        except Exception as e:  # a side leg never takes the headline line down
            e2e = {'error': '%s: %s' % (type(e).__name__, e)}

    tcc = None
    if rank == 0 and world == 1 and not args.no_threshcc:
        progress('thresholded components block')
        torch.cuda.empty_cache()
        try:
            tcc = threshcc_leg(dev)
        except Exception as e:  # a side leg never takes the headline line down
            tcc = {'error': '%s: %s' % (type(e).__name__, e)}

    # ---- VI of the GPU output vs the oracle on the CPU baseline's first block ---------------
    vi = None
    if ref_block is not None and ref_block[1] is not None and m['kept'] is not None:
        from cluster_tools_amd.metrics import vi_scores, rand_scores
        gpu_out = m['kept']
        ref = ref_block[1]
        vs, vm = vi_scores(gpu_out, ref)
        are, _ = rand_scores(gpu_out, ref)
        vi = {'block_id': ref_block[0], 'vi_split': round(vs, 6), 'vi_merge': round(vm, 6),
              'vi': round(vs + vm, 6), 'adapted_rand_error': round(are, 8),
              'bit_exact': bool(np.array_equal(gpu_out, ref)),
              'bar': 'VI <= 0.01, ARand <= 1e-3 (BASELINE.json north_star)'}

    traffic = None
    pmc = os.path.join(HERE, 'profiles', 'pmc_traffic_c%d.json' % args.config)
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get(rf['dom'])

    if rank == 0:
        line = {
            'metric': 'Gvoxel/s DT-watershed (node, 1/2/4/8 GPU) + % HBM roofline; VI vs ref',
            'value': round(value, 4), 'unit': 'Gvoxel/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(rf['ms_per_step'], 3), 'higher_is_better': True,
            'scaling': args.scaling, 'vs_baseline': None, 'dtype': cfg.get('dtype', 'float32').replace('float', 'f'),
            'data': 'synthetic',
            'config': {'workload': cfg['workload'], 'volume': list(cfg['shape']), 'full_volume': list(m['full']),
                       'block_shape': list(cfg['block_shape']),
                       'halo': list(cfg['halo']), 'blocks_per_gpu': m['nblocks'], 'passes': m['npass'],
                       'inner_voxels_per_gpu': m['inner_vox'], 'outer_voxels_per_gpu': m['outer_vox'],
                       'streams_per_gpu': m['nstreams'],
                       'parallelism': 'z-slabs of the block grid, one process per GPU, %d GPU(s), %s scaling'
                                      % (world, args.scaling),
                       'inner_voxels_all_gpus': m['inner_all'],
                       'devices': len(devices), 'dist_backend': backend,
                       'pass2_order': ('dependency levels of the sequential loop (watershed.pass2_levels, as '
                                       'the workflow): %d launch groups' % (m['ngroups'] - 1)) if two_pass else None},
            'ms_per_step_ranks': m['ms_ranks'],
            'roofline': {'bound': 'hbm', 'kernel': '%s (%s)' % (rf['dom'], STAGE_KERNELS[rf['dom']]),
                         'ms_per_step': round(rf['dom_ms'], 3), 'achieved': round(rf['achieved'], 1),
                         'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': round(rf['achieved'] / HBM_PEAK_GBS, 4),
                         'traffic': traffic, 'alg_bytes': rf['dom_bytes'], 'alg_bytes_per_voxel': rf['b_unit'],
                         'voxels': rf['unit'],
                         'timing': 'HIP events on the library stream, one untimed step with all blocks on 1 stream',
                         'traffic_unit': 'HBM bytes per step of the stage (profiles/pmc_traffic_c%d.json)'
                                         % args.config},
            'pipeline_roofline': {'alg_bytes_per_inner_voxel': round(rf['alg_total'] / m['inner_vox'], 1),
                                  'achieved': round(rf['pipe'], 1), 'unit': 'GB/s',
                                  'frac': round(rf['pipe'] / HBM_PEAK_GBS, 4)},
            'strong_config4': strong,
            'config5': c5,
            'host_resident': host,
            'end_to_end': e2e,
            'thresholded_components': tcc,
            'vi_vs_oracle': vi,
            'stage_ms': {k: round(v, 3) for k, v in m['stage_ms'].items()},
            'stage_ms_1stream': {k: round(v, 3) for k, v in m['stage_1'].items()},
            'stage_gbs': rf['stage_gbs'],
            'global_ids': m['n_ids'],
            'cpu_baseline': cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def sharded_gather_devices(dev_index, dev):
    """The device index of every rank (to report how many distinct GPUs the ranks used)."""
    from cluster_tools_amd.watershed import sharded
    return sharded.all_gather_float(dev_index, device=dev)


if __name__ == '__main__':
    main()
