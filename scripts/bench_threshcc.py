"""Throughput of BlockComponents (ctws_threshold_components, k_threshcc.hip) on one MI355X.

Per workload (one block, synthetic): the device path (input and labels in HBM), the host path
(numpy in / out, PCIe included) and the CPU oracle (scipy.ndimage.label, one core) on the same
block; the device labels are checked against the oracle.  Algorithmic bytes per voxel of the
device path: minmax 4 + tile 4 (+1 mask) read + 4 P write + roots 4 + label 4 + 8 write = 28 B
(the face merge reads ~P on the tile shells on top).  One JSON line per workload on stdout.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

WORKLOADS = {
    'reftest_10x256x256_blobs': ((10, 256, 256), 'blobs', .5),
    'blobs_128x256x256': ((128, 256, 256), 'blobs', .5),
    'sparse_64x512x512': ((64, 512, 512), 'random', .92),
    'blobs_128x512x512': ((128, 512, 512), 'blobs', .5),
}


def make(shape, kind, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.random(shape, dtype=np.float32)
    if kind == 'blobs':
        from scipy.ndimage import gaussian_filter
        x = gaussian_filter(x, 1.2).astype(np.float32)
    return x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--only', default='')
    ap.add_argument('--no-cpu', action='store_true')
    args = ap.parse_args()
    import torch
    from cluster_tools_amd import ctws
    from oracle import threshcc as T
    h = ctws.Handle(0)
    dev = torch.device('cuda', 0)
    for name, (shape, kind, thr) in WORKLOADS.items():
        if args.only and args.only not in name:
            continue
        x = make(shape, kind)
        n_vox = x.size
        xd = torch.from_numpy(x).to(dev)
        out = torch.empty(shape, dtype=torch.int64, device=dev)
        for _ in range(2):
            h.threshold_components_device(xd, thr, 'greater', out=out)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            _, n = h.threshold_components_device(xd, thr, 'greater', out=out)
        torch.cuda.synchronize()
        t_dev = (time.perf_counter() - t0) / args.reps
        lab_dev = out.cpu().numpy().view(np.uint64)
        h.threshold_components(x, thr, 'greater')
        t0 = time.perf_counter()
        for _ in range(max(1, args.reps // 4)):
            lab_host, n_host = h.threshold_components(x, thr, 'greater')
        t_host = (time.perf_counter() - t0) / max(1, args.reps // 4)
        rec = {'workload': name, 'shape': list(shape), 'threshold': thr, 'n_labels': n,
               'device_ms': round(t_dev * 1e3, 3), 'device_gvox_s': round(n_vox / t_dev / 1e9, 3),
               'device_alg_gb_s': round(28 * n_vox / t_dev / 1e9, 1),
               'host_ms': round(t_host * 1e3, 3), 'host_gvox_s': round(n_vox / t_host / 1e9, 3)}
        if not args.no_cpu:
            t0 = time.perf_counter()
            ref, rn = T.block_components(x, thr, 'greater')
            t_cpu = time.perf_counter() - t0
            rec.update({'cpu_oracle_ms': round(t_cpu * 1e3, 1), 'cpu_gvox_s': round(n_vox / t_cpu / 1e9, 4),
                        'cpu_cores': 1, 'parity': bool(rn == n and (ref == lab_dev).all() and (ref == lab_host).all())})
        print(json.dumps(rec), flush=True)
    h.close()


if __name__ == '__main__':
    main()
