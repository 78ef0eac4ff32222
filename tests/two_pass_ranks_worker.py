"""Worker of tests/test_bench_two_pass_ranks.py: one rank of bench.run_workload on a small
two-pass volume (strong scaling: the volume in z-slabs over the ranks), the rank's slab of the
final labels saved as .npy.  Ranks share GPU 0 over gloo (the bench's one-GPU rehearsal mode)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402

TEST_CONFIG = 99  # (bench.py prints config ids with %d)

bench.CONFIGS[TEST_CONFIG] = dict(
    shape=(128, 128, 128), full_shape=(128, 128, 128), block_shape=(32, 64, 64), halo=(8, 16, 16), dtype='uint8',
    mask=True, two_pass=True, seed=5, task=dict(bench.D3, size_filter=25, halo=[8, 16, 16]),
    workload='test: 128^3 uint8 + ellipsoid mask, 32x64x64 blocks, halo [8,16,16], two-pass')


def main(out_dir):
    import torch
    import torch.distributed as dist
    world, rank, _ = bench.dist_env()
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    if world > 1:
        dist.init_process_group('gloo')
    m = bench.run_workload(TEST_CONFIG, 'strong', rank, world, dev, 1, 0, 1, keep_volume=True)
    np.save(os.path.join(out_dir, 'rank%d_of%d.npy' % (rank, world)), m['kept_volume'])
    with open(os.path.join(out_dir, 'rank%d_of%d.json' % (rank, world)), 'w') as f:
        json.dump({'z0': m['geo']['z0'], 'n_exchanges': m['n_exchanges'], 'ngroups': m['ngroups']}, f)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main(sys.argv[1])
