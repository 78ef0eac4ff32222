"""HBM traffic of the BlockComponents kernels (k_threshcc.hip) from two rocprofv3 --pmc runs
(FETCH_SIZE, WRITE_SIZE) of `scripts/bench_threshcc.py --no-cpu --only blobs_128x512` (scripts/
gpu_pmc_threshcc.sh): bytes per dispatch of each kernel, averaged over the dispatches of the
128x512x512 block (read = 2 x FETCH_SIZE, the gfx950 correction of MI355X_MICROARCH.md; write =
WRITE_SIZE; KiB), and their sum per block call beside the 28 B per voxel algorithmic bytes."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = ('k_tc_minmax', 'k_tc_tile', 'k_tc_merge', 'k_tc_roots', 'k_bits_chunk_count', 'k_scan_chunks',
           'k_tc_wordoff', 'k_tc_label')


def main(d, voxels=128 * 512 * 512):
    acc = defaultdict(lambda: defaultdict(list))
    for cname in ('FETCH_SIZE', 'WRITE_SIZE'):
        mult = 2.0 if cname == 'FETCH_SIZE' else 1.0
        for path in glob.glob(os.path.join(d, cname, '**', '*counter_collection.csv'), recursive=True):
            with open(path) as f:
                for r in csv.DictReader(f):
                    if r['Counter_Name'] != cname:
                        continue
                    k = r['Kernel_Name'].split('(')[0].replace('ctws::', '')
                    if k in KERNELS:
                        acc[k][cname].append(float(r['Counter_Value']) * 1024.0 * mult)
    out = {'kernels': {}}
    total = 0.0
    for k in KERNELS:
        if k not in acc:
            continue
        rd = sum(acc[k]['FETCH_SIZE']) / max(1, len(acc[k]['FETCH_SIZE']))
        wr = sum(acc[k]['WRITE_SIZE']) / max(1, len(acc[k]['WRITE_SIZE']))
        out['kernels'][k] = {'read_bytes': round(rd), 'write_bytes': round(wr), 'dispatches': len(acc[k]['FETCH_SIZE'])}
        total += rd + wr
    out['total_bytes_per_call'] = round(total)
    out['bytes_per_voxel'] = round(total / voxels, 2)
    out['alg_bytes_per_voxel'] = 28
    out['note'] = ('one 128x512x512 smooth-blob block per call; read = 2 x FETCH_SIZE (gfx950 correction), '
                   'write = WRITE_SIZE')
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(sys.argv[1])
