"""FETCH_SIZE / WRITE_SIZE of scripts/micro/gather_bytes.hip's kernels against the bytes they
move (its first stdout line), per dispatch in launch order: flush, stream16, flush, stream8,
flush, seg512, line8.  Prints JSON with the ratio FETCH_SIZE bytes / algorithmic bytes (a ratio
of 0.5 is the gfx950 half-count of wide reads, MI355X_MICROARCH.md)."""
import csv
import glob
import json
import os
import sys


def main(d, known_path):
    known = json.loads(open(known_path).read().strip().splitlines()[0])
    rows = []
    for path in glob.glob(os.path.join(d, 'FETCH_SIZE', '**', '*counter_collection.csv'), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r['Counter_Name'] == 'FETCH_SIZE':
                    rows.append((int(r['Dispatch_Id']), r['Kernel_Name'].split('(')[0], float(r['Counter_Value']) * 1024))
    rows.sort()
    names = ['flush', 'stream16', 'flush', 'stream8', 'flush', 'seg512', 'line8']
    alg = {'flush': known['flush_bytes'], 'stream16': known['stream16_bytes'], 'stream8': known['stream8_bytes'],
           'seg512': known['seg512_bytes'] + known['permutation_bytes_seg512'],
           'line8': known['line8_lines'] * 128 + known['permutation_bytes_line8']}
    out = {'kernels': []}
    for (i, kname, fetch), lab in zip(rows, names):
        out['kernels'].append({'kernel': lab, 'fetch_size_bytes': fetch, 'bytes_moved': alg[lab],
                               'ratio_fetch_to_bytes': round(fetch / alg[lab], 3)})
    out['note'] = ('bytes_moved: the buffer bytes each kernel reads once (line8: one whole 128-B line per 8-B '
                   'gather, lines in random order, every line of 2 GiB once; + the index permutation it '
                   'streams); ratio 0.5 = FETCH_SIZE counts half the bytes, the x2 correction applies')
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
