"""HBM traffic per pipeline stage from two rocprofv3 --pmc runs (FETCH_SIZE, WRITE_SIZE) of
`bench.py --steps 1 --warmup 0 --streams 1` (scripts/gpu_pmc_traffic.sh).

Every ctws:: dispatch is assigned to its stage by the dispatch-order state machine of
stage_map.py (the same rule roofline_from_trace.py applies to kernel time, so the traffic and
the time of a stage cover the same dispatches; the size filter's regrow launches of k_frontier /
k_flood_verify count as size_filter).  gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE
reports half of the bytes of wide coalesced reads, so read bytes = 2 x FETCH_SIZE; WRITE_SIZE as
reported; both in KiB.  The correction is calibrated for 16-B-per-lane streams only; for the
8-B gathers of the flood see profiles/r04/pmc_gather_calibration.json (scripts/micro/
gather_bytes.hip).  Prints JSON: {stage: bytes per step}, 'total', 'kernels': {kernel:
{read_bytes, write_bytes, dispatches, stage}}; the stages sum to the total of all library
dispatches."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from stage_map import classify, short  # noqa: E402


def runs(d, cname):
    """{(file, run): [(dispatch id, kernel, value KiB)]} of one counter's CSVs."""
    out = defaultdict(list)
    for path in glob.glob(os.path.join(d, cname, '**', '*counter_collection.csv'), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r['Counter_Name'] != cname:
                    continue
                out[path].append((int(r['Dispatch_Id']), r['Kernel_Name'], float(r['Counter_Value'])))
    return out


def main(d, steps=1):
    per_k = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(int)
    stage_of_k = defaultdict(set)
    stages = defaultdict(float)
    for cname in ('FETCH_SIZE', 'WRITE_SIZE'):
        mult = 2.0 if cname == 'FETCH_SIZE' else 1.0
        for path, rows in runs(d, cname).items():
            rows.sort()
            st = classify([n for _, n, _ in rows])
            for (_, n, v), s in zip(rows, st):
                if s is None:
                    continue
                k = short(n)
                b = v * 1024.0 * mult
                per_k[k][cname] += b
                if cname == 'FETCH_SIZE':
                    disp[k] += 1
                stage_of_k[k].add(s)
                stages[s] += b
    out = {'kernels': {}}
    for k, v in sorted(per_k.items()):
        out['kernels'][k] = {'read_bytes': v.get('FETCH_SIZE', 0.0) / steps, 'write_bytes': v.get('WRITE_SIZE', 0.0) / steps,
                             'dispatches': disp[k] / steps, 'stage': sorted(stage_of_k[k])}
    for s, b in stages.items():
        out[s] = b / steps
    out['total'] = sum(stages.values()) / steps
    out['note'] = ('bytes per step; read = 2 x FETCH_SIZE (gfx950 wide-read correction), write = WRITE_SIZE; '
                   'stages by dispatch order (scripts/stage_map.py)')
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
