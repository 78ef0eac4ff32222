"""Recompute bench.py's roofline (the flood stage) from a rocprofv3 kernel trace.

    python scripts/roofline_from_trace.py <run_kernel_trace.csv> <bench line .json> <runs>

The trace must come from `bench.py --streams 1 --no-host --no-cpu-baseline` (one library
stream, no host-resident pass), `runs` = warmup + steps of that command.  Dispatches are
assigned to stages by scripts/stage_map.py (the rule pmc_traffic.py uses for the bytes): the
flood of a batch is every dispatch from its k_descent_tile up to the size filter's first kernel
(the regrow's frontier launches and check belong to the size filter).  Prints the summed
kernel time per step, the achieved GB/s of the stage's algorithmic bytes (12 B per outer voxel,
SURVEY.md §8(d)) and the bench line's own HIP-event figure beside it.
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from stage_map import classify, short as kshort  # noqa: E402


def main():
    trace, bench, runs = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = []
    import gzip
    with (gzip.open(trace, 'rt') if trace.endswith('.gz') else open(trace)) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    line = json.loads([l for l in open(bench).read().splitlines() if l.startswith('{')][-1])
    flood_ns, per_kernel, batches = 0, {}, 0
    rows = [r for r in rows if 'k_copy_to_host' not in r[2]]  # (host-path copies: not the stage)
    stage_ms = {}
    for (s, e, name), st in zip(rows, classify([r[2] for r in rows])):
        if st is None:
            continue  # library kernels of the stage only (no torch)
        stage_ms[st] = stage_ms.get(st, 0) + (e - s)
        if st != 'flood':
            continue
        short = kshort(name)
        if short.startswith('k_descent_tile'):
            batches += 1
        flood_ns += e - s
        per_kernel[short] = per_kernel.get(short, 0) + (e - s)
    ms = flood_ns / 1e6 / runs
    alg = line['roofline']['alg_bytes']
    achieved = alg / (ms * 1e-3) / 1e9
    out = {'trace': trace, 'runs': runs, 'batches_per_run': batches / runs,
           'flood_kernel_ms_per_step': round(ms, 3), 'alg_bytes': alg,
           'achieved_GBs': round(achieved, 1), 'frac': round(achieved / line['roofline']['peak'], 4),
           'bench_hip_event_ms': line['roofline']['ms_per_step'], 'bench_frac': line['roofline']['frac'],
           'agreement': round(ms / line['roofline']['ms_per_step'], 3),
           'per_kernel_ms_per_step': {k: round(v / 1e6 / runs, 3) for k, v in sorted(per_kernel.items())},
           'stage_ms_per_step': {k: round(v / 1e6 / runs, 3) for k, v in sorted(stage_ms.items())}}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
