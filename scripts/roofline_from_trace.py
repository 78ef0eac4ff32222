"""Recompute bench.py's roofline (the flood stage) from a rocprofv3 kernel trace.

    python scripts/roofline_from_trace.py <run_kernel_trace.csv> <bench line .json> <runs>

The trace must come from `bench.py --streams 1 --no-host --no-cpu-baseline` (one library
stream, no host-resident pass), `runs` = warmup + steps of that command.  The flood stage of a
batch is every dispatch from its k_descent_tile up to and including the first k_flood_verify
after it (the second verify of a batch belongs to the size-filter regrow).  Prints the summed
kernel time per step, the achieved GB/s of the stage's algorithmic bytes (12 B per outer voxel,
SURVEY.md §8(d)) and the bench line's own HIP-event figure beside it.
"""
import csv
import json
import sys


def main():
    trace, bench, runs = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = []
    with open(trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    line = json.loads([l for l in open(bench).read().splitlines() if l.startswith('{')][-1])
    flood_ns, per_kernel, in_flood, batches = 0, {}, False, 0
    for s, e, name in rows:
        if 'ctws::' not in name or 'k_copy_to_host' in name:
            continue  # library kernels of the stage only (no torch, no host-path copies)
        short = name.split('(')[0].replace('void ', '').replace('ctws::', '')
        if short.startswith('k_descent_tile'):
            in_flood = True
            batches += 1
        if in_flood:
            flood_ns += e - s
            per_kernel[short] = per_kernel.get(short, 0) + (e - s)
            if short.startswith('k_flood_verify'):
                in_flood = False
    ms = flood_ns / 1e6 / runs
    alg = line['roofline']['alg_bytes']
    achieved = alg / (ms * 1e-3) / 1e9
    out = {'trace': trace, 'runs': runs, 'batches_per_run': batches / runs,
           'flood_kernel_ms_per_step': round(ms, 3), 'alg_bytes': alg,
           'achieved_GBs': round(achieved, 1), 'frac': round(achieved / line['roofline']['peak'], 4),
           'bench_hip_event_ms': line['roofline']['ms_per_step'], 'bench_frac': line['roofline']['frac'],
           'agreement': round(ms / line['roofline']['ms_per_step'], 3),
           'per_kernel_ms_per_step': {k: round(v / 1e6 / runs, 3) for k, v in sorted(per_kernel.items())}}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
