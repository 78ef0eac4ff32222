"""Summarize rocprofv3 --pmc CSVs per kernel (ctws kernels only) and delete the raw files."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]
out = {}
for path in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
    agg = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r['Kernel_Name']
            if 'ctws' not in name:
                continue
            short = name.split('(')[0].replace('void ', '').replace('ctws::', '')
            agg[short][r['Counter_Name']] += float(r['Counter_Value'])
            calls[short].add(r['Dispatch_Id'])
    for k, v in agg.items():
        e = out.setdefault(k, {'dispatches': 0})
        e['dispatches'] = max(e['dispatches'], len(calls[k]))
        e.update(v)
for path in glob.glob(os.path.join(d, '**', '*.csv'), recursive=True):
    os.remove(path)
json.dump(out, open(os.path.join(d, 'pmc_summary.json'), 'w'), indent=1, sort_keys=True)
print(json.dumps(out.get('k_flood_packed<3>', {}), indent=1))
