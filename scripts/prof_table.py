"""Per-kernel table from a rocprofv3 kernel-stats directory (default gpurun_out/prof) and, when
present, gpurun_out/pmc summaries.   python scripts/prof_table.py <steps> [prof_dir]"""
import csv, json, os, sys
calls_per_step = int(sys.argv[1]) if len(sys.argv) > 1 else 4
pdir = sys.argv[2] if len(sys.argv) > 2 else 'gpurun_out/prof'
stats = None
for root, _, files in os.walk(pdir):
    for f in files:
        if f.endswith('kernel_stats.csv'):
            stats = os.path.join(root, f)
rows = list(csv.DictReader(open(stats)))
p1 = json.load(open('gpurun_out/pmc/summary_pass1.json')) if os.path.exists('gpurun_out/pmc/summary_pass1.json') else {}
p2 = json.load(open('gpurun_out/pmc/summary_pass2.json')) if os.path.exists('gpurun_out/pmc/summary_pass2.json') else {}
print("%-28s %6s %8s %8s | %5s %5s %5s %7s %6s %7s" % ("kernel", "calls", "avg_us", "ms/step", "waitA", "waitI", "activ", "valu/wv", "lds/wv", "salu/wv"))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:40]:
    n = r['Name'].split('(')[0].replace('void ', '').replace('ctws::', '')
    if 'at::' in n:
        continue
    q = p1.get(n, {}); q2 = p2.get(n, {})
    wc = q.get('SQ_WAVE_CYCLES', 0) or 1; wv = q.get('SQ_WAVES', 0) or 1
    print("%-28s %6d %8.1f %8.3f | %5.2f %5.2f %5.2f %7.0f %6.0f %7.0f" % (
        n[:28], int(r['Calls']), float(r['AverageNs']) / 1e3, float(r['TotalDurationNs']) / 1e6 / calls_per_step,
        q.get('SQ_WAIT_ANY', 0) / wc, q.get('SQ_WAIT_INST_ANY', 0) / wc, q.get('SQ_ACTIVE_INST_ANY', 0) / wc,
        q.get('SQ_INSTS_VALU', 0) / wv, q.get('SQ_INSTS_LDS', 0) / wv, q2.get('SQ_INSTS_SALU', 0) / wv))
