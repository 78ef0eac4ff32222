#!/bin/bash
# Round 6: is k_frontier bound by the texture-address path (scattered 64-lane loads)?  One PMC
# pass of TA / TCP counters on config 3 (single stream), per kernel, plus the counter list.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r06_ta
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1; echo "list rc=$?"
grep -oE "\b(TA_[A-Z_]*BUSY[A-Za-z_]*|TCP_TOTAL_CACHE_ACCESSES[A-Za-z_]*|TCP_PENDING_STALL_CYCLES[A-Za-z_]*|TA_FLAT_READ_WAVEFRONTS[A-Za-z_]*|TD_BUSY[A-Za-z_]*|TCP_TCC_READ_REQ[A-Za-z_]*)" $O/counters.txt | sort -u | head -20
timeout -s KILL 240 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE SQ_WAVES \
  --kernel-include-regex ctws --output-format csv -d $O/ta -o p -- \
  python3 -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline --no-host --no-e2e --no-strong --no-threshcc --no-config5 --streams 1 > $O/ta.log 2>&1
rc=$?; echo "pmc TA rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/ta.log; exit $rc; }
python3 - <<'PY'
import csv, glob, collections
per = collections.defaultdict(lambda: collections.defaultdict(float))
for path in glob.glob('gpurun_out/r06_ta/ta/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(path)):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('ctws::', '')[:40]
        per[k][r['Counter_Name']] += float(r['Counter_Value'])
rows = sorted(per.items(), key=lambda kv: -kv[1].get('GRBM_GUI_ACTIVE', 0))[:14]
with open('gpurun_out/r06_ta/ta_summary.txt', 'w') as f:
    for k, v in rows:
        g = max(v.get('GRBM_GUI_ACTIVE', 1), 1)
        line = '%-40s gui %9.3f M  ta_busy/gui/256 %.3f  flat_rd_waves %.3e  tcp_acc %.3e  tcc_rd %.3e' % (
            k, g / 1e6, v.get('TA_TA_BUSY_sum', 0) / g / 256, v.get('TA_FLAT_READ_WAVEFRONTS_sum', 0),
            v.get('TCP_TOTAL_CACHE_ACCESSES_sum', 0), v.get('TCP_TCC_READ_REQ_sum', 0))
        print(line); f.write(line + '\n')
PY
