"""Per-workload kernel times of BlockComponents from a rocprofv3 rocpd database
(scripts/gpu_threshcc_bench.sh): the dispatches of k_tc_* grouped by the workload they belong
to (consecutive calls; a new workload starts where k_tc_tile's grid changes)."""
import collections
import json
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute("select s.display_name, d.start, d.end, d.grid_size_x from rocpd_kernel_dispatch d "
                     "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
    groups, cur, grid = [], None, None
    for name, t0, t1, gx in rows:
        short = name.split('(')[0].replace('ctws::', '')
        if not short.startswith(('k_tc_', 'k_bits_chunk_count', 'k_scan_chunks')):
            continue
        if short == 'k_tc_tile' and gx != grid:
            grid = gx
            cur = collections.defaultdict(list)
            groups.append((gx, cur))
        if cur is not None:
            cur[short].append((t1 - t0) / 1e3)
    res = []
    for gx, g in groups:
        calls = len(g['k_tc_tile'])
        per = {k: round(sum(v) / calls, 2) for k, v in g.items()}   # us per block call
        res.append({'tile_grid_threads': gx, 'calls': calls, 'us_per_call': per,
                    'total_us_per_call': round(sum(per.values()), 1)})
    json.dump(res, open(out, 'w'), indent=1)
    for r in res:
        print(json.dumps(r))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
