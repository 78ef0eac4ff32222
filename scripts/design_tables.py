"""Markdown tables for DESIGN.md §3 from a final-run directory (scripts/gpu_r06_final_b.sh
outputs: prof_c{3,4,5}.json, roofline_recompute_c*.json, pmc_traffic_c{3,4}.json)."""
import json
import os
import sys

STAGES = ['prep_edt_x', 'edt_yz', 'smooth_seeds', 'hmap', 'seeds', 'flood', 'size_filter', 'crop_cc', 'output']
NAMES = {'prep_edt_x': 'normalize + EDT x', 'edt_yz': 'EDT y (, z)', 'smooth_seeds': 'seed-map Gaussian',
         'hmap': 'hmap + Gaussian', 'seeds': 'seeds', 'flood': '**flood**', 'size_filter': 'size filter + regrow',
         'crop_cc': 'crop CC', 'output': 'output'}


def last_json(path):
    return json.loads(open(path).read().strip().splitlines()[-1])


def main(d):
    print('| config | Gvoxel/s (1 stream) | ms / step | flood ms / step (trace) | flood frac | pipeline frac | frontier iterations / step |')
    print('|---|---|---|---|---|---|---|')
    for c in (3, 4, 5):
        p = os.path.join(d, 'prof_c%d.json' % c)
        r = os.path.join(d, 'roofline_recompute_c%d.json' % c)
        if not (os.path.exists(p) and os.path.exists(r)):
            continue
        b, rr = last_json(p), json.load(open(r))
        print('| %d | %.2f | %.1f | %.1f | %.4f | %.3f | %.1f |' % (
            c, b['value'], b['ms_per_step'], rr['flood_kernel_ms_per_step'], rr['frac'],
            b['pipeline_roofline']['frac'], b['stage_ms_1stream'].get('frontier_iters', 0)))
    for c in (3, 4):
        r = os.path.join(d, 'roofline_recompute_c%d.json' % c)
        t = os.path.join(d, 'pmc_traffic_c%d.json' % c)
        if not (os.path.exists(r) and os.path.exists(t)):
            continue
        rr, tt = json.load(open(r)), json.load(open(t))
        print()
        print('config %d: | stage | ms / step (trace) | HBM GB / step (PMC) | TB/s |' % c)
        print('|---|---|---|---|')
        tot_ms = tot_gb = 0.0
        for s in STAGES:
            ms = rr['stage_ms_per_step'].get(s, 0.0)
            gb = tt.get(s, 0.0) / 1e9
            tot_ms += ms
            tot_gb += gb
            print('| %s | %.2f | %.1f | %.2f |' % (NAMES[s], ms, gb, gb / ms if ms else 0.0))
        print('| total | %.1f | %.1f | %.2f |' % (tot_ms, tot_gb, tot_gb / tot_ms))


if __name__ == '__main__':
    main(sys.argv[1])
