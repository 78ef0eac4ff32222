#!/usr/bin/env python
"""Tie-order experiment (CPU only, the oracle): how far each deterministic tie
order of the flood is from vigra's binary-heap order on the tie-dominated inputs.

vigra's watershedsNew pops a std::priority_queue keyed by priority alone, so equal priorities
(plateaus of the hmap, a 256-level uint8 input) leave the order to heap positions
(oracle/ctws_oracle.cpp:watersheds_new).  The GPU's flood computes the unique fixpoint of one
total order (k_flood.hip: C, then the hop distance d inside an equal-C plateau, then the label);
oracle watersheds_model restates it.  Orders compared (oracle g_tie_order):
  1 (C, d, label)  -- the GPU's (d saturating at 4095)
  2 (C, label)     -- no hop distance
  3 (C, d, -label)
  4 (C, d, push count): FIFO inside an equal-(C, d) front
  5 (C, push count):    FIFO on a plateau
  6 (C, min(d, 1), label): the hop distance reduced to "entered at its own height or not"
  7 (C, label, d): the label before the hop distance.  The key still strictly
    increases along parent edges, so the fixpoint is unique, and on these inputs it is as close
    to the heap as order 2.  Built on the GPU in round 5 it did not converge: the relaxation's
    keys are not monotone (a voxel's label can rise when its argmin's C drops), a label that has
    lost its source survives as a phantom whose d counts up until the 12-bit field saturates
    (frontier iterations that never empty; the fixpoint check fails) -- not adopted
Orders 2 and 6 are closest to the heap on the tie-dominated inputs, but (C, d) no longer strictly
increases along parent edges: the fixpoint is not unique (a cycle of equal-key plateau voxels
can keep a stale label) and the GPU's relaxation reached another one (round 4) -- not adopted.
Only orders of the form (C, d?, label-ish) are fixpoints a parallel relaxation can reach; 4 and 5
are sequential references for how close an insertion-ordered queue gets.
Output: VI(order, heap) per case, JSON on stdout."""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, 'tests'))

from oracle import oracle as O  # noqa: E402
from cluster_tools_amd.metrics import vi_scores  # noqa: E402


def main():
    O.build()
    L = O.lib()
    import cases as ws_cases
    import test_from_seeds_gpu as fs
    ws = ws_cases.make_cases()
    todo = [('ws', n) for n in ('3d_plateaus', '2d_sparse_fg', '3d_sparse_fg', '3d', '2d') if n in ws]
    todo += [('fs', n) for n in ('uint8', 'raw_plateaus', '4d_max', 'points')]
    out = {}
    for kind, name in todo:
        if kind == 'ws':
            config, block = ws[name]
            run = lambda: O.ws_blocks(config, ws_cases.BLOCK_SHAPE, [dict(block, block_id=3)])[0]['output']
        else:
            config, block = fs.CASES[name]
            run = lambda: O.ws_from_seeds(config, [block])[0]['output']
        heap = run()
        ign = [0] if block.get('mask') is not None else None
        row = {}
        for order in (1, 2, 3, 4, 5, 6, 7):
            L.orc_set_tie_order(order)
            with O.flood_model():
                m = run()
            row[order] = round(float(sum(vi_scores(m, heap, ign))), 4)
        L.orc_set_tie_order(1)
        out['%s:%s' % (kind, name)] = row
        print(name, row, file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
