#!/usr/bin/env python
"""Debug one WatershedWorkflow case of tests/test_workflow_gpu.py: run it, and on failure print
the failed jobs' logs; compare the watershed jobs' cached block uniques with the volume."""
import glob
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, 'tests'))


def main():
    import pathlib
    import test_workflow_gpu as T
    from cluster_tools_amd import luigi_compat as luigi
    from cluster_tools_amd.utils import volume_utils as vu
    from cluster_tools_amd.utils.blocking import Blocking
    from cluster_tools_amd.watershed import WatershedWorkflow
    from cluster_tools_amd.watershed.watershed import block_uniques_file
    name = sys.argv[1] if len(sys.argv) > 1 else 'ws_3d'
    with_mask = (sys.argv[2] == '1') if len(sys.argv) > 2 else True
    tmp = pathlib.Path(tempfile.mkdtemp())
    cfg_dir, inp, x, c = T._setup(tmp, name, with_mask)
    out = str(tmp / 'ws.n5')
    mask_kw = dict(mask_path=inp, mask_key='mask') if with_mask else {}
    wf = WatershedWorkflow(input_path=inp, input_key='boundaries', output_path=out, output_key='ws',
                           config_dir=cfg_dir, tmp_folder=str(tmp / 'tmp'), target='local', max_jobs=2, **mask_kw)
    ok = luigi.build([wf], local_scheduler=True)
    print('workflow ok:', ok)
    for p in sorted(glob.glob(str(tmp / 'tmp' / 'error_logs' / '*.err')) + glob.glob(str(tmp / 'tmp' / 'logs' / 'write*.log'))):
        txt = open(p).read()
        if txt.strip():
            print('====', p)
            print(txt[-3000:])
    blocking = Blocking([0, 0, 0], list(T.SHAPE), T.BLOCK_SHAPE)
    with vu.file_reader(out, 'r') as f:
        vol = f['ws'][:]
    folder = str(tmp / 'tmp' / 'watershed_block_uniques')
    bad = 0
    for bid in range(blocking.numberOfBlocks):
        path = block_uniques_file(folder, bid)
        if os.path.exists(path):
            u = np.load(path)
            v = np.unique(vol[vu.block_to_bb(blocking.getBlock(bid))])
            if not ok and not np.array_equal(u, v):
                bad += 1
                print('block', bid, 'cache', len(u), u[:5], 'volume', len(v), v[:5])
    print('blocks with cache != volume (meaningful only when the relabel did not run):', bad)


if __name__ == '__main__':
    main()
