#!/usr/bin/env python
"""Timeline of one end-to-end WatershedWorkflow run (bench.end_to_end's gzip leg): per task and
job, the first and last log-line times relative to the workflow start, to see where an
end-to-end run spends its time (process start, GPU init, chunk I/O, kernels)."""
import glob
import json
import os
import subprocess
import sys
import time
from datetime import datetime

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    import torch
    import bench
    from cluster_tools_amd.synthetic import boundary_map_torch
    from cluster_tools_amd.utils import volume_utils as vu
    from cluster_tools_amd.watershed.watershed import WatershedLocal
    cfg = bench.CONFIGS[3]
    z = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    jobs = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    in_job = (sys.argv[3] != '0') if len(sys.argv) > 3 else True   # relabel_in_job
    shape = (z,) + tuple(cfg['shape'][1:])
    import shutil
    import tempfile
    d = tempfile.mkdtemp(prefix='ctws_e2e_probe_')   # (data stays off gpurun_out)
    os.makedirs(os.path.join(d, 'configs'), exist_ok=True)
    x = boundary_map_torch(shape, seed=1, device=torch.device('cuda', 0), pitch=cfg['pitch']).cpu().numpy()
    inp = os.path.join(d, 'data.n5')
    with vu.file_reader(inp) as f:
        ds = f.create_dataset('boundaries', shape=shape, dtype=x.dtype,
                              chunks=tuple(b // 2 for b in cfg['block_shape']))
        ds.n_threads = 16
        ds[...] = x
    with open(os.path.join(d, 'configs', 'global.config'), 'w') as f:
        json.dump({'block_shape': list(cfg['block_shape']), 'shebang': '#! ' + sys.executable}, f)
    tc = WatershedLocal.default_task_config()
    tc.update(cfg['task'])
    tc['threads_per_job'] = 4
    with open(os.path.join(d, 'configs', 'watershed.config'), 'w') as f:
        json.dump(tc, f)
    code = ('import sys; sys.path.insert(0, %r)\n'
            'from cluster_tools_amd import luigi_compat as luigi\n'
            'from cluster_tools_amd.watershed import WatershedWorkflow\n'
            'wf = WatershedWorkflow(input_path=%r, input_key="boundaries", output_path=%r, output_key="ws", '
            'config_dir=%r, tmp_folder=%r, target="local", max_jobs=%d, relabel_in_job=%r)\n'
            'sys.exit(0 if luigi.build([wf], local_scheduler=True) else 1)\n'
            % (HERE, inp, os.path.join(d, 'ws.n5'), os.path.join(d, 'configs'), os.path.join(d, 'tmp'), jobs, in_job))
    del x
    print('volume %s, %d jobs, relabel_in_job %s' % (shape, jobs, in_job), flush=True)
    t0 = datetime.now()
    tt = time.perf_counter()
    rc = subprocess.call([sys.executable, '-c', code])
    print('workflow rc %d, %.2f s' % (rc, time.perf_counter() - tt))
    for log in sorted(glob.glob(os.path.join(d, 'tmp', 'logs', '*.log'))):
        lines = [l for l in open(log) if l[:4].isdigit()]
        if not lines:
            continue
        ts = [datetime.strptime(l.split(': ')[0], '%Y-%m-%d %H:%M:%S.%f') for l in lines]
        print('%-40s start %6.2f  end %6.2f  (%d lines)' % (os.path.basename(log), (ts[0] - t0).total_seconds(),
                                                             (ts[-1] - t0).total_seconds(), len(lines)))
        if log.endswith('_0.log'):
            for t, l in zip(ts, lines):
                print('      %6.2f %s' % ((t - t0).total_seconds(), l.split(': ', 1)[1].strip()[:90]))
    shutil.rmtree(d, ignore_errors=True)


if __name__ == '__main__':
    main()
