"""End-to-end ThresholdedComponentsWorkflow on n5 (gzip) on one MI355X: a synthetic blob volume
is written, then the workflow runs -- with --merge-in-job 1 (the default) as one task whose jobs
merge among themselves (merge_in_job.py), with 0 as the five-task chain, BlockComponents timed
as its own luigi build and the rest (MergeOffsets, BlockFaces, MergeAssignments, Write) as a
second one; the result is checked against the CPU oracle on the whole volume.  One JSON line.
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--shape', default='128,1024,1024')
    ap.add_argument('--block', default='64,256,256')
    ap.add_argument('--max-jobs', type=int, default=4)
    ap.add_argument('--no-check', action='store_true')
    ap.add_argument('--merge-in-job', type=int, default=1)
    ap.add_argument('--keep-logs', default='', help='copy the jobs\' logs to this directory')
    args = ap.parse_args()
    shape = tuple(int(s) for s in args.shape.split(','))
    bs = [int(s) for s in args.block.split(',')]
    import torch
    import torch.nn.functional as F
    from cluster_tools_amd import luigi_compat as luigi
    from cluster_tools_amd.cluster_tasks import BaseClusterTask
    from cluster_tools_amd.utils import volume_utils as vu
    from cluster_tools_amd.utils.blocking import Blocking
    from cluster_tools_amd.thresholded_components import ThresholdedComponentsWorkflow
    from cluster_tools_amd.thresholded_components.block_components import BlockComponentsLocal
    g = torch.Generator(device='cuda:0').manual_seed(0)
    x = torch.rand((1, 1) + shape, generator=g, device='cuda:0')
    for _ in range(2):
        x = F.avg_pool3d(x, 5, stride=1, padding=2, count_include_pad=False)
    x = x[0, 0].cpu().numpy()
    torch.cuda.empty_cache()
    tmp = tempfile.mkdtemp(prefix='e2e_tc_', dir=os.environ.get('TMPDIR', '/tmp'))
    try:
        path = os.path.join(tmp, 'data.n5')
        with vu.file_reader(path) as f:
            f.create_dataset('x', data=x, chunks=tuple(b // 2 for b in bs), compression='gzip')
        cfg = os.path.join(tmp, 'configs')
        os.makedirs(cfg)
        gc = BaseClusterTask.default_global_config()
        gc.update({'shebang': '#! ' + sys.executable, 'block_shape': bs})
        with open(os.path.join(cfg, 'global.config'), 'w') as f:
            json.dump(gc, f)
        common = dict(tmp_folder=os.path.join(tmp, 'tmp'), config_dir=cfg, max_jobs=args.max_jobs)
        from cluster_tools_amd.utils.task_utils import DummyTask
        t0 = time.perf_counter()
        import datetime
        started_at = str(datetime.datetime.now())
        if args.merge_in_job:
            ok1 = True
            t1 = t0
        else:
            ok1 = luigi.build([BlockComponentsLocal(input_path=path, input_key='x', output_path=path,
                                                    output_key='cc', threshold=.5, dependency=DummyTask(),
                                                    **common)], local_scheduler=True)
            t1 = time.perf_counter()
        ok2 = luigi.build([ThresholdedComponentsWorkflow(input_path=path, input_key='x', output_path=path,
                                                         output_key='cc', assignment_key='ass', threshold=.5,
                                                         target='local', merge_in_job=bool(args.merge_in_job),
                                                         **common)], local_scheduler=True)
        t2 = time.perf_counter()
        n = int(np.prod(shape))
        rec = {'workload': 'ThresholdedComponentsWorkflow, %s float32 blobs (n5 gzip), blocks %s, %d jobs'
                           % ('x'.join(map(str, shape)), 'x'.join(map(str, bs)), args.max_jobs),
               'merge_in_job': bool(args.merge_in_job), 'ok': bool(ok1 and ok2),
               'started_at': started_at, 'total_s': round(t2 - t0, 2), 'gvoxel_s': round(n / (t2 - t0) / 1e9, 4)}
        if not args.merge_in_job:
            rec.update(block_components_s=round(t1 - t0, 2), rest_s=round(t2 - t1, 2),
                       block_components_gvoxel_s=round(n / (t1 - t0) / 1e9, 4))
        if ok1 and ok2 and not args.no_check:
            from oracle import threshcc as T
            t3 = time.perf_counter()
            ref, ref_ass, _ = T.thresholded_components(x, Blocking([0, 0, 0], list(shape), bs), .5, 'greater',
                                                       faces_jobs=args.max_jobs)
            rec['cpu_oracle_s'] = round(time.perf_counter() - t3, 2)
            with vu.file_reader(path, 'r') as f:
                rec['bit_exact'] = bool(np.array_equal(f['cc'][:], ref) and np.array_equal(f['ass'][:], ref_ass))
        print(json.dumps(rec), flush=True)
        if args.keep_logs:
            os.makedirs(args.keep_logs, exist_ok=True)
            for root, _, files in os.walk(os.path.join(tmp, 'tmp')):
                for fn in files:
                    if fn.endswith('.log'):
                        shutil.copy(os.path.join(root, fn), os.path.join(args.keep_logs, fn))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == '__main__':
    main()
