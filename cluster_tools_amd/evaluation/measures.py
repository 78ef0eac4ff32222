#! /usr/bin/env python
"""GPU measures task: EvaluationWorkflow's overlaps + Measures in one job on the GPU.

The reference computes the seg x gt overlaps blockwise with nifty (NodeLabelWorkflow,
evaluation/evaluation_workflow.py:53-66), serializes them, and one Measures job
(evaluation/measures.py:132-161) merges them into a contingency table and writes
{'vi-split', 'vi-merge', 'adapted-rand-error', 'rand-index'} (validation_utils.py:60-76,
178-198) to output_path.  Here one job streams the two volumes block by block into a
contingency table in HBM (ctws_eval_*, k_eval.hip) and writes the same JSON.  Task surface:
GpuMeasures{Local,Slurm,LSF}, task_name 'gpu_measures'; config keys threads_per_job and
'label_capacity' / 'pair_capacity' (distinct ids / pairs the table is sized for).
"""
import json
import os
import sys
from concurrent import futures

from cluster_tools_amd import luigi_compat as luigi
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu
from cluster_tools_amd.utils.blocking import Blocking
from cluster_tools_amd.cluster_tasks import SlurmTask, LocalTask, LSFTask


class GpuMeasuresBase(luigi.Task):
    task_name = 'gpu_measures'
    src_file = os.path.abspath(__file__)
    allow_retry = False

    seg_path = luigi.Parameter()
    seg_key = luigi.Parameter()
    gt_path = luigi.Parameter()
    gt_key = luigi.Parameter()
    output_path = luigi.Parameter()
    ignore_label = luigi.BoolParameter(default=True)
    dependency = luigi.TaskParameter()

    def requires(self):
        return self.dependency

    @staticmethod
    def default_task_config():
        config = LocalTask.default_task_config()
        config.update({'label_capacity': 1 << 24, 'pair_capacity': 1 << 25})
        return config

    def run_impl(self):
        shebang, block_shape = self.global_config_values()[:2]
        self.init(shebang)
        config = self.get_task_config()
        config.update({'seg_path': self.seg_path, 'seg_key': self.seg_key, 'gt_path': self.gt_path,
                       'gt_key': self.gt_key, 'output_path': self.output_path,
                       'ignore_label': bool(self.ignore_label), 'block_shape': block_shape})
        self.run_jobs(1, None, config)


class GpuMeasuresLocal(GpuMeasuresBase, LocalTask):
    pass


class GpuMeasuresSlurm(GpuMeasuresBase, SlurmTask):
    pass


class GpuMeasuresLSF(GpuMeasuresBase, LSFTask):
    pass


def gpu_measures(job_id, config_path):
    from cluster_tools_amd import ctws
    fu.log("start processing job %i" % job_id)
    fu.log("reading config from %s" % config_path)
    with open(config_path) as f:
        config = json.load(f)
    device = int(os.environ.get('CTWS_DEVICE', os.environ.get('LOCAL_RANK', '0')))
    with vu.file_reader(config['seg_path'], 'r') as fs, vu.file_reader(config['gt_path'], 'r') as fg, \
            ctws.Handle(device) as h, futures.ThreadPoolExecutor(1) as io:
        ds_seg, ds_gt = fs[config['seg_key']], fg[config['gt_key']]
        assert tuple(ds_seg.shape) == tuple(ds_gt.shape)
        blocking = Blocking([0, 0, 0], list(ds_seg.shape), list(config['block_shape']))
        n_blocks = blocking.numberOfBlocks

        def read(bid):
            bb = vu.block_to_bb(blocking.getBlock(bid))
            return ds_seg[bb].astype('uint64'), ds_gt[bb].astype('uint64')

        h.eval_begin(config['label_capacity'], config['pair_capacity'])
        nxt = io.submit(read, 0) if n_blocks else None
        for bid in range(n_blocks):
            seg, gt = nxt.result()
            nxt = io.submit(read, bid + 1) if bid + 1 < n_blocks else None
            h.eval_add(seg, gt, ignore_gt_zero=config['ignore_label'])
        res = h.eval_end()
    results = {k: res[k] for k in ('vi-split', 'vi-merge', 'adapted-rand-error', 'rand-index')}
    with open(config['output_path'], 'w') as f:
        json.dump(results, f)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    gpu_measures(job_id, path)
