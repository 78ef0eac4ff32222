#! /usr/bin/env python
"""MergeOffsets: the per-block label offsets of BlockComponents as one exclusive scan
(cluster_tools/thresholded_components/merge_offsets.py:22-138; task surface unchanged).
Writes {'offsets', 'empty_blocks', 'n_labels'} to save_path."""
import json
import os
import sys

import numpy as np

from cluster_tools_amd import luigi_compat as luigi
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu
from cluster_tools_amd.cluster_tasks import SlurmTask, LocalTask, LSFTask


class MergeOffsetsBase(luigi.Task):
    task_name = 'merge_offsets'
    src_file = os.path.abspath(__file__)
    allow_retry = False

    shape = luigi.ListParameter()
    save_path = luigi.Parameter()
    save_prefix = luigi.Parameter(default='connected_components_offsets')
    dependency = luigi.TaskParameter()

    def requires(self):
        return self.dependency

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        block_list = vu.blocks_in_volume(self.shape, block_shape, roi_begin, roi_end)
        n_jobs = min(len(block_list), self.max_jobs)
        config = self.get_task_config()
        config.update({'tmp_folder': self.tmp_folder, 'n_jobs': n_jobs, 'save_path': self.save_path,
                       'n_blocks': len(block_list), 'save_prefix': self.save_prefix})
        self.run_jobs(1, None, config)


class MergeOffsetsLocal(MergeOffsetsBase, LocalTask):
    pass


class MergeOffsetsSlurm(MergeOffsetsBase, SlurmTask):
    pass


class MergeOffsetsLSF(MergeOffsetsBase, LSFTask):
    pass


def scan_block_counts(counts):
    """{block_id: count} -> (offsets, empty_blocks, n_labels), everything in increasing block id
    order: offsets = the exclusive prefix sum of the counts (a block's count is its `max + 1`,
    0 when empty), empty_blocks = the positions whose count is 0, n_labels = the total + 1, which
    is the reference's `last offset + last count + 1` (merge_offsets.py:111-122)."""
    ids = sorted(int(b) for b in counts)
    c = np.array([int(counts[b]) for b in ids], dtype=np.uint64)
    offs = np.zeros(len(c), dtype=np.uint64)
    if len(c) > 1:
        np.cumsum(c[:-1], out=offs[1:])
    return [int(o) for o in offs], np.flatnonzero(c == 0).tolist(), int(c.sum()) + 1


def merge_offsets(job_id, config_path):
    """Job entry (merge_offsets.py:83-131): the BlockComponents jobs' count files -> one scan."""
    fu.log("start processing job %i" % job_id)
    fu.log("reading config from %s" % config_path)
    with open(config_path) as f:
        config = json.load(f)
    counts = {}
    for j in range(config['n_jobs']):
        path = os.path.join(config['tmp_folder'], '%s_%i.json' % (config['save_prefix'], j))
        with open(path) as f:
            counts.update({int(b): int(v) for b, v in json.load(f).items()})
        os.remove(path)
    n_blocks = config['n_blocks']
    assert len(counts) == n_blocks, (len(counts), n_blocks)
    fu.log("merging offsets for %i blocks" % n_blocks)
    offsets, empty_blocks, n_labels = scan_block_counts(counts)
    fu.log("number of empty blocks: %i / %i" % (len(empty_blocks), n_blocks))
    fu.log("total number of labels: %i" % n_labels)
    fu.log("dumping offsets to %s" % config['save_path'])
    with open(config['save_path'], 'w') as f:
        json.dump({'offsets': offsets, 'empty_blocks': empty_blocks, 'n_labels': n_labels}, f)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    merge_offsets(job_id, path)
