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


def merge_offsets(job_id, config_path):
    """Job entry (merge_offsets.py:83-131): block-id order, exclusive cumulative sum of the
    per-block `max + 1`; n_labels = last offset + last count + 1."""
    fu.log("start processing job %i" % job_id)
    fu.log("reading config from %s" % config_path)
    with open(config_path) as f:
        config = json.load(f)
    offsets = {}
    for block_job_id in range(config['n_jobs']):
        path = os.path.join(config['tmp_folder'], '%s_%i.json' % (config['save_prefix'], block_job_id))
        with open(path) as f:
            offsets.update(json.load(f))
        os.remove(path)
    blocks = [int(b) for b in offsets.keys()]
    offset_list = list(offsets.values())
    n_blocks = config['n_blocks']
    assert len(blocks) == len(offset_list) == n_blocks
    fu.log("merging offsets for %i blocks" % n_blocks)
    key_sort = np.argsort(blocks)
    offset_list = np.array([offset_list[k] for k in key_sort], dtype='uint64')
    last_offset = offset_list[-1]
    empty_blocks = np.where(offset_list == 0)[0].tolist()
    offset_list = np.roll(offset_list, 1)
    offset_list[0] = 0
    offset_list = np.cumsum(offset_list).tolist()
    n_labels = int(offset_list[-1] + last_offset + 1)
    fu.log("number of empty blocks: %i / %i" % (len(empty_blocks), n_blocks))
    fu.log("total number of labels: %i" % n_labels)
    fu.log("dumping offsets to %s" % config['save_path'])
    with open(config['save_path'], 'w') as f:
        json.dump({'offsets': offset_list, 'empty_blocks': empty_blocks, 'n_labels': n_labels}, f)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    merge_offsets(job_id, path)
