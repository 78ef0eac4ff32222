#! /usr/bin/env python
"""FindUniques: per-job unique labels of the watershed output
(cluster_tools/relabel/find_uniques.py:20-159).  numpy implementation; the GPU version of the
relabel stage is the next row of SURVEY.md §8(f)."""
import json
import os
import sys

import numpy as np

from cluster_tools_amd import luigi_compat as luigi
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu
from cluster_tools_amd.utils.blocking import Blocking
from cluster_tools_amd.cluster_tasks import SlurmTask, LocalTask, LSFTask


class FindUniquesBase(luigi.Task):
    task_name = 'find_uniques'
    src_file = os.path.abspath(__file__)

    input_path = luigi.Parameter()
    input_key = luigi.Parameter()
    dependency = luigi.TaskParameter()
    return_counts = luigi.BoolParameter(default=False)

    def requires(self):
        return self.dependency

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        shape = vu.get_shape(self.input_path, self.input_key)
        if self.n_retries == 0:
            block_list = vu.blocks_in_volume(shape, block_shape, roi_begin, roi_end)
        else:
            block_list = self.block_list
            self.clean_up_for_retry(block_list)
        n_jobs = min(len(block_list), self.max_jobs)
        config = {"input_path": self.input_path, "input_key": self.input_key, "block_shape": block_shape,
                  "tmp_folder": self.tmp_folder, "return_counts": self.return_counts}
        self._write_log('scheduling %i blocks to be processed' % len(block_list))
        self.prepare_jobs(n_jobs, block_list, config)
        self.submit_jobs(n_jobs)
        self.wait_for_jobs()
        self.check_jobs(n_jobs)


class FindUniquesLocal(FindUniquesBase, LocalTask):
    pass


class FindUniquesSlurm(FindUniquesBase, SlurmTask):
    pass


class FindUniquesLSF(FindUniquesBase, LSFTask):
    pass


def uniques_in_block(block_id, blocking, ds, return_counts):
    fu.log("start processing block %i" % block_id)
    labels = ds[vu.block_to_bb(blocking.getBlock(block_id))]
    if labels.sum() == 0:
        if return_counts:
            return np.array([0], dtype=labels.dtype), np.array([labels.size], dtype='int64')
        return np.array([0], dtype=labels.dtype)
    res = np.unique(labels, return_counts=return_counts)
    fu.log_block_success(block_id)
    return res


def find_uniques(job_id, config_path):
    fu.log("start processing job %i" % job_id)
    fu.log("reading config from %s" % config_path)
    with open(config_path) as f:
        config = json.load(f)
    return_counts = config['return_counts']
    with vu.file_reader(config['input_path'], 'r') as f:
        ds = f[config['input_key']]
        blocking = Blocking([0, 0, 0], list(ds.shape), list(config['block_shape']))
        uniques = [uniques_in_block(b, blocking, ds, return_counts) for b in config['block_list']]
    tmp = config['tmp_folder']
    if return_counts:
        unique_values = np.unique(np.concatenate([u[0] for u in uniques]))
        counts = np.zeros(int(unique_values[-1] + 1), dtype='uint64')
        for ub, cb in uniques:
            counts[ub] += cb.astype('uint64')
        counts = counts[counts != 0]
        np.save(os.path.join(tmp, 'counts_job_%i.npy' % job_id), counts)
    else:
        unique_values = np.unique(np.concatenate(uniques))
    np.save(os.path.join(tmp, 'find_uniques_job_%i.npy' % job_id), unique_values)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    find_uniques(job_id, path)
