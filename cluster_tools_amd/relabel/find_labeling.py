#! /usr/bin/env python
"""FindLabeling: consecutive new ids for the global uniques, as an (N, 2) uint64 assignment
table (cluster_tools/relabel/find_labeling.py:20-126): 0 stays 0 if present, else ids start
at 1."""
import json
import os
import sys

import numpy as np

from cluster_tools_amd import luigi_compat as luigi
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu
from cluster_tools_amd.cluster_tasks import SlurmTask, LocalTask, LSFTask


class FindLabelingBase(luigi.Task):
    task_name = 'find_labeling'
    src_file = os.path.abspath(__file__)
    allow_retry = False

    input_path = luigi.Parameter()
    input_key = luigi.Parameter()
    assignment_path = luigi.Parameter()
    assignment_key = luigi.Parameter()
    dependency = luigi.TaskParameter()

    def requires(self):
        return self.dependency

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        shape = vu.get_shape(self.input_path, self.input_key)
        block_list = vu.blocks_in_volume(shape, block_shape, roi_begin, roi_end)
        n_jobs = min(len(block_list), self.max_jobs)
        config = self.get_task_config()
        config.update({'shape': list(shape), 'assignment_path': self.assignment_path,
                       'assignment_key': self.assignment_key, 'tmp_folder': self.tmp_folder, 'n_jobs': n_jobs})
        self.prepare_jobs(1, None, config)
        self.submit_jobs(1)
        self.wait_for_jobs()
        self.check_jobs(1)


class FindLabelingLocal(FindLabelingBase, LocalTask):
    pass


class FindLabelingSlurm(FindLabelingBase, SlurmTask):
    pass


class FindLabelingLSF(FindLabelingBase, LSFTask):
    pass


def find_labeling(job_id, config_path):
    fu.log("start processing job %i" % job_id)
    fu.log("reading config from %s" % config_path)
    with open(config_path) as f:
        config = json.load(f)
    tmp = config['tmp_folder']
    fu.log("read uniques")
    uniques = np.concatenate([np.load(os.path.join(tmp, 'find_uniques_job_%i.npy' % j))
                              for j in range(config['n_jobs'])])
    fu.log("compute uniques")
    uniques = np.unique(uniques)
    start, stop = (0, len(uniques)) if uniques[0] == 0 else (1, len(uniques) + 1)
    fu.log("relabel to new max-id %i" % stop)
    new_ids = np.arange(start, stop, dtype='uint64')
    assignments = np.concatenate([uniques[:, None].astype('uint64'), new_ids[:, None]], axis=1)
    fu.log("saving results to %s/%s" % (config['assignment_path'], config['assignment_key']))
    with vu.file_reader(config['assignment_path']) as f:
        chunks = (min(int(1e6), len(assignments)), 2)
        if config['assignment_key'] in f:
            import shutil
            shutil.rmtree(os.path.join(config['assignment_path'], config['assignment_key']))
        ds = f.create_dataset(config['assignment_key'], shape=assignments.shape, dtype='uint64',
                              compression='gzip', chunks=chunks)
        ds.n_threads = config.get('threads_per_job', 1)
        ds[:] = assignments
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    find_labeling(job_id, path)
