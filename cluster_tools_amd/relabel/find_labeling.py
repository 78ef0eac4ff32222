#! /usr/bin/env python
"""FindLabeling: consecutive new ids for the global uniques, as an (N, 2) uint64 assignment
table (cluster_tools/relabel/find_labeling.py:20-126; task surface unchanged), merged on the
GPU: 0 stays 0 if present, else ids start at 1."""
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
        # one job merges the find_uniques results of the n_jobs jobs of the previous task
        cfg = dict(self.get_task_config(), shape=list(shape), assignment_path=self.assignment_path,
                   assignment_key=self.assignment_key, tmp_folder=self.tmp_folder,
                   n_jobs=min(len(block_list), self.max_jobs))
        self.run_jobs(1, None, cfg)


class FindLabelingLocal(FindLabelingBase, LocalTask):
    pass


class FindLabelingSlurm(FindLabelingBase, SlurmTask):
    pass


class FindLabelingLSF(FindLabelingBase, LSFTask):
    pass


def find_labeling(job_id, config_path):
    """Job entry (find_labeling.py:84-126): the global sorted uniques and their new ids.

    The jobs' unique arrays are merged by a GPU unique (ctws_unique_u64); new ids are
    consecutive in the order of the old ones, starting at 0 when 0 is present (it keeps id 0),
    else at 1.  The (N, 2) uint64 table [old, new] is written to assignment_path/key.
    """
    from cluster_tools_amd import ctws
    fu.log("start processing job %i" % job_id)
    fu.log("reading config from %s" % config_path)
    with open(config_path) as f:
        config = json.load(f)
    tmp = config['tmp_folder']
    fu.log("read uniques")
    parts = [np.load(os.path.join(tmp, 'find_uniques_job_%i.npy' % j)) for j in range(config['n_jobs'])]
    fu.log("compute uniques")
    with ctws.Handle(int(os.environ.get('CTWS_DEVICE', '0'))) as h:
        old_ids = h.unique_u64(np.concatenate(parts))
    first = 0 if (len(old_ids) and old_ids[0] == 0) else 1
    n_ids = first + len(old_ids)
    fu.log("relabel to new max-id %i" % n_ids)
    table = np.empty((len(old_ids), 2), dtype='uint64')
    table[:, 0] = old_ids
    table[:, 1] = np.arange(first, n_ids, dtype='uint64')
    fu.log("saving results to %s/%s" % (config['assignment_path'], config['assignment_key']))
    with vu.file_reader(config['assignment_path']) as f:
        if config['assignment_key'] in f:
            del f[config['assignment_key']]
        ds = f.create_dataset(config['assignment_key'], shape=table.shape, dtype='uint64', compression='gzip',
                              chunks=(max(1, min(1000000, len(table))), 2))
        ds.n_threads = config.get('threads_per_job', 1)
        ds[:] = table
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    find_labeling(job_id, path)
