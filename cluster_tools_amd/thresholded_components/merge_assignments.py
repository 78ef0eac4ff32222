#! /usr/bin/env python
"""MergeAssignments: union-find over the face pairs -> the label assignment table
(cluster_tools/thresholded_components/merge_assignments.py:21-148; task surface unchanged).

The representatives are those of nifty's boost_ufd (libctws.so ctws_ufd_find: boost's
disjoint_sets, union by rank, pairs merged in sorted order).  As in the reference the table
written is `ufd.find(labels)` itself: the consecutive relabelling it computes afterwards is
assigned to a misspelled name and dropped (:130-132), so the ids are representatives, not
consecutive.  Also as there: if any BlockFaces job found no pair, no pair is merged at all
(`all(ass.size ...)`, :115).
"""
import json
import os
import sys

import numpy as np

from cluster_tools_amd import luigi_compat as luigi
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu
from cluster_tools_amd.cluster_tasks import SlurmTask, LocalTask, LSFTask


class MergeAssignmentsBase(luigi.Task):
    task_name = 'merge_assignments'
    src_file = os.path.abspath(__file__)
    allow_retry = False

    output_path = luigi.Parameter()
    output_key = luigi.Parameter()
    shape = luigi.ListParameter()
    offset_path = luigi.Parameter()
    save_prefix = luigi.Parameter(default='cc_assignments')
    dependency = luigi.TaskParameter()

    def requires(self):
        return self.dependency

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        block_list = vu.blocks_in_volume(self.shape, block_shape, roi_begin, roi_end)
        config = self.get_task_config()
        config.update({'output_path': self.output_path, 'output_key': self.output_key,
                       'tmp_folder': self.tmp_folder, 'n_jobs': min(len(block_list), self.max_jobs),
                       'offset_path': self.offset_path, 'save_prefix': self.save_prefix})
        self.run_jobs(1, None, config)


class MergeAssignmentsLocal(MergeAssignmentsBase, LocalTask):
    pass


class MergeAssignmentsSlurm(MergeAssignmentsBase, SlurmTask):
    pass


class MergeAssignmentsLSF(MergeAssignmentsBase, LSFTask):
    pass


def merge_assignments(job_id, config_path):
    from cluster_tools_amd import ctws
    fu.log("start processing job %i" % job_id)
    fu.log("reading config from %s" % config_path)
    with open(config_path) as f:
        config = json.load(f)
    with open(config['offset_path']) as f:
        n_labels = int(json.load(f)['n_labels'])
    parts = [np.load(os.path.join(config['tmp_folder'], '%s_%i.npy' % (config['save_prefix'], j)))
             for j in range(config['n_jobs'])]
    if all(p.size for p in parts):
        pairs = np.unique(np.concatenate(parts, axis=0).astype('uint64'), axis=0)
        assert pairs.shape[1] == 2
        fu.log("have %i pairs of node assignments" % len(pairs))
        assert int(pairs.max()) + 1 <= n_labels, "%i, %i" % (int(pairs.max()) + 1, n_labels)
    else:
        fu.log("did not find any node assignments, label assignment will be identity")
        pairs = np.zeros((0, 2), dtype='uint64')
    label_assignments = ctws.ufd_find(n_labels, pairs)
    fu.log("reducing the number of labels from %i to %i" % (n_labels, len(np.unique(label_assignments))))
    with vu.file_reader(config['output_path']) as f:
        if config['output_key'] in f:
            del f[config['output_key']]
        ds = f.create_dataset(config['output_key'], shape=label_assignments.shape, dtype='uint64',
                              compression='gzip', chunks=(min(65334, n_labels),))
        ds[:] = label_assignments
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    merge_assignments(job_id, path)
