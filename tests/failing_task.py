#! /usr/bin/env python
"""Deterministically failing task for the retry machinery (mirrors the reference's
test/retry/failing_task.py): blocks with id % 4 == 1 fail on the first try."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cluster_tools_amd import luigi_compat as luigi  # noqa: E402
import cluster_tools_amd.utils.volume_utils as vu  # noqa: E402
import cluster_tools_amd.utils.function_utils as fu  # noqa: E402
from cluster_tools_amd.utils.blocking import Blocking  # noqa: E402
from cluster_tools_amd.cluster_tasks import LocalTask  # noqa: E402


class FailingTaskBase(luigi.Task):
    task_name = 'failing_task'
    src_file = os.path.abspath(__file__)

    output_path = luigi.Parameter()
    output_key = luigi.Parameter()
    shape = luigi.ListParameter()

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        config = self.get_task_config()
        shape = tuple(self.shape)
        with vu.file_reader(self.output_path) as f:
            f.require_dataset(self.output_key, shape=shape, chunks=tuple(block_shape), dtype='uint8')
        config.update({'output_path': self.output_path, 'output_key': self.output_key,
                       'n_retries': self.n_retries, 'block_shape': block_shape})
        if self.n_retries == 0:
            block_list = vu.blocks_in_volume(shape, block_shape, roi_begin, roi_end)
        else:
            block_list = self.block_list
        n_jobs = min(len(block_list), self.max_jobs)
        self.prepare_jobs(n_jobs, block_list, config)
        self.submit_jobs(n_jobs)
        self.wait_for_jobs()
        self.check_jobs(n_jobs)


class FailingTaskLocal(FailingTaskBase, LocalTask):
    pass


def failing_task(job_id, config_path):
    with open(config_path) as f:
        config = json.load(f)
    shape = vu.get_shape(config['output_path'], config['output_key'])
    blocking = Blocking([0, 0, 0], list(shape), list(config['block_shape']))
    with vu.file_reader(config['output_path']) as f:
        ds = f[config['output_key']]
        for block_id in config['block_list']:
            if config['n_retries'] == 0 and block_id % 4 == 1:
                raise RuntimeError("Fail")
            ds[vu.block_to_bb(blocking.getBlock(block_id))] = 1
            fu.log_block_success(block_id)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    failing_task(job_id, path)
