#! /usr/bin/env python
"""Write: apply an assignment table to every block and set attrs['maxId']
(cluster_tools/write/write.py:28-329).  numpy implementation of takeDict (sorted-table
lookup); the pickled-dict assignment form is not supported (no unpickling of data)."""
import json
import os
import sys

import numpy as np

from cluster_tools_amd import luigi_compat as luigi
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu
from cluster_tools_amd.utils.blocking import Blocking
from cluster_tools_amd.utils.task_utils import DummyTask
from cluster_tools_amd.cluster_tasks import SlurmTask, LocalTask, LSFTask


class WriteBase(luigi.Task):
    task_name = 'write'
    src_file = os.path.abspath(__file__)

    input_path = luigi.Parameter()
    input_key = luigi.Parameter()
    output_path = luigi.Parameter()
    output_key = luigi.Parameter()
    assignment_path = luigi.Parameter()
    assignment_key = luigi.Parameter(default=None)
    dependency = luigi.TaskParameter(default=DummyTask())
    identifier = luigi.Parameter()
    offset_path = luigi.Parameter(default='')

    def requires(self):
        return self.dependency

    @staticmethod
    def default_task_config():
        config = LocalTask.default_task_config()
        config.update({'chunks': None, 'allow_empty_assignments': False})
        return config

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        shape = vu.get_shape(self.input_path, self.input_key)
        config = self.get_task_config()
        chunks = config.pop('chunks', None)
        if chunks is None:
            chunks = tuple(min(bs // 2, sh) for bs, sh in zip(block_shape, shape))
        with vu.file_reader(self.output_path) as f:
            if self.output_key in f:
                chunks = f[self.output_key].chunks
            assert all(bs % ch == 0 for bs, ch in zip(block_shape, chunks)), (block_shape, chunks)
            f.require_dataset(self.output_key, shape=shape, chunks=chunks, compression='gzip', dtype='uint64')
        in_place = (self.input_path == self.output_path) and (self.input_key == self.output_key)
        if self.assignment_key is None:
            raise NotImplementedError("pickled assignment maps are not supported: give an assignment_key")
        config.update({'input_path': self.input_path, 'input_key': self.input_key, 'block_shape': block_shape,
                       'assignment_path': self.assignment_path, 'assignment_key': self.assignment_key})
        if self.offset_path != '':
            config.update({'offset_path': self.offset_path})
        if not in_place:
            config.update({'output_path': self.output_path, 'output_key': self.output_key})
        if self.n_retries == 0:
            block_list = vu.blocks_in_volume(shape, block_shape, roi_begin, roi_end)
        else:
            block_list = self.block_list
            self.clean_up_for_retry(block_list, self.identifier)
        self._write_log('scheduling %i blocks to be processed' % len(block_list))
        n_jobs = min(len(block_list), self.max_jobs)
        self.prepare_jobs(n_jobs, block_list, config, self.identifier)
        self.submit_jobs(n_jobs, self.identifier)
        self.wait_for_jobs(self.identifier)
        self.check_jobs(n_jobs, self.identifier)

    def output(self):
        return luigi.LocalTarget(os.path.join(self.tmp_folder, '%s_%s.log' % (self.task_name, self.identifier)))


class WriteLocal(WriteBase, LocalTask):
    pass


class WriteSlurm(WriteBase, SlurmTask):
    pass


class WriteLSF(WriteBase, LSFTask):
    pass


def _apply_table(seg, table, allow_empty):
    """nt.takeDict with an (N, 2) assignment table sorted by old id."""
    keys, vals = table[:, 0], table[:, 1]
    order = np.argsort(keys, kind='stable')
    keys, vals = keys[order], vals[order]
    pos = np.clip(np.searchsorted(keys, seg), 0, len(keys) - 1)
    hit = keys[pos] == seg
    if not hit.all():
        if not allow_empty:
            raise KeyError("labels missing from the assignment table")
        return np.where(hit, vals[pos], seg)
    return vals[pos]


def write(job_id, config_path):
    fu.log("start processing job %i" % job_id)
    fu.log("loading config from %s" % config_path)
    with open(config_path) as f:
        config = json.load(f)
    input_path, input_key = config['input_path'], config['input_key']
    output_path = config.get('output_path', input_path)
    output_key = config.get('output_key', input_key)
    allow_empty = config.get('allow_empty_assignments', False)
    with vu.file_reader(config['assignment_path'], 'r') as f:
        table = f[config['assignment_key']][:]
    if table.ndim == 1:
        table = np.stack([np.arange(len(table), dtype='uint64'), table.astype('uint64')], axis=1)
    elif table.shape[1] != 2:
        table = table.T
    offsets = None
    if config.get('offset_path'):
        with open(config['offset_path']) as f:
            oc = json.load(f)
        offsets, empty_blocks = oc['offsets'], set(oc['empty_blocks'])
    with vu.file_reader(input_path) as f_in, vu.file_reader(output_path) as f_out:
        ds_in, ds_out = f_in[input_key], f_out[output_key]
        blocking = Blocking([0, 0, 0], list(ds_in.shape), list(config['block_shape']))
        for block_id in config['block_list']:
            if offsets is not None and block_id in empty_blocks:
                continue
            fu.log("start processing block %i" % block_id)
            bb = vu.block_to_bb(blocking.getBlock(block_id))
            seg = ds_in[bb]
            mask = seg != 0
            if mask.sum() == 0:
                fu.log_block_success(block_id)
                continue
            if offsets is not None:
                seg[mask] += np.uint64(offsets[block_id])
            ds_out[bb] = _apply_table(seg, table, allow_empty)
            fu.log_block_success(block_id)
        if job_id == 0:
            ds_out.attrs['maxId'] = int(table[:, 1].max())
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    write(job_id, path)
