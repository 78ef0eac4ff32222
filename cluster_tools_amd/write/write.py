#! /usr/bin/env python
"""Write: apply an assignment table to every block and set attrs['maxId']
(cluster_tools/write/write.py:28-329; task surface unchanged).  takeDict runs on the GPU
(k_u64_lookup); the pickled-dict assignment form is not supported (no unpickling of data)."""
import json
import os
import sys
from concurrent import futures

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
        blocks = self.blocks_to_process(shape, block_shape, roi_begin, roi_end, job_prefix=self.identifier)
        self.run_jobs(min(len(blocks), self.max_jobs), blocks, config, self.identifier)

    def output(self):
        return luigi.LocalTarget(os.path.join(self.tmp_folder, '%s_%s.log' % (self.task_name, self.identifier)))


class WriteLocal(WriteBase, LocalTask):
    pass


class WriteSlurm(WriteBase, SlurmTask):
    pass


class WriteLSF(WriteBase, LSFTask):
    pass


def _load_table(path, key):
    """The assignment as (keys ascending, values): an (N, 2) / (2, N) table [old, new], or a
    1-D array mapping index -> value (write.py:229-261; pickled dicts are not loaded)."""
    with vu.file_reader(path, 'r') as f:
        node_labels = np.asarray(f[key][:])
    if node_labels.ndim == 0:
        node_labels = node_labels.reshape(1)
    if node_labels.ndim == 1:
        return np.arange(len(node_labels), dtype='uint64'), node_labels.astype('uint64'), True
    if node_labels.shape[1] == 2:
        keys, values = node_labels[:, 0], node_labels[:, 1]
    elif node_labels.shape[0] == 2:
        keys, values = node_labels[0], node_labels[1]
    else:
        raise ValueError("Invalid shape for 2d node labels")
    keys = keys.astype('uint64')
    values = values.astype('uint64')
    if len(keys) > 1 and not (keys[1:] > keys[:-1]).all():
        order = np.argsort(keys, kind='stable')   # FindLabeling tables are sorted already
        keys, values = keys[order], values[order]
    return keys, values, False


def write(job_id, config_path):
    """Job entry (write.py:264-329): every block through the assignment on the GPU.

    The table is uploaded once per job and stays resident (ctws_set_table_u64); each block is
    read (next one ahead on a thread), mapped by k_u64_lookup (binary search per voxel) and
    written back.  All-zero blocks are skipped, labels missing from the table raise unless
    allow_empty_assignments (then they keep their id), job 0 writes attrs['maxId'].
    """
    from cluster_tools_amd import ctws
    fu.log("start processing job %i" % job_id)
    fu.log("loading config from %s" % config_path)
    with open(config_path) as f:
        config = json.load(f)
    input_path, input_key = config['input_path'], config['input_key']
    output_path = config.get('output_path', input_path)
    output_key = config.get('output_key', input_key)
    allow_empty = config.get('allow_empty_assignments', False)
    keys, values, is_array = _load_table(config['assignment_path'], config['assignment_key'])
    offsets, skip = None, set()
    if config.get('offset_path'):
        fu.log("loading offsets from %s" % config['offset_path'])
        with open(config['offset_path']) as f:
            oc = json.load(f)
        offsets, skip = oc['offsets'], set(oc['empty_blocks'])
    block_list = [b for b in config['block_list'] if b not in skip]
    with vu.file_reader(input_path) as f_in, vu.file_reader(output_path) as f_out, \
            ctws.Handle(int(os.environ.get('CTWS_DEVICE', '0'))) as h, futures.ThreadPoolExecutor(1) as io:
        ds_in, ds_out = f_in[input_key], f_out[output_key]
        blocking = Blocking([0, 0, 0], list(ds_in.shape), list(config['block_shape']))
        h.set_table_u64(keys, values)

        def read(block_id):
            bb = vu.block_to_bb(blocking.getBlock(block_id))
            return bb, np.ascontiguousarray(ds_in[bb], dtype='uint64')

        nxt = io.submit(read, block_list[0]) if block_list else None
        for k, block_id in enumerate(block_list):
            fu.log("start processing block %i" % block_id)
            bb, seg = nxt.result()
            nxt = io.submit(read, block_list[k + 1]) if k + 1 < len(block_list) else None
            nz = seg != 0
            if not nz.any():
                fu.log_block_success(block_id)
                continue
            if offsets is not None:
                seg[nz] += np.uint64(offsets[block_id])
            missing = h.lookup_u64(seg)
            if missing and (is_array or not allow_empty):
                raise KeyError("block %i: %i labels are not in the assignment table" % (block_id, missing))
            ds_out[bb] = seg
            fu.log_block_success(block_id)
        if job_id == 0:
            ds_out.attrs['maxId'] = int(values.max()) if len(values) else 0
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    write(job_id, path)
