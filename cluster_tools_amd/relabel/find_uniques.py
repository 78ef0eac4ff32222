#! /usr/bin/env python
"""FindUniques: per-job unique labels of the watershed output on the GPU
(cluster_tools/relabel/find_uniques.py:20-159; task surface unchanged)."""
import json
import os
import sys
from concurrent import futures

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
    # not in the reference: the folder the producing watershed task wrote its per-block
    # uniques to (WatershedBase.uniques_path); blocks with a file there are not read
    uniques_path = luigi.Parameter(default='')

    def requires(self):
        return self.dependency

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        blocks = self.blocks_to_process(vu.get_shape(self.input_path, self.input_key), block_shape,
                                        roi_begin, roi_end)
        self.run_jobs(min(len(blocks), self.max_jobs), blocks,
                      dict(input_path=self.input_path, input_key=self.input_key, block_shape=block_shape,
                           tmp_folder=self.tmp_folder, return_counts=self.return_counts,
                           uniques_path=self.uniques_path))


class FindUniquesLocal(FindUniquesBase, LocalTask):
    pass


class FindUniquesSlurm(FindUniquesBase, SlurmTask):
    pass


class FindUniquesLSF(FindUniquesBase, LSFTask):
    pass


def _device():
    return int(os.environ.get('CTWS_DEVICE', os.environ.get('LOCAL_RANK', '0')))


def find_uniques(job_id, config_path):
    """Job entry (find_uniques.py:115-159): the sorted unique ids of the job's blocks.

    Every block goes through the GPU bitmap unique (ctws_unique_u64, k_relabel.hip); the
    per-block id sets are then merged by one more GPU unique over their concatenation.
    Blocks are read ahead on a thread while the GPU works.  As in the reference, an all-zero
    block contributes [0] without logging "processed block" (find_uniques.py:97-101).

    With `uniques_path` (and without return_counts) a block whose uniques the watershed job
    already computed on the GPU from the labels it wrote (watershed.py run_blocks) is taken from
    that file; only the other blocks are read.  A job whose blocks all have files opens no GPU
    handle and merges the sorted per-block sets with numpy.
    """
    from cluster_tools_amd import ctws
    fu.log("start processing job %i" % job_id)
    fu.log("reading config from %s" % config_path)
    with open(config_path) as f:
        config = json.load(f)
    return_counts = config['return_counts']
    block_list = config['block_list']
    cached = {}
    if config.get('uniques_path') and not return_counts:
        from cluster_tools_amd.watershed.watershed import block_uniques_file
        for block_id in block_list:
            path = block_uniques_file(config['uniques_path'], block_id)
            if os.path.exists(path):
                cached[block_id] = np.load(path)
    if len(cached) == len(block_list):
        per_block = []
        for block_id in block_list:
            fu.log("start processing block %i" % block_id)
            u = cached[block_id]
            per_block.append(u)
            if not (len(u) == 1 and u[0] == 0):
                fu.log_block_success(block_id)
        # the blocks' sets are sorted and small (ids, not voxels): a host merge
        unique_values = np.unique(np.concatenate(per_block)) if per_block else np.zeros(0, 'uint64')
        _save(config, job_id, unique_values.astype('uint64'))
        return
    with vu.file_reader(config['input_path'], 'r') as f, ctws.Handle(_device()) as h, \
            futures.ThreadPoolExecutor(1) as io:
        ds = f[config['input_key']]
        blocking = Blocking([0, 0, 0], list(ds.shape), list(config['block_shape']))
        to_read = [b for b in block_list if b not in cached]

        def read(block_id):
            return ds[vu.block_to_bb(blocking.getBlock(block_id))]

        per_block, per_counts = [], []
        nxt = io.submit(read, to_read[0]) if to_read else None
        k = 0
        for block_id in block_list:
            fu.log("start processing block %i" % block_id)
            if block_id in cached:
                u = cached[block_id]
                per_block.append(u)
                if not (len(u) == 1 and u[0] == 0):
                    fu.log_block_success(block_id)
                continue
            labels = nxt.result()
            k += 1
            nxt = io.submit(read, to_read[k]) if k < len(to_read) else None
            if return_counts:
                u, c = h.unique_counts_u64(labels)
                per_counts.append(c)
            else:
                u = h.unique_u64(labels)
            per_block.append(u)
            if not (len(u) == 1 and u[0] == 0):
                fu.log_block_success(block_id)
        if return_counts and per_block:
            # counts of equal values summed over the blocks (find_uniques.py:143-151): a merge of
            # the per-block (value, count) tables -- uniques, not voxels -- on the host
            allv = np.concatenate(per_block)
            allc = np.concatenate(per_counts)
            order = np.argsort(allv, kind='stable')
            allv, allc = allv[order], allc[order]
            unique_values, starts = np.unique(allv, return_index=True)
            counts = np.add.reduceat(allc, starts).astype('uint64')
            count_path = os.path.join(config['tmp_folder'], 'counts_job_%i.npy' % job_id)
            np.save(count_path, counts)
        else:
            unique_values = h.unique_u64(np.concatenate(per_block)) if per_block else np.zeros(0, 'uint64')
    _save(config, job_id, unique_values)


def _save(config, job_id, unique_values):
    save_path = os.path.join(config['tmp_folder'], 'find_uniques_job_%i.npy' % job_id)
    fu.log("saving results to %s" % save_path)
    np.save(save_path, unique_values)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    find_uniques(job_id, path)
