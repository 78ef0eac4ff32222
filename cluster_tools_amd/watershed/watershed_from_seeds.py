#! /usr/bin/env python
"""WatershedFromSeeds task: drop-in for cluster_tools/watershed/watershed_from_seeds.py.

Task surface: WatershedFromSeedsBase / -Local / -Slurm / -LSF with the reference's parameters
(input, seeds, output, optional mask, dependency), task_name 'watershed_from_seeds' and config
keys (channel_begin/end, agglomerate_channels, size_filter 0; watershed_from_seeds.py:21-115).
Job entry `watershed_from_seeds(job_id, config_path)` (:202-249): the blocks (no halo) go to
libctws.so in batches (ctws_ws_from_seeds: normalize, seeds -> order-preserving labels, the
flood, the size filter, labels -> seed values, mask), reads of the next batch overlapping the
GPU work of the current one.  Like the reference job, the seeds are read from the OUTPUT file
(`ds_seeds = f_out[seeds_key]`, :236); `seeds_path` only travels in the job config.
"""
import json
import os
import sys
from concurrent import futures

from cluster_tools_amd import luigi_compat as luigi
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu
from cluster_tools_amd.utils.blocking import Blocking
from cluster_tools_amd.utils.task_utils import DummyTask
from cluster_tools_amd.cluster_tasks import SlurmTask, LocalTask, LSFTask


class WatershedFromSeedsBase(luigi.Task):
    """Seeded watershed of a boundary map, block by block."""

    task_name = 'watershed_from_seeds'
    src_file = os.path.abspath(__file__)

    input_path = luigi.Parameter()
    input_key = luigi.Parameter()
    seeds_path = luigi.Parameter()
    seeds_key = luigi.Parameter()
    output_path = luigi.Parameter()
    output_key = luigi.Parameter()
    mask_path = luigi.Parameter(default='')
    mask_key = luigi.Parameter(default='')
    dependency = luigi.TaskParameter(default=DummyTask())

    def requires(self):
        return self.dependency

    @staticmethod
    def default_task_config():
        config = LocalTask.default_task_config()
        config.update({'channel_begin': 0, 'channel_end': None, 'agglomerate_channels': 'mean', 'size_filter': 0})
        return config

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        shape = vu.get_shape(self.input_path, self.input_key)
        if len(shape) == 4:
            shape = shape[1:]
        config = self.get_task_config()
        # chunks: half a block, at most the volume
        chunks = tuple(min(bs // 2, sh) for bs, sh in zip(block_shape, shape))
        with vu.file_reader(self.output_path) as f:
            f.require_dataset(self.output_key, shape=shape, chunks=chunks, compression='gzip', dtype='uint64')
        config.update({'input_path': self.input_path, 'input_key': self.input_key,
                       'seeds_path': self.seeds_path, 'seeds_key': self.seeds_key,
                       'output_path': self.output_path, 'output_key': self.output_key,
                       'block_shape': block_shape})
        if self.mask_path != '':
            assert self.mask_key != ''
            config.update({'mask_path': self.mask_path, 'mask_key': self.mask_key})
        blocks = self.blocks_to_process(shape, block_shape, roi_begin, roi_end)
        self.run_jobs(min(len(blocks), self.max_jobs), blocks, config)


class WatershedFromSeedsLocal(WatershedFromSeedsBase, LocalTask):
    """WatershedFromSeeds on the local machine (one GPU handle per job process)."""


class WatershedFromSeedsSlurm(WatershedFromSeedsBase, SlurmTask):
    """WatershedFromSeeds on a slurm cluster."""


class WatershedFromSeedsLSF(WatershedFromSeedsBase, LSFTask):
    """WatershedFromSeeds on an lsf cluster."""


#
# Implementation
#

def _device():
    return int(os.environ.get('CTWS_DEVICE', os.environ.get('LOCAL_RANK', '0')))


def _read_block(blocking, block_id, ds_in, ds_seeds, mask, config):
    """One block's inputs (watershed_from_seeds.py:125-140 and :150-155 / :172-184)."""
    bb = vu.block_to_bb(blocking.getBlock(block_id))
    b = {'block_id': block_id, 'bb': bb}
    if mask is not None:
        in_mask = mask[bb].astype('bool')
        if in_mask.sum() == 0:
            b['skip'] = True  # an empty mask writes nothing (:178-181)
            return b
        b['mask'] = in_mask.view('uint8')
    if ds_in.ndim == 4:
        cb, ce = config.get('channel_begin', 0), config.get('channel_end', None)
        b['input'] = ds_in[(slice(cb, ce),) + bb]
    else:
        b['input'] = ds_in[bb]
    b['seeds'] = ds_seeds[bb]
    return b


def run_seeded_blocks(blocking, block_list, ds_in, ds_seeds, ds_out, mask, config, batch_blocks=None):
    """`_ws_block[_masked]` for every block of the job, in batches on the GPU; outputs are written
    and "processed block" logged in block-list order.  A block whose seeds overflow uint32
    raises there, as the reference's assert would."""
    from cluster_tools_amd import ctws
    lib_config = dict(config)
    if ds_in.ndim == 4:
        lib_config['channel_begin'], lib_config['channel_end'] = 0, None  # sliced on the host
    batch_blocks = batch_blocks or int(config.get('gpu_batch_blocks', 16))
    batches = [block_list[k:k + batch_blocks] for k in range(0, len(block_list), batch_blocks)]

    def read_batch(ids):
        return [_read_block(blocking, bid, ds_in, ds_seeds, mask, config) for bid in ids]

    with ctws.Handle(_device()) as h, futures.ThreadPoolExecutor(1) as io:
        nxt = io.submit(read_batch, batches[0]) if batches else None
        for bi in range(len(batches)):
            blocks = nxt.result()
            nxt = io.submit(read_batch, batches[bi + 1]) if bi + 1 < len(batches) else None
            for b in blocks:
                fu.log("start processing block %i" % b['block_id'])
            todo = [b for b in blocks if not b.get('skip')]
            res = h.ws_from_seeds(lib_config, todo) if todo else []
            by_id = {b['block_id']: r for b, r in zip(todo, res)}
            error = h.last_error()
            for b in blocks:
                r = by_id.get(b['block_id'])
                if r is not None and r['status'] == ctws.CTWS_BLOCK_FAILED:
                    raise ctws.CtwsError("block %i: %s" % (b['block_id'], error))
                if r is not None and r['status'] == ctws.CTWS_BLOCK_WRITTEN:
                    ds_out[b['bb']] = r['output']
                fu.log_block_success(b['block_id'])


def watershed_from_seeds(job_id, config_path):
    fu.log("start processing job %i" % job_id)
    fu.log("reading config from %s" % config_path)
    with open(config_path) as f:
        config = json.load(f)
    shape = list(vu.get_shape(config['input_path'], config['input_key']))
    if len(shape) == 4:
        shape = shape[1:]
    block_shape = list(config['block_shape'])
    blocking = Blocking([0, 0, 0], shape, block_shape)
    with vu.file_reader(config['input_path'], 'r') as f_in, vu.file_reader(config['output_path']) as f_out:
        ds_in = f_in[config['input_key']]
        assert ds_in.ndim in (3, 4)
        ds_seeds = f_out[config['seeds_key']]  # (sic) the output file, as the reference job
        assert ds_seeds.ndim == 3
        ds_out = f_out[config['output_key']]
        assert ds_out.ndim == 3
        mask = vu.load_mask(config['mask_path'], config['mask_key'], shape) if 'mask_path' in config else None
        run_seeded_blocks(blocking, config['block_list'], ds_in, ds_seeds, ds_out, mask, config)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    watershed_from_seeds(job_id, path)
