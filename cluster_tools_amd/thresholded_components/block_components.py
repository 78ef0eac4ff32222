#! /usr/bin/env python
"""BlockComponents: threshold every block and label its 26-connected components on the GPU
(cluster_tools/thresholded_components/block_components.py:21-298; task surface unchanged).

Per block the job reads the input (the next block ahead on a thread), calls
ctws_threshold_components (k_threshcc.hip: normalize, threshold, mask, LDS-tiled union-find,
skimage numbering) and writes the labels of a non-empty block; the per-block offsets
(`max + 1`, 0 for an empty block) go to `connected_components_offsets_<job>.json` as in the
reference.  The block crosses to the GPU in the dataset's dtype: raw values are thresholded as
numpy compares them with the Python float threshold, and the Gaussian prefilter
(sigma_prefilter > 0, vigra gaussianSmoothing + normalize) runs on the GPU too
(ctws_threshold_components_ex).
"""
import contextlib
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


class BlockComponentsBase(luigi.Task):
    task_name = 'block_components'
    src_file = os.path.abspath(__file__)
    allow_retry = False

    input_path = luigi.Parameter()
    input_key = luigi.Parameter()
    output_path = luigi.Parameter()
    output_key = luigi.Parameter()
    dependency = luigi.TaskParameter()
    threshold = luigi.FloatParameter()
    threshold_mode = luigi.Parameter(default='greater')
    mask_path = luigi.Parameter(default='')
    mask_key = luigi.Parameter(default='')
    channel = luigi.Parameter(default=None)
    # the merge tail in the jobs (merge_in_job.py; set by ThresholdedComponentsWorkflow for a local
    # target): the assignment dataset, MergeOffsets' offsets file and BlockFaces' max_jobs
    assignment_key = luigi.Parameter(default='')
    offsets_path = luigi.Parameter(default='')

    threshold_modes = ('greater', 'less', 'equal')

    @staticmethod
    def default_task_config():
        config = LocalTask.default_task_config()
        config.update({'sigma_prefilter': 0})
        return config

    def requires(self):
        return self.dependency

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        shape = vu.get_shape(self.input_path, self.input_key)
        assert self.threshold_mode in self.threshold_modes
        config = self.get_task_config()
        config.update({'input_path': self.input_path, 'input_key': self.input_key,
                       'output_path': self.output_path, 'output_key': self.output_key,
                       'block_shape': block_shape, 'tmp_folder': self.tmp_folder,
                       'threshold': self.threshold, 'threshold_mode': self.threshold_mode})
        if self.mask_path != '':
            assert self.mask_key != ''
            config.update({'mask_path': self.mask_path, 'mask_key': self.mask_key})
        chunks = config.pop('chunks', None)
        if chunks is None:
            chunks = tuple(bs // 2 for bs in block_shape)
        if self.channel is None:
            assert len(shape) == 3, str(len(shape))
        else:
            assert isinstance(self.channel, (int, tuple, list))
            assert len(shape) == 4, str(len(shape))
            chans = [self.channel] if isinstance(self.channel, int) else list(self.channel)
            assert all(isinstance(c, int) for c in chans)
            assert shape[0] > max(chans), "%i, %i" % (shape[0], max(chans))
            shape = shape[1:]
            config.update({'channel': self.channel})
        chunks = tuple(min(ch, sh) for ch, sh in zip(chunks, shape))
        compression = config.pop('compression', 'gzip')
        with vu.file_reader(self.output_path) as f:
            f.require_dataset(self.output_key, shape=tuple(shape), dtype='uint64', compression=compression,
                              chunks=chunks)
        block_list = vu.blocks_in_volume(shape, block_shape, roi_begin, roi_end)
        n_jobs = min(len(block_list), self.max_jobs)
        consecutive = False
        if self.assignment_key != '' and isinstance(self, LocalTask):
            from cluster_tools_amd.watershed.watershed import job_group_config
            merge = job_group_config(self.tmp_folder, n_jobs)
            merge.update({'assignment_key': self.assignment_key, 'offsets_path': self.offsets_path,
                          'output_path': self.output_path, 'faces_max_jobs': self.max_jobs,
                          'block_list': list(block_list)})
            config['merge'] = merge
            self.allow_retry = False   # the offsets, pairs and ids depend on every block
            consecutive = True         # face planes of consecutive blocks stay in the job
        self.run_jobs(n_jobs, block_list, config, consecutive_blocks=consecutive)


class BlockComponentsLocal(BlockComponentsBase, LocalTask):
    pass


class BlockComponentsSlurm(BlockComponentsBase, SlurmTask):
    pass


class BlockComponentsLSF(BlockComponentsBase, LSFTask):
    pass


def _device():
    return int(os.environ.get('CTWS_DEVICE', os.environ.get('LOCAL_RANK', '0')))


def _read_block(blocking, block_id, ds_in, mask, channel):
    """One block's input and mask (block_components.py:147-158 / :188-206): the unmasked single
    channel block is normalized on the GPU; channels are summed in the dataset dtype."""
    bb = vu.block_to_bb(blocking.getBlock(block_id))
    b = {'block_id': block_id, 'bb': bb, 'mask': None}
    if mask is not None:
        in_mask = np.asarray(mask[bb]).astype('bool')
        if in_mask.sum() == 0:
            b['skip'] = True
            return b
        b['mask'] = in_mask
    if channel is None:
        b['input'] = ds_in[bb]
    else:
        shape = tuple(s.stop - s.start for s in bb)
        x = np.zeros(shape, dtype=ds_in.dtype)
        for chan in ([channel] if isinstance(channel, int) else channel):
            x += ds_in[(slice(chan, chan + 1),) + bb].squeeze()
        b['input'] = x
    return b


def run_component_blocks(blocking, block_list, ds_in, ds_out, mask, config, keep=None, started=None,
                         spill=False):
    """`_cc_block[_with_mask]` for every block of the job -> {block_id: offset}.  keep (a list):
    the blocks' labels are collected there as (block_id, bb, labels or None, count) instead of
    written (the in-job merge writes the final ids): uint32 (a block has < 2^32 voxels, ctws
    refuses larger ones), or with spill=True written to ds_out as they are and re-read by the
    merge (merge_in_job.SpilledBlock) when the job's labels would not fit its share of host
    memory.  started: called once the first read is under way (the merge's process group starts
    there, its torch import overlapping the read)."""
    from cluster_tools_amd.thresholded_components.merge_in_job import SpilledBlock
    from cluster_tools_amd import ctws
    sigma = float(config.get('sigma_prefilter', 0) or 0)
    threshold, mode = config['threshold'], config['threshold_mode']
    channel = config.get('channel', None)
    offsets = {}
    # chunk inflate / deflate on a pool of the job's threads (libdeflate releases the GIL)
    ds_in.n_threads = ds_out.n_threads = max(1, int(config.get('threads_per_job', 1)))
    with futures.ThreadPoolExecutor(1) as io, contextlib.ExitStack() as stack:
        nxt = io.submit(_read_block, blocking, block_list[0], ds_in, mask, channel) if block_list else None
        if started is not None:
            started()
        h = stack.enter_context(ctws.Handle(_device()))
        for k, block_id in enumerate(block_list):
            b = nxt.result()
            nxt = (io.submit(_read_block, blocking, block_list[k + 1], ds_in, mask, channel)
                   if k + 1 < len(block_list) else None)
            fu.log("start processing block %i" % block_id)
            if b.get('skip'):
                offsets[block_id] = 0
                if keep is not None:
                    keep.append((block_id, b['bb'], None, 0))
                else:
                    fu.log_block_success(block_id)
                continue
            # normalized first: the unmasked single-channel block (`_cc_block`,
            # block_components.py:150-151) and, before its prefilter, a masked block (:208-209);
            # otherwise raw values (sigma 0) or the raw channel sum smoothed (:160-162)
            prenorm = (mask is None and channel is None) or (mask is not None and sigma > 0)
            labels, n = h.threshold_components(b['input'], threshold, mode, mask=b['mask'], normalize=prenorm,
                                               sigma=sigma)
            offsets[block_id] = n + 1 if n else 0
            if keep is not None:
                lab = None
                if n and spill:
                    ds_out[b['bb']] = labels
                    lab = SpilledBlock(ds_out, b['bb'])
                elif n:
                    lab = labels.astype(np.uint32)
                keep.append((block_id, b['bb'], lab, offsets[block_id]))
                continue
            if n:
                ds_out[b['bb']] = labels
            fu.log_block_success(block_id)
    return offsets


def block_components(job_id, config_path):
    fu.log("start processing job %i" % job_id)
    fu.log("reading config from %s" % config_path)
    with open(config_path) as f:
        config = json.load(f)
    fu.log("Applying threshold %f with mode %s" % (config['threshold'], config['threshold_mode']))
    channel = config.get('channel', None)
    with vu.file_reader(config['input_path'], 'r') as f_in, vu.file_reader(config['output_path']) as f_out:
        ds_in = f_in[config['input_key']]
        ds_out = f_out[config['output_key']]
        shape = list(ds_in.shape)
        if channel is not None:
            shape = shape[1:]
        assert len(shape) == 3
        blocking = Blocking([0, 0, 0], shape, list(config['block_shape']))
        mask = None
        if config.get('mask_path', ''):
            mask = vu.load_mask(config['mask_path'], config['mask_key'], shape)
        if config.get('merge'):
            _run_blocks_merge(job_id, blocking, ds_in, ds_out, mask, config)
            fu.log_job_success(job_id)
            return
        offsets = run_component_blocks(blocking, config['block_list'], ds_in, ds_out, mask, config)
    save_path = os.path.join(config['tmp_folder'], 'connected_components_offsets_%i.json' % job_id)
    with open(save_path, 'w') as f:
        json.dump({int(k): int(v) for k, v in offsets.items()}, f)
    fu.log_job_success(job_id)


def spill_labels(blocking, block_list, n_jobs, config):
    """Whether this job writes its blocks' labels as it goes and re-reads them in the merge
    (config 'merge_spill': true / false; default: when the job's uint32 labels plus the largest
    block's uint64 write buffer exceed its share -- the local jobs of the task on this node -- of
    half the available host memory)."""
    force = config.get('merge_spill')
    if force is not None:
        return bool(force)
    import psutil
    vox = [int(np.prod([s.stop - s.start for s in vu.block_to_bb(blocking.getBlock(b))])) for b in block_list]
    need = 4 * sum(vox) + 8 * max(vox, default=0)
    return need > psutil.virtual_memory().available // (2 * max(1, n_jobs))


def _run_blocks_merge(job_id, blocking, ds_in, ds_out, mask, config):
    """The job's blocks, then the merge tail over the jobs' process group (merge_in_job.py)."""
    import torch.distributed as dist
    from cluster_tools_amd.thresholded_components.merge_in_job import merge_in_job
    from cluster_tools_amd.watershed import job_relabel
    from cluster_tools_amd.cluster_tasks import split_blocks
    m = config['merge']
    block_list = m['block_list']
    owner = {}
    for j, blocks in enumerate(split_blocks(block_list, m['n_jobs'], consecutive=True)):
        for b in blocks:
            owner[b] = j
    group, init_err = [], []

    def start_group():
        try:
            job_relabel.init_group(job_id, m['n_jobs'], m['rendezvous'], m['backend'], device=_device())
        except Exception as e:  # recorded: a second rendezvous would only wait out the timeout again
            init_err.append(e)
            raise
        group.append(True)

    failed = None
    keep = []
    spill = spill_labels(blocking, config['block_list'], m['n_jobs'], config)
    if spill:
        fu.log("labels of this job's blocks written as they are and re-read by the merge (host memory)")
    try:
        try:
            run_component_blocks(blocking, config['block_list'], ds_in, ds_out, mask, config, keep=keep,
                                 started=start_group, spill=spill)
        except Exception as e:  # still take part in the exchange: every job then raises
            import traceback
            traceback.print_exc()
            failed = e
        if init_err:
            raise init_err[0]
        if not group:   # (failed before its first read)
            start_group()
        merge_in_job(job_id, [] if failed else keep, blocking, block_list, owner, dict(m, tmp_folder=config['tmp_folder']),
                     ds_out, log=fu.log, device=_device(), failed=failed is not None)
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()
    if failed is not None:
        raise failed


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    block_components(job_id, path)
