#! /usr/bin/env python
"""Watershed task: drop-in for cluster_tools/watershed/watershed.py.

Task surface (same classes, parameters, task_name, config keys and defaults as
watershed.py:34-128): WatershedBase / WatershedLocal / WatershedSlurm / WatershedLSF.
Job entry `watershed(job_id, config_path)` (watershed.py:344-384): the per-block loop of
`_ws_block` (:285-341) becomes batched calls into libctws.so (the gfx950 kernels); this module
keeps the dataset I/O, the outer/inner bounding boxes (_get_bbs, :252-264) and the
"processed block"/"processed job" log protocol.  Input reads of the next batch and output
writes of the previous one overlap the GPU work of the current batch.
"""
import contextlib
import json
import os
import shutil
import sys
from concurrent import futures

import numpy as np

from cluster_tools_amd import luigi_compat as luigi
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu
from cluster_tools_amd.utils.blocking import Blocking
from cluster_tools_amd.cluster_tasks import SlurmTask, LocalTask, LSFTask


class WatershedBase(luigi.Task):
    """Watershed base class."""

    task_name = 'watershed'
    src_file = os.path.abspath(__file__)

    input_path = luigi.Parameter()
    input_key = luigi.Parameter()
    output_path = luigi.Parameter()
    output_key = luigi.Parameter()
    mask_path = luigi.Parameter(default='')
    mask_key = luigi.Parameter(default='')
    # not in the reference: a folder for the per-block uniques of the written labels, which a
    # following FindUniques (RelabelWorkflow's uniques_path) reads instead of the volume
    uniques_path = luigi.Parameter(default='')
    # not in the reference: with an assignment key (target 'local', one pass), the jobs form a
    # process group after their blocks and write the relabelled ids themselves, with the
    # assignment table and maxId of RelabelWorkflow (job_relabel.py); WatershedWorkflow sets it
    assignment_path = luigi.Parameter(default='')
    assignment_key = luigi.Parameter(default='')

    @staticmethod
    def default_task_config():
        config = LocalTask.default_task_config()
        config.update({'threshold': .5,
                       'apply_dt_2d': True, 'pixel_pitch': None,
                       'apply_ws_2d': True, 'sigma_seeds': 2., 'size_filter': 25,
                       'sigma_weights': 2., 'halo': [0, 0, 0],
                       'channel_begin': 0, 'channel_end': None,
                       'agglomerate_channels': 'mean', 'alpha': 0.8,
                       'invert_inputs': False, 'non_maximum_suppression': False})
        return config

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end, block_list_path = self.global_config_values(True)
        self.init(shebang)
        shape, ws_config = ws_task_setup(self, block_shape)
        blocks = self.blocks_to_process(shape, block_shape, roi_begin, roi_end, block_list_path)
        n_jobs = min(len(blocks), self.max_jobs)
        consecutive = False
        if self.assignment_key != '' and isinstance(self, LocalTask):
            ws_config['relabel'] = relabel_job_config(self, n_jobs)
            self.allow_retry = False  # the group numbers all blocks at once: no partial re-runs
            # a job takes consecutive blocks (neighbours: their halo chunks are inflated once,
            # ds_in's chunk cache); which job runs a block does not change its result
            consecutive = True
        self.run_jobs(n_jobs, blocks, ws_config, consecutive_blocks=consecutive)


def ws_task_setup(task, block_shape):
    """Shared by the watershed tasks: the 3-D output shape (a 4-D input's channel axis dropped),
    the gzip uint64 output dataset with half-block chunks, and the job config = task config +
    paths (+ mask)."""
    shape = tuple(vu.get_shape(task.input_path, task.input_key))[-3:]
    with vu.file_reader(task.output_path) as f:
        f.require_dataset(task.output_key, shape=shape, chunks=tuple(b // 2 for b in block_shape),
                          compression='gzip', dtype='uint64')
    cfg = dict(task.get_task_config(), input_path=task.input_path, input_key=task.input_key,
               output_path=task.output_path, output_key=task.output_key, block_shape=block_shape)
    if task.mask_path != '':
        assert task.mask_key != ''
        cfg.update(mask_path=task.mask_path, mask_key=task.mask_key)
    if task.uniques_path != '':
        # every block of this run rewrites its file; files of an earlier run must not survive
        shutil.rmtree(task.uniques_path, ignore_errors=True)
        os.makedirs(task.uniques_path)
        cfg['uniques_path'] = task.uniques_path
    return shape, cfg


def job_group_config(tmp_folder, n_jobs):
    """The process group of a task's local jobs: rendezvous, group size and backend (RCCL when
    every job owns a GPU, gloo when jobs share one; CTWS_JOB_DIST_BACKEND overrides).  The
    rendezvous is a file store in tmp_folder, fresh per run (a TCP port picked here could be
    taken by another process before the jobs bind it)."""
    import uuid
    from cluster_tools_amd.cluster_tasks import _count_gpus
    store = os.path.join(os.path.abspath(tmp_folder), 'job_rendezvous_%s' % uuid.uuid4().hex)
    n_gpus = _count_gpus()
    backend = 'nccl' if (n_gpus >= n_jobs and 'CTWS_DEVICE' not in os.environ) else 'gloo'
    backend = os.environ.get('CTWS_JOB_DIST_BACKEND', backend)
    return {'n_jobs': n_jobs, 'rendezvous': 'file://' + store, 'backend': backend, 'tmp_folder': tmp_folder}


def relabel_job_config(task, n_jobs):
    """The in-job relabel of the local jobs: their process group and the assignment table."""
    return dict(job_group_config(task.tmp_folder, n_jobs), assignment_path=task.assignment_path,
                assignment_key=task.assignment_key)


def block_uniques_file(folder, block_id):
    return os.path.join(folder, 'block_%i.npy' % block_id)


class WatershedLocal(WatershedBase, LocalTask):
    """Watershed on the local machine (one GPU handle per job process)."""


class WatershedSlurm(WatershedBase, SlurmTask):
    """Watershed on a slurm cluster."""


class WatershedLSF(WatershedBase, LSFTask):
    """Watershed on an lsf cluster."""


#
# Implementation
#

def _get_bbs(blocking, block_id, config):
    """(input_bb, inner_bb, output_bb) as watershed.py:252-264."""
    halo = list(config.get('halo', [0, 0, 0]))
    if sum(halo) > 0:
        block = blocking.getBlockWithHalo(block_id, halo)
        input_bb = vu.block_to_bb(block.outerBlock)
        output_bb = vu.block_to_bb(block.innerBlock)
        inner_bb = vu.block_to_bb(block.innerBlockLocal)
    else:
        block = blocking.getBlock(block_id)
        input_bb = output_bb = vu.block_to_bb(block)
        inner_bb = tuple(slice(0, b.stop - b.start) for b in input_bb)
    return input_bb, inner_bb, output_bb


def _read_block(blocking, block_id, ds_in, ds_out, mask, config, pass_id, read_input=True):
    """Everything `_ws_block` reads for one block (watershed.py:287-303), as a libctws block
    (read_input=False: the input's index in 'input_index' instead, for a batched read)."""
    input_bb, inner_bb, output_bb = _get_bbs(blocking, block_id, config)
    b = {'block_id': block_id, 'output_bb': output_bb, 'crop_relabel': output_bb != input_bb,
         'inner_begin': [s.start for s in inner_bb], 'inner_shape': [s.stop - s.start for s in inner_bb]}
    if mask is not None:
        in_mask = np.asarray(mask[input_bb]).astype('bool')
        if in_mask[inner_bb].sum() == 0:
            b['skip'] = True  # watershed.py:295-297: nothing to do, nothing written
            return b
        b['mask'] = in_mask.view('uint8')
    if ds_in.ndim == 4:
        cb, ce = config.get('channel_begin', 0), config.get('channel_end', None)
        index = (slice(cb, ce),) + input_bb
    else:
        index = input_bb
    if read_input:
        b['input'] = ds_in[index]
    else:
        b['input_index'] = index
    if pass_id == 1:
        b['initial_seeds'] = ds_out[input_bb]
    return b


def _device():
    return int(os.environ.get('CTWS_DEVICE', os.environ.get('LOCAL_RANK', '0')))


def _overlaps(a, b):
    return all(sa.start < sb.stop and sb.start < sa.stop for sa, sb in zip(a, b))


def pass2_levels(bbs):
    """Dependency levels of pass-2 blocks in list order: a sequential-equivalent schedule.

    `bbs` = [(input_bb, output_bb)] in block-list order.  In the reference's sequential loop
    (two_pass_watershed.py:296-299) block y reads ds_out[input_bb] after every earlier block
    wrote and before every later one writes; same-colour checkerboard blocks interact only where
    a diagonal neighbour's inner block lies in the other's halo.  level(y) = 1 + max level of
    the earlier blocks that overlap y (either way round), 0 without one.  Blocks of one level
    never overlap; running the levels in order, each level's blocks reading before any of them
    writes, gives every block exactly the ds_out the sequential loop gives it."""
    levels = []
    for j, (in_j, out_j) in enumerate(bbs):
        lv = 0
        for i in range(j):
            in_i, out_i = bbs[i]
            if levels[i] + 1 > lv and (_overlaps(in_j, out_i) or _overlaps(in_i, out_j)):
                lv = levels[i] + 1
        levels.append(lv)
    return levels


def make_batches(blocking, block_list, config, pass_id, batch_blocks):
    """Split the job's block list (in order) into GPU batches.

    Pass 0 reads only ds_in, so any split works.  Pass 1 (`_ws_pass2`) reads ds_out[input_bb]:
    the batches follow pass2_levels (every batch holds blocks of one level, levels in order),
    the schedule that reproduces the reference's sequential loop.
    """
    if pass_id == 1:
        levels = pass2_levels([_get_bbs(blocking, bid, config)[0::2] for bid in block_list])
        batches = []
        for lv in range(max(levels) + 1 if levels else 0):
            ids = [bid for bid, l in zip(block_list, levels) if l == lv]
            batches += [ids[k:k + batch_blocks] for k in range(0, len(ids), batch_blocks)]
        return batches
    return [list(block_list[k:k + batch_blocks]) for k in range(0, len(block_list), batch_blocks)]


def run_blocks(blocking, block_list, ds_in, ds_out, mask, config, pass_id=0, batch_blocks=None, keep=None,
               started=None):
    """Run `_ws_block` (pass 0) or `_ws_pass2` (pass 1) for `block_list` on the GPU.

    Blocks are processed in batches with the same results as the reference's sequential loop:
    pass 0 in block-list order; pass 1 by the dependency levels of pass2_levels, which give
    every block the ds_out it reads in the sequential loop.  Outputs are written and "processed
    block" is logged batch by batch; a block the kernels cannot finish (status
    CTWS_BLOCK_FAILED, e.g. the reference's own takeDict failure) raises after the batches
    before it are written, as the reference job raises at that block (pass 1: blocks of earlier
    levels may lie after it in the list).

    keep (a list; pass 0): nothing is written -- each block's (block_id, output_bb, labels or None
    for a skipped block, uniques) is appended instead, for the in-job relabel (job_relabel.py).
    The labels then stay in HBM (torch tensors) when the job's outputs fit in half the free
    device memory (config 'keep_on_device', default on): the relabel maps them there and each
    block crosses PCIe once, with its final ids.

    started: called once the first batch's read is under way (the in-job relabel's process
    group starts there, so that torch's import overlaps the read).
    """
    from cluster_tools_amd import ctws
    block_shape = list(config['block_shape'])
    lib_config = dict(config)
    if ds_in.ndim == 4:
        # the host already sliced the channel range
        lib_config['channel_begin'], lib_config['channel_end'] = 0, None
    if config.get('non_maximum_suppression', True if pass_id == 1 else False):
        fu.log("non-maximum suppression was activated, but is not available")
    # keep (in-job relabel): small batches, so that the GPU runs a batch while the next is read
    batch_blocks = batch_blocks or int(config.get('gpu_batch_blocks') or (4 if keep is not None else 16))
    batches = make_batches(blocking, block_list, config, pass_id, batch_blocks)
    # chunk inflate / deflate on a pool of the job's threads_per_job (not more)
    ds_in.n_threads = ds_out.n_threads = max(1, int(config.get('threads_per_job', 1)))
    if hasattr(ds_in, 'cache_bytes'):
        # inflate each input chunk once for the job's blocks with halos (n5 / zarr reader)
        ds_in.cache_bytes = int(float(config.get('read_cache_gb', 2.0)) * (1 << 30))

    def read_batch(ids):
        batched = hasattr(ds_in, 'read_many')
        blocks = [_read_block(blocking, bid, ds_in, ds_out, mask, config, pass_id, read_input=not batched)
                  for bid in ids]
        if batched:
            need = [b for b in blocks if 'input_index' in b]
            for b, x in zip(need, ds_in.read_many([b.pop('input_index') for b in need])):
                b['input'] = x
        return blocks

    uniques_path = config.get('uniques_path')

    def write_batch(blocks, results, error, uniques):
        for b, r, u in zip(blocks, results, uniques):
            if r is not None and r['status'] == ctws.CTWS_BLOCK_FAILED:
                raise ctws.CtwsError("block %i: %s" % (b['block_id'], error))
            if keep is not None:
                written = r is not None and r['status'] in (0, 2)
                keep.append((b['block_id'], b['output_bb'], r['output'] if written else None, u if written else None))
                continue
            if r is not None and r['status'] in (0, 2):   # written / empty block: constant offset
                ds_out[b['output_bb']] = r['output']
            if u is not None:
                # after the block's data: a file never describes labels that are not written.
                # A block that writes nothing gets no file (FindUniques reads what it holds).
                np.save(block_uniques_file(uniques_path, b['block_id']), u)
            fu.log_block_success(b['block_id'])

    with futures.ThreadPoolExecutor(2) as io, contextlib.ExitStack() as stack:
        # the first read overlaps the HIP (and torch) start-up
        nxt = io.submit(read_batch, batches[0]) if batches else None
        if started is not None:
            started()
        h = stack.enter_context(ctws.Handle(_device()))
        on_device = keep is not None and _keep_on_device(blocking, block_list, config)
        pending_write = None
        for bi in range(len(batches)):
            blocks = nxt.result()
            if pass_id == 0:
                # inputs never depend on outputs: read the next batch while this one runs
                nxt = io.submit(read_batch, batches[bi + 1]) if bi + 1 < len(batches) else None
            for b in blocks:
                fu.log("start processing block %i" % b['block_id'])
            _test_fail_once(blocks)
            todo = [b for b in blocks if not b.get('skip')]
            if not todo:
                res = []
            elif on_device:
                res = _ws_blocks_resident(h, lib_config, block_shape, todo)
            else:
                res = h.ws_blocks(lib_config, block_shape, todo, pass_id=pass_id)
            error = h.last_error()
            by_id = {b['block_id']: r for b, r in zip(todo, res)}
            results = [by_id.get(b['block_id']) for b in blocks]
            uniq = h.unique_u64_device if on_device else h.unique_u64
            uniques = [uniq(r['output']) if (uniques_path or keep is not None) and r is not None
                       and r['status'] in (0, 2) else None for r in results]
            if pending_write is not None:
                pending_write.result()
            pending_write = io.submit(write_batch, blocks, results, error, uniques)
            if pass_id == 1:
                # the next batch's halos may hold this batch's outputs: read after the write
                pending_write.result()
                pending_write = None
                nxt = io.submit(read_batch, batches[bi + 1]) if bi + 1 < len(batches) else None
        if pending_write is not None:
            pending_write.result()


def _test_fail_once(blocks):
    """Test hook of the retry test (tests/test_workflow_gpu.py, as the reference's
    test/retry/failing_task.py): with CTWS_TEST_FAIL_ONCE=<folder>, the first attempt at a block
    with id % 4 == 1 raises (a marker file in the folder records it), the retry succeeds."""
    folder = os.environ.get('CTWS_TEST_FAIL_ONCE')
    if not folder:
        return
    fail = []
    for b in blocks:
        marker = os.path.join(folder, 'failed_block_%i' % b['block_id'])
        if b['block_id'] % 4 == 1 and not os.path.exists(marker):
            open(marker, 'w').close()
            fail.append(b['block_id'])
    if fail:
        raise RuntimeError("injected failure of blocks %s (CTWS_TEST_FAIL_ONCE)" % fail)


def _keep_on_device(blocking, block_list, config):
    """Whether the job's uint64 outputs fit in its share of half the free memory of its GPU
    (the jobs of the task that share the GPU -- job_id % n_gpus -- decide at the same time)."""
    if not config.get('keep_on_device', True):
        return False
    import torch
    need = 0
    for bid in block_list:
        _, inner_bb, _ = _get_bbs(blocking, bid, config)
        need += 8 * int(np.prod([s.stop - s.start for s in inner_bb]))
    n_jobs = int((config.get('relabel') or {}).get('n_jobs', 1))
    share = max(1, -(-n_jobs // max(1, torch.cuda.device_count())))
    free, _ = torch.cuda.mem_get_info(_device())
    return need <= free // (2 * share)


def _ws_blocks_resident(h, lib_config, block_shape, todo):
    """Pass-0 blocks through ctws_ws_blocks_device: the inputs uploaded, the outputs left in HBM
    as int64 tensors (uint64 bits) -> [{'output': tensor, 'status', 'max_label', 'n_ids'}]."""
    import torch
    dev = torch.device('cuda', _device())
    dblocks = []
    for b in todo:
        db = {'block_id': b['block_id'], 'inner_begin': b['inner_begin'], 'crop_relabel': b['crop_relabel'],
              'input': torch.from_numpy(np.ascontiguousarray(b['input'])).to(dev),
              'output': torch.empty(tuple(b['inner_shape']), dtype=torch.int64, device=dev)}
        if b.get('mask') is not None:
            db['mask'] = torch.from_numpy(np.ascontiguousarray(b['mask'], dtype=np.uint8)).to(dev)
        dblocks.append(db)
    st = h.ws_blocks_device(lib_config, block_shape, dblocks, pass_id=0)
    return [{'output': db['output'], 'status': s, 'max_label': m, 'n_ids': n} for db, (s, m, n) in zip(dblocks, st)]


def run_job(job_id, config_path, pass_id=None):
    """Job entry shared by the watershed tasks: the job's blocks through run_blocks, pass 0
    (`_ws_block`) unless the config's 'pass' says 1 (`_ws_pass2`)."""
    fu.log("start processing job %i" % job_id)
    fu.log("reading config from %s" % config_path)
    with open(config_path) as f:
        config = json.load(f)
    pass_id = config.get('pass', 0) if pass_id is None else pass_id
    shape = list(vu.get_shape(config['input_path'], config['input_key']))[-3:]
    blocking = Blocking([0, 0, 0], shape, list(config['block_shape']))
    rel = config.get('relabel') if pass_id == 0 else None
    with vu.file_reader(config['input_path'], 'r') as fi, vu.file_reader(config['output_path']) as fo:
        ds_in, ds_out = fi[config['input_key']], fo[config['output_key']]
        assert ds_in.ndim in (3, 4) and ds_out.ndim == 3, (ds_in.ndim, ds_out.ndim)
        mask = vu.load_mask(config['mask_path'], config['mask_key'], shape) if 'mask_path' in config else None
        if rel is None:
            run_blocks(blocking, config['block_list'], ds_in, ds_out, mask, config, pass_id=pass_id)
        else:
            _run_blocks_relabel(job_id, blocking, ds_in, ds_out, mask, config, rel)
    fu.log_job_success(job_id)


def _run_blocks_relabel(job_id, blocking, ds_in, ds_out, mask, config, rel):
    """The job's blocks, then the in-job relabel over the jobs' process group (job_relabel.py):
    the job writes its blocks with the final ids; job 0 writes the assignment table and maxId."""
    from cluster_tools_amd import ctws
    from cluster_tools_amd.watershed import job_relabel
    # the group as soon as the first read is under way: all jobs start together, so the
    # rendezvous is immediate; a job that dies later breaks its peers' pending collective (gloo /
    # RCCL report the lost peer) instead of leaving them waiting out the timeout
    group, init_err = [], []

    def start_group():
        try:
            job_relabel.init_group(job_id, rel['n_jobs'], rel['rendezvous'], rel['backend'], device=_device())
        except Exception as e:  # recorded: a second rendezvous would only wait out the timeout again
            init_err.append(e)
            raise
        group.append(True)

    keep, failed = [], None
    try:
        try:
            run_blocks(blocking, config['block_list'], ds_in, ds_out, mask, config, pass_id=0, keep=keep,
                       started=start_group)
        except Exception as e:  # still take part in the exchange: every job then raises
            import traceback
            traceback.print_exc()
            failed = e
        if init_err:
            raise init_err[0]
        if not group:   # (run_blocks failed before its first read)
            start_group()
        if failed is None:
            with ctws.Handle(_device()) as h:
                def mapper(lab, keys, vals):
                    if hasattr(lab, 'data_ptr'):   # resident in HBM: map there, then download
                        if len(keys):
                            h.lookup_u64_device(lab, keys, vals)
                        return lab.cpu().numpy().view(np.uint64)
                    if len(keys):
                        h.lookup_u64(lab, keys, vals)
                    return lab
                job_relabel.relabel_in_job(job_id, keep, ds_out, rel['tmp_folder'], rel['assignment_path'],
                                           rel['assignment_key'], mapper, log=fu.log, device=_device())
        else:
            job_relabel.relabel_in_job(job_id, [], ds_out, rel['tmp_folder'], rel['assignment_path'],
                                       rel['assignment_key'], None, failed=True, log=fu.log, device=_device())
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
    if failed is not None:
        raise failed


def watershed(job_id, config_path):
    run_job(job_id, config_path, pass_id=0)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    watershed(job_id, path)
