"""RelabelWorkflow fused into the watershed jobs: the per-block id-count exchange over a process
group of the jobs (BASELINE north star: "the per-block max-label exclusive scan
that assigns global ID offsets").

The reference numbers the watershed ids with three more tasks and two file round trips:
FindUniques (per-job np.unique, relabel/find_uniques.py:115-159), FindLabeling (np.unique of
the concatenation, new ids consecutive from 1, 0 kept as 0 if present; find_labeling.py:84-126)
and Write (every block through the table, attrs['maxId']; write/write.py:153-278).  Watershed
ids of block b lie in [b * V, (b + 1) * V] (V = prod(block_shape), watershed.py:305-307), so
the sorted global uniques are the blocks' sorted uniques in block-id order, and the new id of
the k-th nonzero unique of block b is offsets[b] + 1 + k with offsets the exclusive scan of the
blocks' nonzero-unique counts (thresholded_components/merge_offsets.py:106-122 does the same
scan with files).  The one overlap the id ranges allow -- block b - 1's id b * V (a local label
equal to V) and block b's bare offset b * V -- is detected from the blocks' first / last
nonzero uniques and counted once, as np.unique would.

Here the local jobs of one watershed task (all started at once by LocalTask) form one process
group (rank = job id; RCCL when every job owns a GPU, gloo when jobs share one), all-gather one
row per block (block id, nonzero count, first, last, has zero), scan, and write their blocks
with the final ids -- the relabelled volume, the (N, 2) assignment table and maxId equal the
three-task RelabelWorkflow's exactly (tests/test_job_relabel.py, tests/test_workflow_gpu.py).
The table rows go through files (rank 0 writes the dataset), the scan through the group.
"""
import os
from datetime import timedelta

import numpy as np


def block_row(block_id, uniques):
    """(block id, nonzero count, first nonzero, last nonzero, has 0) of one block's sorted uniques."""
    u = np.asarray(uniques, dtype=np.uint64)
    nz = u[u != 0]
    first = int(nz[0]) if len(nz) else -1
    last = int(nz[-1]) if len(nz) else -1
    return [int(block_id), len(nz), first, last, int(len(nz) != len(u))]


def scan(rows):
    """Offsets of every block from the rows of all blocks (any order).

    Returns {block_id: (offset, dup)} and the number of new nonzero ids: block b's k-th nonzero
    unique gets offset + 1 + k - dup, where dup = 1 when its first unique is the previous
    block's last one (that id keeps the previous block's new id)."""
    rows = sorted((tuple(int(v) for v in r) for r in rows), key=lambda r: r[0])
    out, total, prev_last, prev_id = {}, 0, None, None
    for bid, cnt, first, last, _ in rows:
        dup = 1 if (cnt and prev_last is not None and prev_id == bid - 1 and first == prev_last) else 0
        out[bid] = (total, dup)
        total += cnt - dup
        if cnt:
            prev_last, prev_id = last, bid
        else:
            prev_last, prev_id = None, bid
    return out, total


def block_table(uniques, offset, dup):
    """(keys, values) of one block: its nonzero uniques -> offset + 1 + k - dup."""
    u = np.asarray(uniques, dtype=np.uint64)
    nz = u[u != 0]
    vals = np.arange(offset + 1 - dup, offset + 1 - dup + len(nz), dtype=np.uint64)
    return nz, vals


def write_blocks(ds_out, written, log, n_threads=None):
    """ds_out[bb] = labels for every (block_id, bb, labels) of the iterable `written`: the chunks
    of all blocks through one pool (a block's chunks alone are too few to keep the job's threads
    busy), each block submitted as soon as the iterable yields it; "processed block" after each
    block's last chunk, in block order."""
    from concurrent import futures
    n_threads = n_threads or max(4, getattr(ds_out, 'n_threads', 1))
    single = getattr(ds_out, 'n_threads', 1)
    ds_out.n_threads = 1
    try:
        with futures.ThreadPoolExecutor(n_threads) as pool:
            futs = [(bid, pool.submit(ds_out.__setitem__, bb, lab)) for bid, bb, lab in written]
            for bid, f in futs:
                f.result()
                log("processed block %i" % bid)  # (the reference's line: after the block's write)
    finally:
        ds_out.n_threads = single


def rows_file(tmp_folder, job_id):
    return os.path.join(tmp_folder, 'watershed_relabel_rows_job_%i.npy' % job_id)


def _gather_rows(rows, device):
    """All ranks' rows (k x 5 int64 each, k may differ per rank), concatenated."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    local = torch.as_tensor(np.asarray(rows, dtype=np.int64).reshape(-1, 5), device=device)
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    m = max(max(sizes), 1)
    padded = torch.zeros((m, 5), dtype=torch.int64, device=device)
    padded[:local.shape[0]] = local
    parts = [torch.zeros_like(padded) for _ in range(world)]
    dist.all_gather(parts, padded)
    return np.concatenate([p[:s].cpu().numpy() for p, s in zip(parts, sizes)])


def _agree(err, device, what):
    """Every rank learns whether any rank failed in the phase just ended (an all-reduce of a
    success flag instead of a bare barrier): a job that raised while writing would otherwise
    leave its peers waiting in the barrier until the group's timeout.  Re-raises the local
    error, or raises for a peer's."""
    import torch
    import torch.distributed as dist
    ok = torch.tensor([0 if err is not None else 1], dtype=torch.int32, device=device)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if err is not None:
        raise err
    if int(ok.item()) == 0:
        raise RuntimeError("a watershed job of the group failed while %s" % what)


def init_group(job_id, n_jobs, rendezvous, backend, device=None, timeout_s=900):
    """rendezvous: a TCP port on 127.0.0.1 (int) or an init_method URL such as the file store
    the watershed task hands its jobs (no port chosen ahead of the jobs that another process
    could take in between)."""
    import torch.distributed as dist
    init = rendezvous if isinstance(rendezvous, str) else 'tcp://127.0.0.1:%d' % rendezvous
    kw = dict(init_method=init, rank=job_id, world_size=n_jobs, timeout=timedelta(seconds=timeout_s))
    if backend == 'nccl':
        import torch
        torch.cuda.set_device(device)
        dist.init_process_group('nccl', device_id=torch.device('cuda', device), **kw)
    else:
        dist.init_process_group('gloo', **kw)


def relabel_in_job(job_id, results, ds_out, tmp_folder, assignment_path, assignment_key, mapper,
                   failed=False, log=print, device=None):
    """The exchange, then the job's blocks written with their final ids.

    results: [(block_id, output_bb, labels or None (skipped: nothing written), uniques)] of this
    job; labels may be a numpy array or a tensor resident on the GPU.  mapper(labels, keys,
    values) returns the block with its final ids as a numpy uint64 array (ctws lookup on the GPU;
    an empty table leaves the labels as they are).  A job whose blocks failed still joins
    (failed=True) so that every job raises instead of waiting."""
    import torch.distributed as dist
    from cluster_tools_amd.utils import volume_utils as vu
    comm_dev = device if dist.get_backend() == 'nccl' else None
    rows = [block_row(bid, u) for bid, _, lab, u in results if lab is not None]
    skipped = any(lab is None for _, _, lab, _ in results)
    status = _gather_rows([[-1, int(failed), 0, 0, int(skipped)]] + rows, comm_dev)
    flags, rows_all = status[status[:, 0] < 0], status[status[:, 0] >= 0]
    if flags[:, 1].any():
        raise RuntimeError("a watershed job of the group failed: no relabelling")
    offs, n_new = scan(rows_all)
    has_zero = bool(flags[:, 4].any() or rows_all[:, 4].any())
    log("global ids: %i (offset scan over %i blocks)" % (n_new, len(rows_all)))
    # map the blocks one by one (GPU lookup) while the chunk writers compress the ones before
    tables = {}

    def mapped():
        for bid, bb, lab, u in results:
            if lab is None:
                continue
            off, dup = offs[bid]
            keys, vals = block_table(u, off, dup)
            # (a duplicated first id keeps the previous block's row in the table)
            tables[bid] = (keys[dup:], vals[dup:])
            yield bid, bb, mapper(lab, keys, vals)

    err = None
    try:
        write_blocks(ds_out, mapped(), log)
        # this job's table rows in block order, with each block's row count
        bids = sorted(tables)
        np.save(rows_file(tmp_folder, job_id), np.stack([
            np.concatenate([tables[b][0] for b in bids]) if bids else np.zeros(0, np.uint64),
            np.concatenate([tables[b][1] for b in bids]) if bids else np.zeros(0, np.uint64)], axis=1))
        np.save(rows_file(tmp_folder, job_id) + '.blocks.npy',
                np.array([[b, len(tables[b][0])] for b in bids], np.int64).reshape(-1, 2))
    except Exception as e:  # noqa: BLE001 -- re-raised after the peers have been told
        err = e
    _agree(err, comm_dev, 'writing its blocks')
    err = None
    if job_id == 0:
        try:
            # the assignment table as FindLabeling writes it (rows sorted by old id = block order),
            # assembled from the jobs' per-block row runs without a sort, and Write's maxId
            runs = []
            for j in range(dist.get_world_size()):
                rows = np.load(rows_file(tmp_folder, j))
                blocks = np.load(rows_file(tmp_folder, j) + '.blocks.npy')
                start = 0
                for b, n in blocks:
                    runs.append((int(b), rows[start:start + n]))
                    start += n
            runs.sort(key=lambda r: r[0])
            table = np.concatenate([r for _, r in runs]) if runs else np.zeros((0, 2), np.uint64)
            if has_zero:
                table = np.concatenate([np.zeros((1, 2), np.uint64), table])
            table = np.ascontiguousarray(table, dtype=np.uint64)
            with vu.file_reader(assignment_path) as f:
                if assignment_key in f:
                    del f[assignment_key]
                ds = f.create_dataset(assignment_key, shape=table.shape, dtype='uint64', compression='gzip',
                                      chunks=(max(1, min(1000000, len(table))), 2))
                ds.n_threads = 8
                ds[:] = table
            ds_out.attrs['maxId'] = int(table[:, 1].max()) if len(table) else 0
            for j in range(dist.get_world_size()):
                os.remove(rows_file(tmp_folder, j))
                os.remove(rows_file(tmp_folder, j) + '.blocks.npy')
        except Exception as e:  # noqa: BLE001
            err = e
    _agree(err, comm_dev, 'writing the assignment table')
    return n_new
