"""ThresholdedComponentsWorkflow's merge tail folded into the BlockComponents jobs.

The reference merges the per-block components with four more tasks, each a round of job
processes and file round trips (thresholded_components_workflow.py:54-88):
  MergeOffsets      exclusive scan of the per-block `max + 1` counts   (merge_offsets.py:83-131)
  BlockFaces        unique (a + off_a, b + off_b) label pairs across every block's upper faces,
                    np.unique per block and per job                    (block_faces.py:87-177)
  MergeAssignments  np.unique of all jobs' pairs, nifty boost_ufd merge in that order, find
                    (merge_assignments.py:88-141)
  Write             every block through the assignments, with its offset (write.py:178-211)
Here the local BlockComponents jobs of one task form a process group (rank = job id, the same
rendezvous as the watershed's in-job relabel, watershed/job_relabel.py): they keep their blocks'
labels, all-gather the counts and scan them, take the face pairs from the labels they hold (a
face whose upper block another job owns reads that job's plane from tmp_folder), job 0 merges
the pairs with ctws_ufd_find and writes the assignment dataset and cc_offsets.json, and every
job writes its blocks with their final ids.  The result -- segmentation, assignment table,
offsets file, maxId -- is the five-task chain's (tests/test_threshcc.py, tests/test_threshcc_gpu.py).

Two reference behaviours are kept on purpose: only axial face neighbours pair, and when one of
BlockFaces' jobs finds no pair at all the merge is the identity (merge_assignments.py:116-123:
`if all(ass.size for ass in assignments)`), which depends on BlockFaces' round-robin partition of
the block list -- so that partition (min(n_blocks, max_jobs) jobs, block_list[j::n]) is what the
check uses, whatever the BlockComponents jobs' partition was.
"""
import json
import os

import numpy as np

from cluster_tools_amd.thresholded_components.merge_offsets import scan_block_counts


class SpilledBlock:
    """A block's labels written to ds_out as they are (uint64) instead of kept in host memory
    (block_components.spill_labels); the merge reads its face planes and, for the final write,
    the whole block back."""

    def __init__(self, ds, bb):
        self.ds, self.bb = ds, tuple(bb)

    def plane(self, axis, index):
        bb = list(self.bb)
        bb[axis] = slice(self.bb[axis].start + index, self.bb[axis].start + index + 1)
        return np.ascontiguousarray(np.asarray(self.ds[tuple(bb)]).squeeze(axis))

    def extent(self, axis):
        return self.bb[axis].stop - self.bb[axis].start

    def read(self):
        return np.asarray(self.ds[self.bb])


def lower_plane(labels, axis):
    """The block's first plane along `axis` (the face its lower neighbour pairs with)."""
    return np.ascontiguousarray(np.take(labels, 0, axis=axis))


def upper_plane(labels, axis):
    return np.ascontiguousarray(np.take(labels, labels.shape[axis] - 1, axis=axis))


def face_pairs(plane_a, plane_b, off_a, off_b):
    """`_process_face` (block_faces.py:87-113): both labels nonzero, offsets added, unique rows."""
    a = plane_a.ravel().astype('uint64')
    b = plane_b.ravel().astype('uint64')
    have = (a != 0) & (b != 0)
    if not have.any():
        return None
    return np.unique(np.stack([a[have] + np.uint64(off_a), b[have] + np.uint64(off_b)], axis=1), axis=0)


def faces_partition(block_list, max_jobs):
    """BlockFaces' job lists: n = min(n_blocks, max_jobs) jobs, block_list[j::n] (the reference's
    LocalTask split, cluster_tasks.py:328)."""
    n = max(1, min(len(block_list), max_jobs))
    return [block_list[j::n] for j in range(n)]


def merge_pairs(block_pairs, block_list, max_jobs):
    """MergeAssignments' pair set: {block_id: pairs or None} -> the (N, 2) uint64 rows merged in
    order, or an empty array when any BlockFaces job of the reference partition has no pair."""
    parts = []
    for blocks in faces_partition(block_list, max_jobs):
        ps = [block_pairs[b] for b in blocks if block_pairs.get(b) is not None]
        parts.append(np.unique(np.concatenate(ps, axis=0), axis=0) if ps else np.zeros((0, 2), 'uint64'))
    if not parts or not all(p.size for p in parts):
        return np.zeros((0, 2), dtype='uint64')
    return np.unique(np.concatenate(parts, axis=0), axis=0)


def _plane_file(tmp_folder, block_id, axis):
    return os.path.join(tmp_folder, 'cc_face_%i_%i.npy' % (block_id, axis))


def _pairs_file(tmp_folder, job_id):
    return os.path.join(tmp_folder, 'cc_block_pairs_job_%i.npz' % job_id)


def _assignments_file(tmp_folder):
    return os.path.join(tmp_folder, 'cc_assignments_merged.npy')


def _gather_counts(rows, device):
    """All ranks' (block id, count, failed) rows, concatenated."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    local = torch.as_tensor(np.asarray(rows, dtype=np.int64).reshape(-1, 3), device=device)
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    padded = torch.zeros((max(max(sizes), 1), 3), dtype=torch.int64, device=device)
    padded[:local.shape[0]] = local
    parts = [torch.zeros_like(padded) for _ in range(world)]
    dist.all_gather(parts, padded)
    return np.concatenate([p[:s].cpu().numpy() for p, s in zip(parts, sizes)])


def merge_in_job(job_id, results, blocking, block_list, owner, config, ds_out, log=print, device=None,
                 failed=False, to_numpy=None):
    """The exchange and the final write of one BlockComponents job.

    results: [(block_id, bb, labels or None, count)] of this job (count = the reference's
    `max + 1`, 0 for an empty block; labels numpy or an on-device tensor, None when empty);
    block_list: every block of the task; owner: {block_id: job id}; config: the job config
    (tmp_folder, offsets_path, output_path, assignment_key, faces_max_jobs).  A job whose blocks
    failed joins with failed=True so that every job raises instead of waiting."""
    import torch.distributed as dist
    from cluster_tools_amd import ctws
    from cluster_tools_amd.utils import volume_utils as vu
    from cluster_tools_amd.watershed.job_relabel import _agree
    to_numpy = to_numpy or (lambda a: a if isinstance(a, np.ndarray) else
                            a.read() if isinstance(a, SpilledBlock) else a.cpu().numpy())
    comm_dev = device if dist.get_backend() == 'nccl' else None
    tmp = config['tmp_folder']
    try:
        return _merge(job_id, results, blocking, block_list, owner, config, ds_out, log, device, failed, to_numpy,
                      dist, ctws, vu, _agree, comm_dev, tmp)
    finally:
        # job 0 removes the run's files whether the merge ended or failed (every job leaves the
        # merge at the same _agree, so no peer reads them any more)
        if job_id == 0:
            _remove_run_files(tmp, dist.get_world_size(), block_list)


def _remove_run_files(tmp, world, block_list):
    paths = [_pairs_file(tmp, j) for j in range(world)] + [_assignments_file(tmp)]
    paths += [_plane_file(tmp, bid, axis) for bid in block_list for axis in range(3)]
    for p in paths:
        if os.path.exists(p):
            os.remove(p)


def _merge(job_id, results, blocking, block_list, owner, config, ds_out, log, device, failed, to_numpy,
           dist, ctws, vu, _agree, comm_dev, tmp):
    rows = [[-1, 0, int(failed)]] + [[bid, int(cnt), 0] for bid, _, _, cnt in results]
    allr = _gather_counts(rows, comm_dev)
    if allr[:, 2].any():
        raise RuntimeError("a block components job of the group failed: no merge")
    counts = {int(b): int(c) for b, c, _ in allr if b >= 0}
    assert len(counts) == len(block_list), (len(counts), len(block_list))
    offs, empty_pos, n_labels = scan_block_counts(counts)
    ids = sorted(counts)
    offsets = {b: offs[k] for k, b in enumerate(ids)}
    empty = {ids[k] for k in empty_pos}
    log("merging offsets for %i blocks: %i labels, %i empty blocks" % (len(ids), n_labels, len(empty)))
    mine = {bid: lab for bid, _, lab, _ in results}
    err = None
    try:
        # the lower planes an other job's block pairs with (its upper face meets this block)
        for bid, _, lab, _ in results:
            if bid in empty:
                continue
            for axis in range(3):
                lo = blocking.getNeighborId(bid, axis, True)
                if lo != -1 and lo in counts and owner[lo] != job_id:
                    np.save(_plane_file(tmp, bid, axis), to_numpy(lower_plane_any(lab, axis)))
    except Exception as e:  # noqa: BLE001 -- re-raised after the peers have been told
        err = e
    _agree(err, comm_dev, 'writing its face planes')
    err = None
    try:
        # BlockFaces (block_faces.py:116-177): each block with its upper neighbours
        pairs = {}
        for bid, _, lab, _ in results:
            if bid in empty:
                continue
            ps = []
            for axis in range(3):
                up = blocking.getNeighborId(bid, axis, False)
                if up == -1 or up in empty or up not in counts:
                    continue
                pb = (to_numpy(lower_plane_any(mine[up], axis)) if owner[up] == job_id
                      else np.load(_plane_file(tmp, up, axis)))
                p = face_pairs(to_numpy(upper_plane_any(lab, axis)), pb, offsets[bid], offsets[up])
                if p is not None:
                    ps.append(p)
            if ps:
                pairs[bid] = np.unique(np.concatenate(ps, axis=0), axis=0)
        np.savez(_pairs_file(tmp, job_id), ids=np.array(sorted(pairs), np.int64),
                 **{'b%i' % b: p for b, p in pairs.items()})
    except Exception as e:  # noqa: BLE001
        err = e
    _agree(err, comm_dev, 'collecting its face pairs')
    err = None
    if job_id == 0:
        try:
            allp = {}
            for j in range(dist.get_world_size()):
                with np.load(_pairs_file(tmp, j)) as z:
                    for b in z['ids'].tolist():
                        allp[int(b)] = z['b%i' % b]
            merged = merge_pairs(allp, list(block_list), int(config.get('faces_max_jobs', 1)))
            if len(merged):
                assert int(merged.max()) + 1 <= n_labels, "%i, %i" % (int(merged.max()) + 1, n_labels)
                log("have %i pairs of node assignments" % len(merged))
            else:
                log("did not find any node assignments, label assignment will be identity")
            assignments = ctws.ufd_find(n_labels, merged)
            log("reducing the number of labels from %i to %i" % (n_labels, len(np.unique(assignments))))
            with vu.file_reader(config['output_path']) as f:
                if config['assignment_key'] in f:
                    del f[config['assignment_key']]
                ds = f.create_dataset(config['assignment_key'], shape=assignments.shape, dtype='uint64',
                                      compression='gzip', chunks=(min(65334, n_labels),))
                ds[:] = assignments
            np.save(_assignments_file(tmp), assignments)
            # MergeOffsets' file (merge_offsets.py:124-130), for the tasks that read it
            with open(config['offsets_path'], 'w') as f:
                json.dump({'offsets': offs, 'empty_blocks': empty_pos, 'n_labels': n_labels}, f)
        except Exception as e:  # noqa: BLE001
            err = e
    _agree(err, comm_dev, 'merging the assignments')
    err = None
    try:
        from cluster_tools_amd.watershed.job_relabel import write_blocks
        assignments = np.load(_assignments_file(tmp))
        for bid, _, _, _ in results:
            if bid in empty:
                log("processed block %i" % bid)

        def final_ids():
            # Write (write.py:178-211): nonzero label l of the block -> assignments[l + offset],
            # as one table lookup per voxel (the block's labels are 0..count-1)
            for bid, bb, lab, cnt in results:
                if bid in empty:
                    continue
                lut = np.zeros(cnt, dtype='uint64')
                lut[1:] = assignments[offsets[bid] + 1:offsets[bid] + cnt]
                lab = to_numpy(lab)
                yield bid, bb, np.take(lut, lab.view('int64') if lab.dtype == np.uint64 else lab)

        # the chunks of all blocks through one pool, each block submitted once its ids are there
        write_blocks(ds_out, final_ids(), log)
        if job_id == 0:
            ds_out.attrs['maxId'] = int(assignments.max()) if len(assignments) else 0
    except Exception as e:  # noqa: BLE001
        err = e
    _agree(err, comm_dev, 'writing its blocks')
    return n_labels


def lower_plane_any(lab, axis):
    """lower_plane on a numpy array, a spilled block (one plane read back) or a torch tensor
    (the plane only crosses PCIe)."""
    if isinstance(lab, np.ndarray):
        return lower_plane(lab, axis)
    if isinstance(lab, SpilledBlock):
        return lab.plane(axis, 0)
    return lab.select(axis, 0).contiguous()


def upper_plane_any(lab, axis):
    if isinstance(lab, np.ndarray):
        return upper_plane(lab, axis)
    if isinstance(lab, SpilledBlock):
        return lab.plane(axis, lab.extent(axis) - 1)
    return lab.select(axis, lab.shape[axis] - 1).contiguous()
