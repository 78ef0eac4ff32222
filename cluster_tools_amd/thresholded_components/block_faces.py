#! /usr/bin/env python
"""BlockFaces: the label pairs that touch across block faces
(cluster_tools/thresholded_components/block_faces.py:21-184; task surface unchanged).

Each block looks at its upper neighbour along every axis (utils/volume_utils.py:221-270
iterate_faces(return_only_lower=True) / get_face with halo 1): the two facing planes of the
segmentation, both nonzero, plus the two blocks' offsets -> unique (a, b) rows, saved per job
as cc_assignments_<job>.npy.  Only the axial face neighbours are paired, as in the reference:
components that meet only diagonally across a block face stay apart.
"""
import json
import os
import sys

import numpy as np

from cluster_tools_amd import luigi_compat as luigi
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu
from cluster_tools_amd.utils.blocking import Blocking
from cluster_tools_amd.cluster_tasks import SlurmTask, LocalTask, LSFTask


class BlockFacesBase(luigi.Task):
    task_name = 'block_faces'
    src_file = os.path.abspath(__file__)
    allow_retry = False

    input_path = luigi.Parameter()
    input_key = luigi.Parameter()
    offsets_path = luigi.Parameter()
    dependency = luigi.TaskParameter()

    def requires(self):
        return self.dependency

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        shape = vu.get_shape(self.input_path, self.input_key)
        config = self.get_task_config()
        config.update({'input_path': self.input_path, 'input_key': self.input_key,
                       'offsets_path': self.offsets_path, 'block_shape': block_shape,
                       'tmp_folder': self.tmp_folder})
        block_list = vu.blocks_in_volume(shape, block_shape, roi_begin, roi_end)
        self.run_jobs(min(len(block_list), self.max_jobs), block_list, config)


class BlockFacesLocal(BlockFacesBase, LocalTask):
    pass


class BlockFacesSlurm(BlockFacesBase, SlurmTask):
    pass


class BlockFacesLSF(BlockFacesBase, LSFTask):
    pass


def _face_pairs(ds, blocking, block_id, ngb_id, axis, offsets):
    """`_process_face` (block_faces.py:87-113) for the face between block_id and its upper
    neighbour ngb_id along axis."""
    blk = blocking.getBlock(block_id)
    face = tuple(slice(b, e) if d != axis else slice(e - 1, e + 1)
                 for d, (b, e) in enumerate(zip(blk.begin, blk.end)))
    seg = ds[face]
    labels_a = np.take(seg, 0, axis=axis).ravel().astype('uint64')
    labels_b = np.take(seg, 1, axis=axis).ravel().astype('uint64')
    have = np.logical_and(labels_a != 0, labels_b != 0)
    labels_a, labels_b = labels_a[have], labels_b[have]
    if labels_a.size == 0:
        return None
    labels_a += np.uint64(offsets[block_id])
    labels_b += np.uint64(offsets[ngb_id])
    return np.unique(np.stack([labels_a, labels_b], axis=1), axis=0)


def _process_faces(block_id, blocking, ds, offsets, empty_blocks):
    fu.log("start processing block %i" % block_id)
    if block_id in empty_blocks:
        fu.log_block_success(block_id)
        return None
    pairs = []
    for axis in range(3):
        ngb_id = blocking.getNeighborId(block_id, axis, False)
        if ngb_id == -1 or ngb_id in empty_blocks:
            continue
        p = _face_pairs(ds, blocking, block_id, ngb_id, axis, offsets)
        if p is not None:
            pairs.append(p)
    fu.log_block_success(block_id)
    return np.unique(np.concatenate(pairs, axis=0), axis=0) if pairs else None


def block_faces(job_id, config_path):
    fu.log("start processing job %i" % job_id)
    fu.log("reading config from %s" % config_path)
    with open(config_path) as f:
        config = json.load(f)
    with open(config['offsets_path']) as f:
        oc = json.load(f)
    offsets, empty_blocks, n_labels = oc['offsets'], set(oc['empty_blocks']), oc['n_labels']
    with vu.file_reader(config['input_path'], 'r') as f:
        ds = f[config['input_key']]
        blocking = Blocking([0, 0, 0], list(ds.shape), list(config['block_shape']))
        pairs = [_process_faces(b, blocking, ds, offsets, empty_blocks) for b in config['block_list']]
    pairs = [p for p in pairs if p is not None]
    if pairs:
        pairs = np.unique(np.concatenate(pairs, axis=0), axis=0)
        assert pairs.max() < n_labels, "%i, %i" % (int(pairs.max()), n_labels)
    else:
        pairs = np.zeros((0, 2), dtype='uint64')
    np.save(os.path.join(config['tmp_folder'], 'cc_assignments_%i.npy' % job_id), pairs)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    block_faces(job_id, path)
