"""CPU: ThresholdedComponentsWorkflow pieces that need no GPU.

* the oracle's BlockComponents labelling (oracle/threshcc.py) against skimage 0.18.3
  (tests/golden/threshcc_label.npz, scripts/make_threshcc_golden.py);
* ctws_ufd_find (libctws.so host code: nifty boost_ufd) against the oracle's restatement;
* MergeOffsets -> BlockFaces -> MergeAssignments as tasks on a segmentation the oracle labelled
  block by block, against the oracle's table;
* without a GPU the BlockComponents jobs fail and the workflow reports failure (no CPU path).
"""
import json
import os
import sys

import numpy as np
import pytest

from cluster_tools_amd import luigi_compat as luigi
from cluster_tools_amd.utils import volume_utils as vu
from cluster_tools_amd.utils.blocking import Blocking
from oracle import threshcc as T

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'threshcc_label.npz')


def golden_cases():
    g = np.load(GOLDEN)
    names = sorted({k.split('__')[0] for k in g.files})
    out = []
    for n in names:
        thr, mode, masked = g[n + '__params']
        mask = g[n + '__mask'] if n + '__mask' in g.files else None
        out.append((n, g[n + '__input'], float(thr), T.MODES[int(mode)], mask, not bool(masked), g[n + '__labels']))
    return out


@pytest.mark.parametrize('case', golden_cases(), ids=lambda c: c[0])
def test_oracle_labels_match_skimage(case):
    name, x, thr, mode, mask, norm, expected = case
    lab, n = T.block_components(x, thr, mode, mask, normalize_input=norm)
    np.testing.assert_array_equal(lab, expected)
    assert n == int(expected.max())


def test_ufd_find_matches_boost_restatement():
    from cluster_tools_amd import ctws
    rng = np.random.default_rng(0)
    for n, m in [(1, 0), (10, 4), (200, 150), (5000, 6000)]:
        pairs = rng.integers(1, max(2, n), size=(m, 2)).astype('uint64') if m else np.zeros((0, 2), 'uint64')
        pairs = np.unique(pairs, axis=0)
        np.testing.assert_array_equal(ctws.ufd_find(n, pairs), T.boost_ufd_find(n, pairs))
    # union by rank: equal ranks put the first root under the second; the higher rank wins
    np.testing.assert_array_equal(ctws.ufd_find(5, [[1, 2], [3, 4], [1, 3]]), [0, 4, 4, 4, 4])
    np.testing.assert_array_equal(ctws.ufd_find(5, [[1, 2], [2, 3]]), [0, 2, 2, 2, 4])
    with pytest.raises(ctws.CtwsError):
        ctws.ufd_find(3, [[1, 3]])


def _configs(tmp_path, block_shape):
    from cluster_tools_amd.cluster_tasks import BaseClusterTask
    cfg_dir = tmp_path / 'configs'
    cfg_dir.mkdir(exist_ok=True)
    g = BaseClusterTask.default_global_config()
    g.update({'shebang': '#! ' + sys.executable, 'block_shape': list(block_shape)})
    (cfg_dir / 'global.config').write_text(json.dumps(g))
    return str(cfg_dir)


def _volume(shape, seed):
    from scipy.ndimage import gaussian_filter
    rng = np.random.default_rng(seed)
    return gaussian_filter(rng.random(shape).astype('float32'), 1.2).astype('float32')


@pytest.mark.parametrize('max_jobs', [1, 3])
def test_offsets_faces_assignments_tasks_match_oracle(tmp_path, max_jobs):
    """BlockComponents' outputs written from the oracle, then the three merge tasks run as jobs."""
    from cluster_tools_amd.thresholded_components.merge_offsets import MergeOffsetsLocal
    from cluster_tools_amd.thresholded_components.block_faces import BlockFacesLocal
    from cluster_tools_amd.thresholded_components.merge_assignments import MergeAssignmentsLocal
    from cluster_tools_amd.utils.task_utils import DummyTask
    shape, bs = (24, 40, 52), (8, 16, 16)
    x = _volume(shape, 1)
    blocking = Blocking([0, 0, 0], list(shape), list(bs))
    ref_seg, ref_ass, ref_off = T.thresholded_components(x, blocking, 0.55, 'greater')
    path, tmp = str(tmp_path / 'cc.n5'), tmp_path / 'tmp'
    tmp.mkdir()
    seg = np.zeros(shape, 'uint64')
    counts = {}
    for bid in range(blocking.numberOfBlocks):
        bb = vu.block_to_bb(blocking.getBlock(bid))
        lab, n = T.block_components(x[bb], 0.55, 'greater')
        seg[bb] = lab
        counts[bid] = n + 1 if n else 0
    n_jobs = min(blocking.numberOfBlocks, max_jobs)
    for j in range(n_jobs):   # BlockComponents' per-job offset files (block_components.py:286-290)
        with open(str(tmp / ('connected_components_offsets_%i.json' % j)), 'w') as f:
            json.dump({b: counts[b] for b in range(j, blocking.numberOfBlocks, n_jobs)}, f)
    with vu.file_reader(path) as f:
        f.create_dataset('cc', data=seg, chunks=(4, 8, 8))
    cfg = _configs(tmp_path, bs)
    off_path = str(tmp / 'cc_offsets.json')
    common = dict(tmp_folder=str(tmp), config_dir=cfg, max_jobs=max_jobs)
    t = MergeOffsetsLocal(shape=list(shape), save_path=off_path, dependency=DummyTask(), **common)
    t = BlockFacesLocal(input_path=path, input_key='cc', offsets_path=off_path, dependency=t, **common)
    t = MergeAssignmentsLocal(output_path=path, output_key='ass', shape=list(shape), offset_path=off_path,
                              dependency=t, **common)
    assert luigi.build([t], local_scheduler=True)
    with open(off_path) as f:
        off = json.load(f)
    assert off == ref_off
    with vu.file_reader(path, 'r') as f:
        ass = f['ass'][:]
    np.testing.assert_array_equal(ass, ref_ass)
    # the table merges components across block faces: fewer representatives than labels
    assert len(np.unique(ass)) < off['n_labels']


def test_oracle_workflow_is_a_partition_of_the_global_labelling():
    """The reference's own test (test/thresholded_components/thresholded_components.py:57-77)
    compares the workflow with skimage.label of the whole volume by adjusted Rand index; on a
    volume whose blocks all span [0, 1] and with no diagonal-only contact across block faces the
    two partitions agree exactly.  Here: every merged component lies inside one global component
    of the same members, and some are merged across block faces."""
    shape, bs = (16, 32, 64), (8, 16, 32)
    x = _volume(shape, 3)
    seg, _, _ = T.thresholded_components(x, Blocking([0, 0, 0], list(shape), list(bs)), 0.5, 'greater')
    glob_, _ = T.label26(seg != 0)   # (each block is normalized on its own)
    pairs = np.unique(np.stack([seg.ravel(), glob_.ravel()], 1), axis=0)
    assert len(np.unique(pairs[:, 0])) == len(pairs)   # each merged id inside one global id
    assert len(np.unique(seg)) < len(np.unique(seg[:, :, :32])) + len(np.unique(seg[:, :, 32:]))


def test_workflow_fails_loudly_without_gpu(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    from cluster_tools_amd.thresholded_components import ThresholdedComponentsWorkflow
    path = str(tmp_path / 'in.n5')
    with vu.file_reader(path) as f:
        f.create_dataset('x', data=_volume((16, 32, 32), 2), chunks=(8, 16, 16))
    wf = ThresholdedComponentsWorkflow(input_path=path, input_key='x', output_path=path, output_key='cc',
                                       assignment_key='ass', threshold=.5, tmp_folder=str(tmp_path / 'tmp'),
                                       config_dir=_configs(tmp_path, (8, 16, 16)), max_jobs=2, target='local')
    assert not luigi.build([wf], local_scheduler=True)
    assert os.path.exists(str(tmp_path / 'tmp' / 'block_components_job_0.config'))


def test_scan_block_counts_matches_oracle_merge_offsets():
    from cluster_tools_amd.thresholded_components.merge_offsets import scan_block_counts
    rng = np.random.default_rng(2)
    for n in (1, 2, 7, 64):
        c = rng.integers(0, 50, n) * (rng.random(n) > .3)
        ids = rng.permutation(n)
        got = scan_block_counts({int(b): int(c[b]) for b in ids})
        assert got == T.merge_offsets(c.tolist())


# ---- the merge tail in the BlockComponents jobs (merge_in_job.py): 2 gloo jobs ---------------
MJ_SHAPE, MJ_BLOCK = (32, 96, 160), (16, 32, 64)


def _mj_worker(rank, world, root, faces_max_jobs, masked):
    import torch.distributed as dist
    from cluster_tools_amd.cluster_tasks import split_blocks
    from cluster_tools_amd.thresholded_components.merge_in_job import merge_in_job
    from cluster_tools_amd.utils.blocking import Blocking
    from cluster_tools_amd.utils import volume_utils as vu
    from cluster_tools_amd.watershed import job_relabel
    x = _volume(MJ_SHAPE, 7)
    mask = _mj_mask() if masked else None
    blocking = Blocking([0, 0, 0], list(MJ_SHAPE), list(MJ_BLOCK))
    block_list = list(range(blocking.numberOfBlocks))
    runs = split_blocks(block_list, world, consecutive=True)
    owner = {b: j for j, r in enumerate(runs) for b in r}
    job_relabel.init_group(rank, world, 'file://' + os.path.join(root, 'rdv'), 'gloo', timeout_s=120)
    try:
        results = []
        for b in runs[rank]:
            bb = vu.block_to_bb(blocking.getBlock(b))
            if mask is not None and not mask[bb].any():
                results.append((b, bb, None, 0))
                continue
            lab, n = T.block_components(x[bb], .55, 'greater', None if mask is None else mask[bb],
                                        normalize_input=mask is None)
            results.append((b, bb, lab if n else None, n + 1 if n else 0))
        cfg = dict(tmp_folder=root, offsets_path=os.path.join(root, 'cc_offsets.json'),
                   output_path=os.path.join(root, 'out.n5'), assignment_key='ass', faces_max_jobs=faces_max_jobs)
        with vu.file_reader(cfg['output_path']) as f:
            merge_in_job(rank, results, blocking, block_list, owner, cfg, f['cc'], log=lambda m: None)
    finally:
        dist.destroy_process_group()


def _mj_mask():
    m = np.zeros(MJ_SHAPE, bool)
    m[:, 10:80, 20:150] = True
    m[:, :, :64] = False
    return m


@pytest.mark.parametrize('masked', [False, True])
@pytest.mark.parametrize('faces_max_jobs', [1, 100])
def test_merge_in_job_matches_the_five_task_chain(tmp_path, masked, faces_max_jobs):
    """Offsets, face pairs, boost_ufd assignments and the final write of two jobs over gloo
    equal the oracle's whole pipeline; with as many BlockFaces jobs as blocks the last block has
    no upper face, one job has no pair and the reference's merge is the identity
    (merge_assignments.py:116-123)."""
    import torch.multiprocessing as tmp
    from cluster_tools_amd.utils.blocking import Blocking
    from cluster_tools_amd.utils import volume_utils as vu
    root = str(tmp_path)
    with vu.file_reader(os.path.join(root, 'out.n5')) as f:
        f.create_dataset('cc', shape=MJ_SHAPE, dtype='uint64', chunks=tuple(b // 2 for b in MJ_BLOCK))
    tmp.spawn(_mj_worker, args=(2, root, faces_max_jobs, masked), nprocs=2, join=True)
    x = _volume(MJ_SHAPE, 7)
    blocking = Blocking([0, 0, 0], list(MJ_SHAPE), list(MJ_BLOCK))
    seg, ass, oc = T.thresholded_components(x, blocking, .55, 'greater', mask=_mj_mask() if masked else None,
                                            faces_jobs=faces_max_jobs)
    # (with as many BlockFaces jobs as blocks the oracle's merge is the identity too)
    assert (faces_max_jobs > 1) == np.array_equal(ass, np.arange(len(ass), dtype='uint64'))
    with vu.file_reader(os.path.join(root, 'out.n5'), 'r') as f:
        np.testing.assert_array_equal(f['ass'][:], ass)
        np.testing.assert_array_equal(f['cc'][:], seg)
        assert f['cc'].attrs['maxId'] == int(ass.max())
    with open(os.path.join(root, 'cc_offsets.json')) as fo:
        got = json.load(fo)
    assert got == {'offsets': [int(o) for o in oc['offsets']], 'empty_blocks': oc['empty_blocks'],
                   'n_labels': oc['n_labels']}
    assert not [n for n in os.listdir(root) if n.startswith(('cc_face_', 'cc_block_pairs', 'cc_assignments_merged'))]
