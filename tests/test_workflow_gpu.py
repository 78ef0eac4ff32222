"""End-to-end WatershedWorkflow (target='local') on the GPU, with the reference's test configs
(test/watershed/test_watershed.py:86-136) on a synthetic n5 volume.  Checks the reference's
`_check_result` invariants (:53-70) and compares the watershed stage with the oracle run
block by block (same blocking, halos and offsets)."""
import json
import os
import sys

import numpy as np
import pytest

from conftest import luigi_build

from cluster_tools_amd import luigi_compat as luigi
from cluster_tools_amd.utils import volume_utils as vu
from cluster_tools_amd.utils.blocking import Blocking
from cluster_tools_amd.synthetic import boundary_map, ellipsoid_mask
from cluster_tools_amd.metrics import vi_scores
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SHAPE = (40, 128, 128)
BLOCK_SHAPE = [10, 64, 64]

CONFIGS = {
    'ws_2d': dict(apply_dt_2d=True, apply_ws_2d=True, threshold=0.25, sigma_weights=0., halo=[0, 16, 16]),
    'ws_3d': dict(apply_dt_2d=False, apply_ws_2d=False, sigma_seeds=(.5, 2., 2.), sigma_weights=(.5, 2., 2.),
                  halo=[2, 16, 16]),
    'ws_pixel_pitch': dict(apply_dt_2d=False, apply_ws_2d=False, pixel_pitch=(10, 1, 1)),
}


def _setup(tmp_path, name, with_mask):
    from cluster_tools_amd.watershed.watershed import WatershedLocal
    cfg_dir = tmp_path / 'configs'
    cfg_dir.mkdir()
    g = WatershedLocal.default_global_config()
    g['shebang'] = '#! ' + sys.executable
    g['block_shape'] = BLOCK_SHAPE
    (cfg_dir / 'global.config').write_text(json.dumps(g))
    c = WatershedLocal.default_task_config()
    c.update(CONFIGS[name])
    (cfg_dir / 'watershed.config').write_text(json.dumps(c))
    inp = str(tmp_path / 'data.n5')
    x = boundary_map(SHAPE, seed=3)
    with vu.file_reader(inp) as f:
        f.create_dataset('boundaries', data=x, chunks=(10, 64, 64))
        if with_mask:
            f.create_dataset('mask', data=ellipsoid_mask(SHAPE), chunks=(10, 64, 64))
    return str(cfg_dir), inp, x, c


def _oracle_volume(x, c, mask):
    """The reference's per-block `_ws_block` over the volume, via the oracle."""
    blocking = Blocking([0, 0, 0], list(SHAPE), BLOCK_SHAPE)
    out = np.zeros(SHAPE, np.uint64)
    halo = c.get('halo', [0, 0, 0])
    for bid in range(blocking.numberOfBlocks):
        if sum(halo) > 0:
            bh = blocking.getBlockWithHalo(bid, halo)
            ib, ob, il = vu.block_to_bb(bh.outerBlock), vu.block_to_bb(bh.innerBlock), vu.block_to_bb(bh.innerBlockLocal)
        else:
            ib = ob = vu.block_to_bb(blocking.getBlock(bid))
            il = tuple(slice(0, s.stop - s.start) for s in ib)
        b = dict(input=x[ib], block_id=bid, inner_begin=[s.start for s in il],
                 inner_shape=[s.stop - s.start for s in il], crop_relabel=ob != ib)
        if mask is not None:
            b['mask'] = mask[ib]
        r = O.ws_blocks(c, BLOCK_SHAPE, [b])[0]
        if r['status'] in (0, 2):
            out[ob] = r['output']
    return out


def _build(task, tmp_folder):
    luigi_build(task, tmp_folder)


def _n_ids_and_ccs(res):
    cc, _ = O.label_with_background(res.astype('uint32'))
    return len(np.unique(res)), len(np.unique(cc))


def _check_result(res, with_mask, ref=None):
    """test_watershed.py:53-70.  With `ref` (the reference semantics via the oracle), the
    "no disconnected segments" invariant is required to hold exactly as far as it holds for
    the reference: the sequential two-pass watershed can itself produce a disconnected id
    (a pass-2 block floods from a diagonal neighbour's labels in its halo corner)."""
    assert res.shape == SHAPE
    assert not np.allclose(res, 0)
    assert (0 in res) == with_mask
    n_ids, n_cc = _n_ids_and_ccs(res)
    if ref is None:
        assert n_ids == n_cc, "disconnected segments"
    else:
        assert (n_ids, n_cc) == _n_ids_and_ccs(ref), "disconnected segments differ from the reference's"


@pytest.mark.parametrize('name', sorted(CONFIGS))
@pytest.mark.parametrize('with_mask', [False, True])
@pytest.mark.parametrize('relabel_in_job', [True, False])
def test_watershed_workflow(tmp_path, name, with_mask, relabel_in_job):
    """relabel_in_job: the relabel folded into the watershed jobs (their process group's offset
    scan, job_relabel.py) must give the three-task RelabelWorkflow's volume, table and maxId."""
    from cluster_tools_amd.watershed import WatershedWorkflow
    from cluster_tools_amd.watershed.watershed import WatershedLocal
    cfg_dir, inp, x, c = _setup(tmp_path, name, with_mask)
    out = str(tmp_path / 'ws.n5')
    mask_kw = dict(mask_path=inp, mask_key='mask') if with_mask else {}
    # 1. the watershed task alone: compare with the oracle block by block
    ws = WatershedLocal(input_path=inp, input_key='boundaries', output_path=out, output_key='ws_raw',
                        config_dir=cfg_dir, tmp_folder=str(tmp_path / 'tmp_ws'), max_jobs=2, **mask_kw)
    assert luigi.build([ws], local_scheduler=True)
    with vu.file_reader(out, 'r') as f:
        raw = f['ws_raw'][:]
    ref = _oracle_volume(x, c, ellipsoid_mask(SHAPE) if with_mask else None)
    vis, vim = vi_scores(raw, ref, [0] if with_mask else None)
    assert vis + vim <= 0.01, (vis, vim)
    # 2. the whole workflow (watershed + relabel)
    wf = WatershedWorkflow(input_path=inp, input_key='boundaries', output_path=out, output_key='ws',
                           config_dir=cfg_dir, tmp_folder=str(tmp_path / 'tmp'), target='local', max_jobs=2,
                           relabel_in_job=relabel_in_job, **mask_kw)
    _build(wf, tmp_path / 'tmp')
    with vu.file_reader(out, 'r') as f:
        res = f['ws'][:]
        assert f['ws'].attrs['maxId'] == int(res.max())
        table = f['relabel_watershed'][:]
    _check_result(res.astype('uint64'), with_mask)
    assert len(np.unique(res)) == len(table)
    # RelabelWorkflow parity: find_labeling.py:104-116 (sorted uniques -> consecutive ids from
    # 0 if 0 occurs, else 1) + write.py (takeDict) applied to the raw watershed output
    np.testing.assert_array_equal(res.astype('uint64'), _reference_relabel(raw))
    uniq = np.unique(raw)
    start = 0 if uniq[0] == 0 else 1
    np.testing.assert_array_equal(table[:, 0], uniq)
    np.testing.assert_array_equal(table[:, 1], np.arange(start, start + len(uniq), dtype='uint64'))
    if relabel_in_job:
        return
    # the watershed jobs' per-block uniques that FindUniques read instead of the volume: one
    # file per written block (mask-skipped blocks have none and are read), each np.unique of
    # the block's raw labels
    from cluster_tools_amd.watershed.watershed import block_uniques_file
    blocking = Blocking([0, 0, 0], list(SHAPE), BLOCK_SHAPE)
    folder = str(tmp_path / 'tmp' / 'watershed_block_uniques')
    n_files = 0
    for bid in range(blocking.numberOfBlocks):
        path = block_uniques_file(folder, bid)
        if os.path.exists(path):
            n_files += 1
            np.testing.assert_array_equal(np.load(path), np.unique(raw[vu.block_to_bb(blocking.getBlock(bid))]))
    assert n_files == blocking.numberOfBlocks or (with_mask and n_files > 0)


def _reference_relabel(raw):
    """RelabelWorkflow restated with numpy: FindUniques/FindLabeling (np.unique, arange from 0
    or 1, find_labeling.py:104-116) then Write (takeDict, write.py:153-175)."""
    uniq, inv = np.unique(raw, return_inverse=True)
    start = 0 if uniq[0] == 0 else 1
    return (inv.reshape(raw.shape) + start).astype('uint64')


def _oracle_two_pass(x, c, mask):
    """The reference's TwoPassWatershed over the volume via the oracle: pass 1 on the
    checkerboard colour of block 0, then pass 2 on the other colour with the pass-1 labels
    as initial seeds, block by block in list order: each pass-2 block reads ds_out[input_bb]
    after the writes of the blocks before it (two_pass_watershed.py:228,252 in the job's
    sequential loop, one job)."""
    blocking = Blocking([0, 0, 0], list(SHAPE), BLOCK_SHAPE)
    lists = vu.make_checkerboard_block_lists(blocking)
    out = np.zeros(SHAPE, np.uint64)
    halo = c.get('halo', [0, 0, 0])

    def bbs(bid):
        if sum(halo) > 0:
            bh = blocking.getBlockWithHalo(bid, halo)
            return (vu.block_to_bb(bh.outerBlock), vu.block_to_bb(bh.innerBlock),
                    vu.block_to_bb(bh.innerBlockLocal))
        ib = vu.block_to_bb(blocking.getBlock(bid))
        return ib, ib, tuple(slice(0, s.stop - s.start) for s in ib)

    for pass_id, blist in enumerate(lists):
        for bid in blist:
            ib, ob, il = bbs(bid)
            b = dict(input=x[ib], block_id=bid, inner_begin=[s.start for s in il],
                     inner_shape=[s.stop - s.start for s in il], crop_relabel=(ob != ib) and pass_id == 0)
            if mask is not None:
                b['mask'] = mask[ib]
            if pass_id == 1:
                b['initial_seeds'] = out[ib].copy()
            r = O.ws_blocks(c, BLOCK_SHAPE, [b], pass_id=pass_id)[0]
            if r['status'] in (0, 2):
                out[ob] = r['output']
    return out


@pytest.mark.parametrize('batch_blocks', [16, 1000])
@pytest.mark.parametrize('name', ['ws_2d', 'ws_3d'])
def test_two_pass_workflow(tmp_path, name, batch_blocks):
    """test_watershed.py:102-103,121-122 (two_pass=True) with the halo configs, pass 2 on GPU.
    Whatever the GPU batch size, the result is the reference's sequential block order."""
    from cluster_tools_amd.watershed import WatershedWorkflow
    from cluster_tools_amd.watershed.two_pass_watershed import TwoPassWatershedLocal
    cfg_dir, inp, x, c = _setup(tmp_path, name, False)
    c2 = TwoPassWatershedLocal.default_task_config()
    c2.update(CONFIGS[name])
    c2['gpu_batch_blocks'] = batch_blocks
    with open(os.path.join(cfg_dir, 'two_pass_watershed.config'), 'w') as f:
        json.dump(c2, f)
    out = str(tmp_path / 'ws.n5')
    wf = WatershedWorkflow(input_path=inp, input_key='boundaries', output_path=out, output_key='ws',
                           config_dir=cfg_dir, tmp_folder=str(tmp_path / 'tmp'), target='local', max_jobs=1,
                           two_pass=True)
    assert luigi.build([wf], local_scheduler=True)
    with vu.file_reader(out, 'r') as f:
        res = f['ws'][:].astype('uint64')
    ref = _oracle_two_pass(x, c2, None)
    _check_result(res, False, ref)
    vis, vim = vi_scores(res, ref)
    print('two-pass %s: VI %.2e' % (name, vis + vim))
    assert vis + vim <= 0.01, (vis, vim)


def test_watershed_low_res_mask(tmp_path):
    """A mask stored at half resolution goes through load_mask -> InterpolatedVolume
    (volume_utils.py:208-218, volume_classes.py:155-232) in the job; the oracle gets the same
    per-block masks from the same InterpolatedVolume requests."""
    from cluster_tools_amd.watershed.watershed import WatershedLocal
    cfg_dir, inp, x, c = _setup(tmp_path, 'ws_3d', False)
    low = ellipsoid_mask(SHAPE)[::2, ::2, ::2]
    with vu.file_reader(inp) as f:
        f.create_dataset('mask_low', data=low, chunks=(10, 32, 32))
    out = str(tmp_path / 'ws.n5')
    ws = WatershedLocal(input_path=inp, input_key='boundaries', output_path=out, output_key='ws_raw',
                        config_dir=cfg_dir, tmp_folder=str(tmp_path / 'tmp_ws'), max_jobs=2,
                        mask_path=inp, mask_key='mask_low')
    assert luigi.build([ws], local_scheduler=True)
    with vu.file_reader(out, 'r') as f:
        raw = f['ws_raw'][:]
    mask = vu.load_mask(inp, 'mask_low', SHAPE)
    assert isinstance(mask, vu.InterpolatedVolume)
    ref = _oracle_volume(x, c, mask)
    assert (raw == 0).any() and ((raw == 0) == (ref == 0)).all()
    vis, vim = vi_scores(raw, ref, [0])
    assert vis + vim <= 0.01, (vis, vim)


@pytest.mark.parametrize('with_mask', [False, True])
def test_watershed_workflow_roi_relabel_in_job(tmp_path, with_mask):
    """the in-job relabel hands each job a consecutive run of the block list; with a
    ROI that list is not 0..N-1.  Both relabel modes must process exactly the ROI's blocks and
    agree on the volume, the table and maxId."""
    from cluster_tools_amd.watershed import WatershedWorkflow
    cfg_dir, inp, x, c = _setup(tmp_path, 'ws_3d', with_mask)
    g = json.loads((tmp_path / 'configs' / 'global.config').read_text())
    g['roi_begin'], g['roi_end'] = [10, 64, 0], [40, 128, 128]
    (tmp_path / 'configs' / 'global.config').write_text(json.dumps(g))
    mask_kw = dict(mask_path=inp, mask_key='mask') if with_mask else {}
    res = {}
    for rij in (True, False):
        out = str(tmp_path / ('ws_%d.n5' % rij))
        wf = WatershedWorkflow(input_path=inp, input_key='boundaries', output_path=out, output_key='ws',
                               config_dir=cfg_dir, tmp_folder=str(tmp_path / ('tmp_%d' % rij)), target='local',
                               max_jobs=2, relabel_in_job=rij, **mask_kw)
        _build(wf, tmp_path / ('tmp_%d' % rij))
        with vu.file_reader(out, 'r') as f:
            res[rij] = (f['ws'][:], f['relabel_watershed'][:], f['ws'].attrs['maxId'])
    np.testing.assert_array_equal(res[True][0], res[False][0])
    np.testing.assert_array_equal(res[True][1], res[False][1])
    assert res[True][2] == res[False][2]
    vol = res[True][0]
    # blocks outside the ROI are never written
    assert not vol[:10].any() and not vol[:, :64].any()
    assert vol[10:, 64:].any()


def test_watershed_workflow_retry(tmp_path, monkeypatch):
    """VERDICT r05 #7, the reference's test/retry/test_retry.py:34-54 on the watershed: with
    max_num_retries = 1 the blocks with id % 4 == 1 fail on the first attempt
    (CTWS_TEST_FAIL_ONCE), the task resubmits them (cluster_tasks.py:127-142) and the workflow
    ends with the same relabelled volume, table and maxId as a run without failures."""
    from cluster_tools_amd.watershed import WatershedWorkflow
    cfg_dir, inp, x, c = _setup(tmp_path, 'ws_2d', False)
    res = {}
    for retry in (False, True):
        if retry:
            g = json.loads((tmp_path / 'configs' / 'global.config').read_text())
            g['max_num_retries'] = 1
            (tmp_path / 'configs' / 'global.config').write_text(json.dumps(g))
            fail_dir = tmp_path / 'fail'
            fail_dir.mkdir()
            monkeypatch.setenv('CTWS_TEST_FAIL_ONCE', str(fail_dir))
        out = str(tmp_path / ('ws_%d.n5' % retry))
        tmp = tmp_path / ('tmp_%d' % retry)
        # 4 jobs: the failing blocks 1, 5, 9, 13 are all job 1's, fewer than half the jobs fail
        wf = WatershedWorkflow(input_path=inp, input_key='boundaries', output_path=out, output_key='ws',
                               config_dir=cfg_dir, tmp_folder=str(tmp), target='local', max_jobs=4)
        _build(wf, tmp)
        with vu.file_reader(out, 'r') as f:
            res[retry] = (f['ws'][:], f['relabel_watershed'][:], f['ws'].attrs['maxId'])
    assert sorted(os.listdir(fail_dir)) == sorted('failed_block_%d' % b for b in (1, 5, 9, 13))
    logs = open(os.path.join(str(tmp_path / 'tmp_1'), 'watershed.log')).read()
    assert 'resubmitting 4 failed blocks in 1 retry attempt' in logs
    for a, b in zip(res[False], res[True]):
        np.testing.assert_array_equal(a, b)
    _check_result(res[True][0].astype('uint64'), False)
