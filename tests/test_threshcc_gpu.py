"""GPU: ThresholdedComponentsWorkflow on the MI355X against the CPU oracle (oracle/threshcc.py).

* ctws_threshold_components (k_threshcc.hip) on the skimage golden vectors and on random blocks
  sized to cross many 8x8x64 tiles (sparse / dense / all members / empty, the three modes, masks,
  partial tiles): labels bit-exact, including skimage's C-order numbering;
* the workflow as tasks (BlockComponents on the GPU, the merges, the GPU write) against the
  oracle's whole pipeline, bit-exact segmentation and assignment table;
* ThresholdAndWatershedWorkflow: the components grown by WatershedFromSeeds, against the oracle
  composition (oracle threshcc -> orc_ws_from_seeds per block).
"""
import json
import os
import sys

import numpy as np
import pytest

from cluster_tools_amd.utils import volume_utils as vu
from cluster_tools_amd.utils.blocking import Blocking
from oracle import threshcc as T
from test_threshcc import golden_cases, _volume

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('case', golden_cases(), ids=lambda c: c[0])
def test_block_components_match_skimage_golden(gpu_handle, case):
    name, x, thr, mode, mask, norm, expected = case
    lab, n = gpu_handle.threshold_components(x, thr, mode, mask=mask, normalize=norm)
    np.testing.assert_array_equal(lab, expected)
    assert n == int(expected.max())


def _random_cases():
    rng = np.random.default_rng(11)
    cases = []
    for shape, thr, mode in [((1, 1, 1), .5, 'greater'), ((1, 7, 200), .6, 'greater'), ((9, 17, 129), .8, 'greater'),
                             ((20, 70, 300), .9, 'greater'), ((20, 70, 300), .55, 'greater'),
                             ((33, 65, 130), .2, 'less'), ((16, 64, 64), 1.0, 'less'), ((8, 9, 65), .0, 'equal'),
                             ((64, 256, 256), .92, 'greater'), ((64, 256, 256), .7, 'greater')]:
        cases.append(('%s_%s_%g' % ('x'.join(map(str, shape)), mode, thr), rng.random(shape, dtype=np.float32),
                      thr, mode, None))
    sh = (24, 50, 140)
    m = (rng.random(sh) > .3).astype(np.uint8)
    cases.append(('masked', rng.random(sh, dtype=np.float32), .75, 'greater', m))
    cases.append(('integers_equal', rng.integers(0, 4, size=sh).astype(np.float32), 2.0, 'equal', m))
    cases.append(('constant', np.full(sh, 3.0, np.float32), .5, 'greater', None))
    return cases


@pytest.mark.parametrize('case', _random_cases(), ids=lambda c: c[0])
def test_block_components_match_oracle(gpu_handle, case):
    name, x, thr, mode, mask = case
    norm = mask is None and name != 'integers_equal'
    lab, n = gpu_handle.threshold_components(x, thr, mode, mask=mask, normalize=norm)
    ref, rn = T.block_components(x, thr, mode, mask, normalize_input=norm)
    assert n == rn
    np.testing.assert_array_equal(lab, ref)


def test_block_components_smooth_volume_large(gpu_handle):
    """A 96x256x256 block of smooth blobs: long components across many tiles (merge chains)."""
    x = _volume((96, 256, 256), 5)
    lab, n = gpu_handle.threshold_components(x, .5, 'greater')
    ref, rn = T.block_components(x, .5, 'greater')
    assert n == rn and n > 10
    np.testing.assert_array_equal(lab, ref)


def _configs(tmp_path, block_shape, task_configs=None):
    from cluster_tools_amd.cluster_tasks import BaseClusterTask
    cfg_dir = tmp_path / 'configs'
    cfg_dir.mkdir(exist_ok=True)
    g = BaseClusterTask.default_global_config()
    g.update({'shebang': '#! ' + sys.executable, 'block_shape': list(block_shape)})
    (cfg_dir / 'global.config').write_text(json.dumps(g))
    for name, c in (task_configs or {}).items():
        (cfg_dir / ('%s.config' % name)).write_text(json.dumps(c))
    return str(cfg_dir)


@pytest.mark.parametrize('merge_in_job', [True, False, 'spill'])
@pytest.mark.parametrize('masked,max_jobs', [(False, 1), (False, 3), (True, 2)])
def test_thresholded_components_workflow_matches_oracle(tmp_path, masked, max_jobs, merge_in_job):
    """merge_in_job: the merge tail in the BlockComponents jobs (merge_in_job.py), else the
    reference's five-task chain; with max_jobs > 1 BlockFaces has several jobs (one of them
    without any pair makes the reference's merge the identity -- both modes must agree).
    'spill': the in-job merge with the labels written as they come and re-read by the merge
    (block_components.spill_labels, the path a job takes when its labels would not fit its
    share of host memory)."""
    from conftest import luigi_build
    from cluster_tools_amd.thresholded_components import ThresholdedComponentsWorkflow
    from cluster_tools_amd.thresholded_components.block_components import BlockComponentsLocal
    task_configs = None
    if merge_in_job == 'spill':
        bc = BlockComponentsLocal.default_task_config()
        bc['merge_spill'] = True
        task_configs = {'block_components': bc}
        merge_in_job = True
    shape, bs = (32, 96, 160), (16, 32, 64)
    x = _volume(shape, 7)
    path = str(tmp_path / 'data.n5')
    mask = None
    with vu.file_reader(path) as f:
        f.create_dataset('x', data=x, chunks=(8, 16, 32))
        if masked:
            mask = np.zeros(shape, np.uint8)
            mask[:, 10:80, 20:150] = 1
            mask[:, :, :64] = 0     # whole blocks outside the mask
            f.create_dataset('mask', data=mask, chunks=(8, 16, 32))
    wf = ThresholdedComponentsWorkflow(input_path=path, input_key='x', output_path=path, output_key='cc',
                                       assignment_key='ass', threshold=.55, tmp_folder=str(tmp_path / 'tmp'),
                                       config_dir=_configs(tmp_path, bs, task_configs), max_jobs=max_jobs,
                                       target='local', mask_path=path if masked else '',
                                       mask_key='mask' if masked else '', merge_in_job=merge_in_job)
    luigi_build(wf, tmp_path / 'tmp')
    ref_seg, ref_ass, ref_off = T.thresholded_components(x, Blocking([0, 0, 0], list(shape), list(bs)), .55,
                                                         'greater', mask=mask, faces_jobs=max_jobs)
    # the merge removes its per-run files (face planes, pair files, merged assignments)
    left = [n for n in os.listdir(str(tmp_path / 'tmp'))
            if n.startswith(('cc_face_', 'cc_block_pairs_', 'cc_assignments_merged'))]
    assert not left, left
    with vu.file_reader(path, 'r') as f:
        seg, ass = f['cc'][:], f['ass'][:]
        max_id = f['cc'].attrs['maxId']
    np.testing.assert_array_equal(ass, ref_ass)
    np.testing.assert_array_equal(seg, ref_seg)
    assert max_id == int(ref_ass.max())
    assert len(np.unique(seg)) > 2


def test_thresholded_components_channels_match_oracle(tmp_path):
    """A 4-D input with channel=[0, 2]: the channels are summed in the dataset dtype and
    thresholded raw (block_components.py:152-158), here in 'less' mode."""
    from conftest import luigi_build
    from cluster_tools_amd.thresholded_components import ThresholdedComponentsWorkflow
    shape, bs = (24, 64, 130), (12, 32, 64)
    chans = np.stack([_volume(shape, s) for s in (1, 2, 3)])
    path = str(tmp_path / 'data.n5')
    with vu.file_reader(path) as f:
        f.create_dataset('x', data=chans, chunks=(1, 6, 16, 32))
    wf = ThresholdedComponentsWorkflow(input_path=path, input_key='x', output_path=path, output_key='cc',
                                       assignment_key='ass', threshold=.98, threshold_mode='less', channel=[0, 2],
                                       tmp_folder=str(tmp_path / 'tmp'), config_dir=_configs(tmp_path, bs),
                                       max_jobs=2, target='local')
    luigi_build(wf, tmp_path / 'tmp')
    summed = (chans[0] + chans[2]).astype(np.float32)
    ref_seg, ref_ass, _ = T.thresholded_components(summed, Blocking([0, 0, 0], list(shape), list(bs)), .98, 'less',
                                                   normalize_input=False)
    with vu.file_reader(path, 'r') as f:
        np.testing.assert_array_equal(f['ass'][:], ref_ass)
        np.testing.assert_array_equal(f['cc'][:], ref_seg)
    assert len(np.unique(ref_seg)) > 2


def test_threshold_and_watershed_workflow_matches_oracle(tmp_path):
    from conftest import luigi_build
    from cluster_tools_amd.thresholded_components import ThresholdAndWatershedWorkflow
    from cluster_tools_amd.watershed.watershed_from_seeds import WatershedFromSeedsLocal
    from cluster_tools_amd.synthetic import boundary_map
    from oracle import oracle as O
    shape, bs = (20, 96, 128), (10, 48, 64)
    x = boundary_map(shape, seed=4).astype(np.float32)
    path = str(tmp_path / 'data.n5')
    with vu.file_reader(path) as f:
        f.create_dataset('x', data=x, chunks=(5, 24, 32))
    wcfg = WatershedFromSeedsLocal.default_task_config()
    wf = ThresholdAndWatershedWorkflow(input_path=path, input_key='x', output_path=path, output_key='seg',
                                       assignment_key='ass', threshold=.3, threshold_mode='less',
                                       tmp_folder=str(tmp_path / 'tmp'), max_jobs=2, target='local',
                                       config_dir=_configs(tmp_path, bs, {'watershed_from_seeds': wcfg}))
    luigi_build(wf, tmp_path / 'tmp')
    blocking = Blocking([0, 0, 0], list(shape), list(bs))
    seeds, _, _ = T.thresholded_components(x, blocking, .3, 'less')
    ref = np.zeros(shape, np.uint64)
    for bid in range(blocking.numberOfBlocks):
        bb = vu.block_to_bb(blocking.getBlock(bid))
        with O.flood_model():
            ref[bb] = O.ws_from_seeds(wcfg, [dict(input=x[bb], seeds=seeds[bb])])[0]['output']
    with vu.file_reader(path, 'r') as f:
        res = f['seg'][:]
    np.testing.assert_array_equal(res, ref)
    assert (res != 0).mean() > .9


def _dtype_cases():
    """Raw (masked / channel-sum) blocks in the dataset's own dtype: the
    reference compares `ds_in[bb] > threshold` with a Python float, float64 for float64 and
    integer data -- values straddling the threshold within float32's rounding, integers above
    2^24 that float32 cannot tell apart."""
    rng = np.random.default_rng(5)
    sh = (12, 40, 150)
    m = (rng.random(sh) > .2).astype(np.uint8)
    thr = 0.3
    f64 = np.where(rng.random(sh) > .5, thr + 1e-12, thr - 1e-12)          # all round to float32(0.3)
    big = np.int64(2 ** 24 + 1)
    i32 = np.where(rng.random(sh) > .5, big, big - 1).astype(np.int32)      # 2^24 and 2^24+1 are one float32
    u64 = np.where(rng.random(sh) > .5, 2 ** 53 + 2, 2 ** 40).astype(np.uint64)
    return [('f64_straddle', f64, thr, 'greater', m), ('f64_less', f64, thr, 'less', m),
            ('i32_equal_2p24', i32, float(big), 'equal', m), ('i32_greater', i32, float(big - 1), 'greater', m),
            ('u64_greater', u64, 2.0 ** 41, 'greater', m),
            ('u8_raw', rng.integers(0, 256, sh).astype(np.uint8), 99.5, 'greater', m),
            ('i16_less', rng.integers(-300, 300, sh).astype(np.int16), -7.0, 'less', m),
            ('i8_equal', rng.integers(-3, 3, sh).astype(np.int8), -1.0, 'equal', m)]


@pytest.mark.parametrize('case', _dtype_cases(), ids=lambda c: c[0])
def test_block_components_raw_dtypes_match_numpy(gpu_handle, case):
    name, x, thr, mode, mask = case
    lab, n = gpu_handle.threshold_components(x, thr, mode, mask=mask, normalize=False)
    ref, rn = T.block_components(x, thr, mode, mask, normalize_input=False)
    assert rn > 0 and n == rn
    np.testing.assert_array_equal(lab, ref)
    if name in ('f64_straddle', 'i32_equal_2p24'):
        # the float32 path would have classified these differently
        f32, _ = T.block_components(x.astype(np.float32), thr, mode, mask, normalize_input=False)
        assert not np.array_equal(f32 != 0, ref != 0)


@pytest.mark.parametrize('sigma', [1.0, 2.0])
@pytest.mark.parametrize('kind', ['unmasked', 'masked', 'channel_sum_u8', 'f64_unmasked'])
def test_block_components_sigma_prefilter_match_oracle(gpu_handle, kind, sigma):
    """sigma_prefilter > 0 (block_components.py:160-162 / :208-211): vigra gaussianSmoothing and
    normalize on the GPU, bit-exact against the oracle's vigra restatement."""
    rng = np.random.default_rng(int(sigma * 10))
    sh = (20, 64, 140)
    x = _volume(sh, 9)
    mask = None
    if kind == 'masked':
        mask = (rng.random(sh) > .1).astype(np.uint8)
        x = (x * 1000).astype(np.float32)
    elif kind == 'channel_sum_u8':
        x = (x * 120).astype(np.uint8) + rng.integers(0, 3, sh).astype(np.uint8)
    elif kind == 'f64_unmasked':
        x = x.astype(np.float64) * 3 - 1
    prenorm = kind in ('unmasked', 'f64_unmasked') or mask is not None
    lab, n = gpu_handle.threshold_components(x, .5, 'greater', mask=mask, normalize=prenorm, sigma=sigma)
    ref, rn = T.block_components(x, .5, 'greater', mask, normalize_input=prenorm and mask is None, sigma=sigma)
    assert rn > 0 and n == rn
    np.testing.assert_array_equal(lab, ref)


def test_block_components_sigma_longer_than_block_refused(gpu_handle):
    from cluster_tools_amd.ctws import CtwsError
    with pytest.raises(CtwsError):
        gpu_handle.threshold_components(np.zeros((4, 32, 32), np.float32), .5, sigma=2.0)


def test_thresholded_components_workflow_sigma_prefilter(tmp_path):
    """The workflow with sigma_prefilter = 1.0 in block_components.config, masked."""
    from conftest import luigi_build
    from cluster_tools_amd.thresholded_components import ThresholdedComponentsWorkflow
    from cluster_tools_amd.thresholded_components.block_components import BlockComponentsLocal
    shape, bs = (32, 96, 160), (16, 48, 64)
    x = _volume(shape, 8)
    path = str(tmp_path / 'data.n5')
    mask = np.zeros(shape, np.uint8)
    mask[:, 10:90, 5:150] = 1
    with vu.file_reader(path) as f:
        f.create_dataset('x', data=x, chunks=(8, 16, 32))
        f.create_dataset('mask', data=mask, chunks=(8, 16, 32))
    bc = BlockComponentsLocal.default_task_config()
    bc['sigma_prefilter'] = 1.0
    wf = ThresholdedComponentsWorkflow(input_path=path, input_key='x', output_path=path, output_key='cc',
                                       assignment_key='ass', threshold=.5, tmp_folder=str(tmp_path / 'tmp'),
                                       config_dir=_configs(tmp_path, bs, {'block_components': bc}), max_jobs=2,
                                       target='local', mask_path=path, mask_key='mask')
    luigi_build(wf, tmp_path / 'tmp')
    ref_seg, ref_ass, _ = T.thresholded_components(x, Blocking([0, 0, 0], list(shape), list(bs)), .5, 'greater',
                                                   mask=mask, sigma=1.0)
    with vu.file_reader(path, 'r') as f:
        np.testing.assert_array_equal(f['ass'][:], ref_ass)
        np.testing.assert_array_equal(f['cc'][:], ref_seg)
    assert len(np.unique(ref_seg)) > 2
