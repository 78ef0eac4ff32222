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


@pytest.mark.parametrize('masked,max_jobs', [(False, 1), (False, 3), (True, 2)])
def test_thresholded_components_workflow_matches_oracle(tmp_path, masked, max_jobs):
    from conftest import luigi_build
    from cluster_tools_amd.thresholded_components import ThresholdedComponentsWorkflow
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
                                       config_dir=_configs(tmp_path, bs), max_jobs=max_jobs, target='local',
                                       mask_path=path if masked else '', mask_key='mask' if masked else '')
    luigi_build(wf, tmp_path / 'tmp')
    ref_seg, ref_ass, ref_off = T.thresholded_components(x, Blocking([0, 0, 0], list(shape), list(bs)), .55,
                                                         'greater', mask=mask)
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
