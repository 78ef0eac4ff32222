"""GPU evaluation (ctws_eval_*, k_eval.hip) against the reference's formulas restated on the
host (cluster_tools_amd/metrics.py = validation_utils.py:60-76, 178-198 with the contingency
of validation_utils.py:9-35), and the EvaluationWorkflow / WatershedFromSeeds task surfaces
end to end on small n5 volumes.  Scores are double sums in a different order: rel. tol 1e-9."""
import json
import os
import sys

import numpy as np
import pytest

from cluster_tools_amd import luigi_compat as luigi
from cluster_tools_amd.metrics import vi_scores, rand_scores
from cluster_tools_amd.utils import volume_utils as vu

pytestmark = pytest.mark.gpu


def _blocky(shape, cell, rng, offset=0):
    """A segmentation of boxes of side ~cell with random ids."""
    z, y, x = np.meshgrid(*[np.arange(s) // c for s, c in zip(shape, cell)], indexing='ij')
    key = (z * 1000 + y) * 1000 + x
    u, inv = np.unique(key, return_inverse=True)
    ids = rng.permutation(len(u)).astype(np.uint64) + np.uint64(offset)
    return ids[inv].reshape(shape)


def _host(seg, gt, ignore):
    vs, vm = vi_scores(seg, gt, [0] if ignore else None)
    are, ri = rand_scores(seg, gt, [0] if ignore else None)
    return {'vi-split': vs, 'vi-merge': vm, 'adapted-rand-error': are, 'rand-index': ri}


def _close(a, b):
    for k in ('vi-split', 'vi-merge', 'adapted-rand-error', 'rand-index'):
        assert abs(a[k] - b[k]) <= 1e-9 * max(1.0, abs(b[k])), (k, a[k], b[k])


def _cases():
    rng = np.random.default_rng(5)
    sh = (20, 96, 80)
    gt = _blocky(sh, (10, 24, 20), rng)
    split = _blocky(sh, (5, 12, 20), rng, offset=10 ** 12)          # splits every gt box
    merge = _blocky(sh, (20, 48, 40), rng)                            # merges gt boxes
    noisy = gt.copy()
    flip = rng.random(sh) < 0.05
    noisy[flip] = rng.integers(1, 50, size=int(flip.sum())).astype(np.uint64)
    gt0 = gt.copy()
    gt0[:, :10] = 0
    # -1 in an int64 volume cast to uint64: the hash tables' empty marker as a real label
    maxlab = noisy.copy()
    maxlab[:, 30:40] = np.uint64(2 ** 64 - 1)
    gtmax = gt.copy()
    gtmax[5:8] = np.uint64(2 ** 64 - 1)
    return {'max_uint64_seg': (maxlab, gt, False), 'max_uint64_gt': (noisy, gtmax, False),
            'max_uint64_both': (maxlab, gtmax, False),
            'identical': (gt.copy(), gt, False), 'split': (split, gt, False), 'merge': (merge, gt, False),
            'noisy': (noisy, gt, False), 'ignore_gt0': (noisy, gt0, True), 'no_ignore_gt0': (noisy, gt0, False)}


CASES = _cases()


@pytest.mark.parametrize('name', sorted(CASES))
def test_eval_matches_reference_formulas(gpu_handle, name):
    seg, gt, ignore = CASES[name]
    got = gpu_handle.evaluate(seg, gt, ignore_gt_zero=ignore)
    ref = _host(seg, gt, ignore)
    print(name, got)
    _close(got, ref)
    assert got['n_points'] == (int((gt != 0).sum()) if ignore else gt.size)
    if name == 'split':
        assert got['vi-split'] > 0.5 and abs(got['vi-merge']) < 1e-9
    if name == 'merge':
        assert got['vi-merge'] > 0.5 and abs(got['vi-split']) < 1e-9


def test_eval_blockwise_and_device_equal_single(gpu_handle):
    import torch
    seg, gt, _ = CASES['noisy']
    single = gpu_handle.evaluate(seg, gt)
    gpu_handle.eval_begin(1 << 16, 1 << 18)
    for z in range(0, seg.shape[0], 7):
        if z % 2:
            gpu_handle.eval_add(seg[z:z + 7], gt[z:z + 7])
        else:  # device tensors for every other block
            gpu_handle.eval_add(torch.from_numpy(seg[z:z + 7].astype(np.int64)).cuda(),
                                torch.from_numpy(gt[z:z + 7].astype(np.int64)).cuda())
    blockwise = gpu_handle.eval_end()
    _close(blockwise, single)


def test_eval_table_full_is_an_error(gpu_handle):
    from cluster_tools_amd.ctws import CtwsError
    seg, gt, _ = CASES['noisy']
    gpu_handle.eval_begin(8, 8)
    gpu_handle.eval_add(seg, gt)
    with pytest.raises(CtwsError):
        gpu_handle.eval_end()


def _configs(tmp_path, task_configs):
    from cluster_tools_amd.cluster_tasks import BaseClusterTask
    cfg_dir = tmp_path / 'configs'
    cfg_dir.mkdir(exist_ok=True)
    g = BaseClusterTask.default_global_config()
    g['shebang'] = '#! ' + sys.executable
    g['block_shape'] = [10, 48, 40]
    (cfg_dir / 'global.config').write_text(json.dumps(g))
    for name, c in task_configs.items():
        (cfg_dir / ('%s.config' % name)).write_text(json.dumps(c))
    return str(cfg_dir)


def test_evaluation_workflow(tmp_path):
    from cluster_tools_amd.evaluation import EvaluationWorkflow
    seg, gt, _ = CASES['ignore_gt0']
    path = str(tmp_path / 'data.n5')
    with vu.file_reader(path) as f:
        f.create_dataset('seg', data=seg, chunks=(10, 48, 40))
        f.create_dataset('gt', data=gt, chunks=(10, 48, 40))
    cfg_dir = _configs(tmp_path, {})
    out = str(tmp_path / 'scores.json')
    wf = EvaluationWorkflow(seg_path=path, seg_key='seg', gt_path=path, gt_key='gt', output_path=out,
                            tmp_folder=str(tmp_path / 'tmp'), config_dir=cfg_dir, max_jobs=1, target='local')
    assert luigi.build([wf], local_scheduler=True)
    with open(out) as f:
        res = json.load(f)
    assert set(res) == {'vi-split', 'vi-merge', 'adapted-rand-error', 'rand-index'}
    _close(res, _host(seg, gt, True))


def test_watershed_from_seeds_task(tmp_path):
    """WatershedFromSeedsLocal on n5: blocks of [10, 48, 40], seeds read from the output file
    (watershed_from_seeds.py:236), against the oracle block by block."""
    from scipy.ndimage import gaussian_filter
    from cluster_tools_amd.synthetic import boundary_map
    from cluster_tools_amd.utils.blocking import Blocking
    from cluster_tools_amd.watershed.watershed_from_seeds import WatershedFromSeedsLocal
    from oracle import oracle as O
    sh = (20, 96, 80)
    x = gaussian_filter(boundary_map(sh, seed=9), 1.0).astype(np.float32)
    rng = np.random.default_rng(4)
    seeds = np.zeros(sh, np.uint64)
    idx = rng.choice(x.size, 300, replace=False)
    seeds.flat[idx] = rng.integers(1, 2 ** 32 - 2, size=300).astype(np.uint64)
    path = str(tmp_path / 'data.n5')
    with vu.file_reader(path) as f:
        f.create_dataset('boundaries', data=x, chunks=(10, 48, 40))
        f.create_dataset('seeds', data=seeds, chunks=(10, 48, 40))
    c = WatershedFromSeedsLocal.default_task_config()
    c['size_filter'] = 10
    cfg_dir = _configs(tmp_path, {'watershed_from_seeds': c})
    t = WatershedFromSeedsLocal(input_path=path, input_key='boundaries', seeds_path=path, seeds_key='seeds',
                                output_path=path, output_key='ws', tmp_folder=str(tmp_path / 'tmp'),
                                config_dir=cfg_dir, max_jobs=2)
    assert luigi.build([t], local_scheduler=True)
    with vu.file_reader(path, 'r') as f:
        res = f['ws'][:]
    blocking = Blocking([0, 0, 0], list(sh), [10, 48, 40])
    ref = np.zeros(sh, np.uint64)
    for bid in range(blocking.numberOfBlocks):
        bb = vu.block_to_bb(blocking.getBlock(bid))
        with O.flood_model():
            ref[bb] = O.ws_from_seeds(c, [dict(input=x[bb], seeds=seeds[bb])])[0]['output']
    np.testing.assert_array_equal(res, ref)
