"""BASELINE config 1 at its real block shape: the reference's own workflow test
(test/watershed/test_watershed.py:39-100) — WatershedWorkflow, target 'local', global
block_shape [10, 256, 256], the default watershed task config, a 4-D (channel, z, y, x) float32
affinity map aggregated by the channel mean — on a synthetic 3 x 20 x 512 x 512 volume (the
reference's ~100 x 1024 x 1024 test data is not available here; the block shape, configs and
checks are the test's).  Checks the test's `_check_result` invariants (:53-70) for the single-
and the two-pass workflow, and the single-pass watershed stage against the oracle block by block
(VI <= 0.01, BASELINE.json north_star).
"""
import json
import sys

import numpy as np
import pytest

from cluster_tools_amd import luigi_compat as luigi
from cluster_tools_amd.utils import volume_utils as vu
from cluster_tools_amd.utils.blocking import Blocking
from cluster_tools_amd.synthetic import boundary_map
from cluster_tools_amd.metrics import vi_scores
from oracle import oracle as O
from conftest import luigi_build

pytestmark = pytest.mark.gpu

SHAPE = (20, 512, 512)
BLOCK_SHAPE = [10, 256, 256]


def _setup(tmp_path):
    from cluster_tools_amd.watershed.watershed import WatershedLocal
    cfg_dir = tmp_path / 'configs'
    cfg_dir.mkdir()
    g = WatershedLocal.default_global_config()
    g['shebang'] = '#! ' + sys.executable
    g['block_shape'] = BLOCK_SHAPE
    (cfg_dir / 'global.config').write_text(json.dumps(g))
    # three "affinity" channels: the same cells seen with different noise
    x = np.stack([boundary_map(SHAPE, seed=11 + c) for c in range(3)])
    inp = str(tmp_path / 'data.n5')
    with vu.file_reader(inp) as f:
        f.create_dataset('affinities', data=x, chunks=(1, 10, 256, 256))
    return str(cfg_dir), inp, x


def _n_ids_and_ccs(res):
    cc, _ = O.label_with_background(res.astype('uint32'))
    return len(np.unique(res)), len(np.unique(cc))


def _check_result(res):
    """test_watershed.py:53-70 without a mask."""
    assert res.shape == SHAPE
    assert not np.allclose(res, 0)
    assert 0 not in res
    n_ids, n_cc = _n_ids_and_ccs(res)
    assert n_ids == n_cc, "disconnected segments"


def _oracle_volume(x, c):
    """The reference's `_ws_block` over the volume (no halo by default), via the oracle."""
    blocking = Blocking([0, 0, 0], list(SHAPE), BLOCK_SHAPE)
    out = np.zeros(SHAPE, np.uint64)
    for bid in range(blocking.numberOfBlocks):
        bb = vu.block_to_bb(blocking.getBlock(bid))
        b = dict(input=x[(slice(None),) + bb], block_id=bid, inner_begin=[0, 0, 0],
                 inner_shape=[s.stop - s.start for s in bb], crop_relabel=False)
        r = O.ws_blocks(c, BLOCK_SHAPE, [b])[0]
        if r['status'] in (0, 2):
            out[bb] = r['output']
    return out


def test_config1_watershed_workflow(tmp_path):
    from cluster_tools_amd.watershed import WatershedWorkflow
    from cluster_tools_amd.watershed.watershed import WatershedLocal
    cfg_dir, inp, x = _setup(tmp_path)
    out = str(tmp_path / 'ws.n5')
    ws = WatershedLocal(input_path=inp, input_key='affinities', output_path=out, output_key='ws_raw',
                        config_dir=cfg_dir, tmp_folder=str(tmp_path / 'tmp_ws'), max_jobs=8)
    luigi_build(ws, tmp_path / 'tmp')
    with vu.file_reader(out, 'r') as f:
        raw = f['ws_raw'][:]
    ref = _oracle_volume(x, WatershedLocal.default_task_config())
    vis, vim = vi_scores(raw, ref)
    assert vis + vim <= 0.01, (vis, vim)
    wf = WatershedWorkflow(input_path=inp, input_key='affinities', output_path=out, output_key='ws',
                           config_dir=cfg_dir, tmp_folder=str(tmp_path / 'tmp'), target='local', max_jobs=8)
    luigi_build(wf, tmp_path / 'tmp')
    with vu.file_reader(out, 'r') as f:
        res = f['ws'][:]
    _check_result(res.astype('uint64'))


def test_config1_two_pass_workflow(tmp_path):
    from cluster_tools_amd.watershed import WatershedWorkflow
    cfg_dir, inp, _ = _setup(tmp_path)
    out = str(tmp_path / 'ws.n5')
    wf = WatershedWorkflow(input_path=inp, input_key='affinities', output_path=out, output_key='ws',
                           config_dir=cfg_dir, tmp_folder=str(tmp_path / 'tmp'), target='local', max_jobs=8,
                           two_pass=True)
    luigi_build(wf, tmp_path / 'tmp')
    with vu.file_reader(out, 'r') as f:
        res = f['ws'][:]
    assert res.shape == SHAPE and not np.allclose(res, 0) and 0 not in res
