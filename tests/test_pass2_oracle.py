"""CPU checks of the pass-2 scenarios (oracle only): the structural invariants the reference's
own test asserts (test/watershed/test_watershed.py:53-70) hold for `_ws_pass2` outputs, and the
pass-1 labels in the halo are reused as seeds (stitching)."""
import numpy as np
import pytest

from oracle import oracle as O
from pass2_cases import scenario


@pytest.mark.parametrize('name', ['3d', '2d', '3d_mask', '3d_wrap'])
def test_oracle_pass2_invariants(name):
    config, block_shape, blocks = scenario(name)
    res = O.ws_blocks(config, block_shape, blocks, pass_id=1)
    for b, r in zip(blocks, res):
        assert r['status'] == 0
        out = r['output']
        assert out.shape == tuple(b['inner_shape'])
        if b.get('mask') is None:
            assert (out != 0).all()
        # pass-2 values are uint32 (takeDict of the uint32 seeds, Appendix B.2)
        assert out.max() < 2 ** 32
        init = b['initial_seeds']
        ids = set(np.unique(init[init != 0] & np.uint64(0xFFFFFFFF)).tolist())
        assert ids & set(np.unique(out).tolist())
        assert r['max_label'] == int(out.max())



@pytest.mark.parametrize('name', ['2d_collide', '2d_collide_mask'])
def test_oracle_collide_scenario_merges(name):
    """The scenario really exercises the merge: every block offset is 0 mod 2^32, so new seeds
    and initial ids share uint32 values and relabelConsecutive merges segments -- fewer distinct
    ids than the same blocks with consecutive block ids (scenario without the stride)."""
    config, block_shape, blocks = scenario(name)
    V = int(np.prod(block_shape))
    assert all((b['block_id'] * V) % 2 ** 32 == 0 for b in blocks)
    plain_name = '2d_mask' if name.endswith('mask') else '2d'
    res = O.ws_blocks(config, block_shape, blocks, pass_id=1)
    pc, pbs, pblocks = scenario(plain_name)
    plain = O.ws_blocks(pc, pbs, pblocks, pass_id=1)
    fewer = 0
    for r, p in zip(res, plain):
        assert r['status'] == p['status'] == 0
        fewer += len(np.unique(r['output'])) < len(np.unique(p['output']))
    assert fewer > 0
