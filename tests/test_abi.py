"""The C-ABI library builds, loads and exports every entry point of include/ctws.h, and the
ctypes mirror matches the C struct layout.  CPU only: no compute call is made."""
import ctypes as C
import os
import re
import subprocess

import pytest

from cluster_tools_amd import _abi, ctws

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'ctws.h')


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r'^\s*(?:int|void|const char\*)\s+(ctws_\w+)\(', src, re.M)))


def test_header_declares_entry_points():
    fns = declared_functions()
    for f in ('ctws_open', 'ctws_close', 'ctws_ws_blocks', 'ctws_ws_blocks_device', 'ctws_unique_u64',
              'ctws_unique_counts_u64', 'ctws_lookup_u64', 'ctws_eval_begin'):
        assert f in fns


def test_library_exports_every_declared_symbol():
    lib = ctws.lib()
    for f in declared_functions():
        assert hasattr(lib, f), f
    assert set(declared_functions()) == set(ctws.EXPORTED_SYMBOLS)
    assert lib.ctws_abi_version() == ctws.ABI_VERSION == 2


def test_struct_layout_matches_header(tmp_path):
    prog = tmp_path / 'sz.c'
    prog.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "ctws.h"\nint main(void){'
                    'printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(ctws_cfg), sizeof(ctws_block), '
                    'offsetof(ctws_cfg, block_shape), offsetof(ctws_block, output), '
                    'offsetof(ctws_block, status), offsetof(ctws_cfg, pass_id));return 0;}')
    exe = tmp_path / 'sz'
    subprocess.check_call(['gcc', '-I', os.path.join(ROOT, 'include'), str(prog), '-o', str(exe)])
    vals = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    assert vals == [C.sizeof(_abi.CtwsCfg), C.sizeof(_abi.CtwsBlock), _abi.CtwsCfg.block_shape.offset,
                    _abi.CtwsBlock.output.offset, _abi.CtwsBlock.status.offset, _abi.CtwsCfg.pass_id.offset]


def test_make_cfg_defaults_follow_reference_inline_defaults():
    cfg = _abi.make_cfg({}, (64, 256, 256))
    assert cfg.threshold == .5 and cfg.alpha == .8 and cfg.size_filter == 25
    assert cfg.apply_dt_2d == 1 and cfg.apply_ws_2d == 1 and cfg.has_pixel_pitch == 0
    assert list(cfg.sigma_seeds) == [2., 2., 2.] and cfg.sigma_seeds_is_list == 0
    assert cfg.channel_end == -1 and cfg.agglomerate_channels == 0
    cfg = _abi.make_cfg({'sigma_seeds': (.5, 2., 2.), 'pixel_pitch': (10, 1, 1), 'channel_end': 2}, (1, 2, 3))
    assert cfg.sigma_seeds_is_list == 1 and list(cfg.pixel_pitch) == [10., 1., 1.] and cfg.channel_end == 2
    with pytest.raises(ValueError):
        _abi.make_cfg({'sigma_seeds': (1., 2.)}, (1, 2, 3))


def test_no_gpu_fails_loudly():
    """The product path has no CPU fallback: without a GPU, opening the library raises."""
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    with pytest.raises(ctws.CtwsError):
        ctws.Handle(0)
