"""CPU tests of the drop-in task surface: blocking, checkerboard, n5/zarr I/O, job configs,
the log protocol and retry (mirroring the reference's test/utils and test/retry tests)."""
import json
import os
import sys

import numpy as np
import pytest

from cluster_tools_amd import luigi_compat as luigi
from cluster_tools_amd.utils.blocking import Blocking
from cluster_tools_amd.utils import volume_utils as vu
from cluster_tools_amd.utils.function_utils import tail
from cluster_tools_amd.utils import parse_utils as pu


def test_blocking_c_order_and_halo():
    b = Blocking([0, 0, 0], [100, 100, 60], [64, 32, 32])
    assert b.blocksPerAxis == [2, 4, 2] and b.numberOfBlocks == 16
    assert b.getBlock(1).begin == [0, 0, 32] and b.getBlock(1).end == [64, 32, 60]
    assert b.getBlock(2).begin == [0, 32, 0]
    bh = b.getBlockWithHalo(3, [8, 8, 8])
    assert bh.outerBlock.begin == [0, 24, 24] and bh.outerBlock.end == [72, 72, 60]
    assert bh.innerBlockLocal.begin == [0, 8, 8] and bh.innerBlockLocal.end == [64, 40, 36]
    assert b.getNeighborId(0, 0, False) == 8 and b.getNeighborId(0, 2, True) == -1
    assert b.coordinatesToBlockId([70, 40, 40]) == 11
    assert list(b.getBlockIdsOverlappingBoundingBox([0, 0, 0], [10, 40, 10])) == [0, 2]


def _checkerboard_recursive(blocking):
    """The reference's recursive DFS (utils/volume_utils.py:142-164), for comparison."""
    blocks_a, blocks_b, all_blocks = [0], [], [0]

    def recurse(current, insert_list):
        other = blocks_a if insert_list is blocks_b else blocks_b
        for dim in range(3):
            ngb = blocking.getNeighborId(current, dim, False)
            if ngb != -1 and ngb not in all_blocks:
                insert_list.append(ngb)
                all_blocks.append(ngb)
                recurse(ngb, other)
    recurse(0, blocks_b)
    return blocks_a, blocks_b


@pytest.mark.parametrize('grid', [(2, 2, 2), (4, 2, 2), (2, 6, 4), (5, 4, 3)])
def test_checkerboard_matches_recursive_reference(grid):
    b = Blocking([0, 0, 0], [g * 10 for g in grid], [10, 10, 10])
    ref = _checkerboard_recursive(b)
    a, bb = vu.make_checkerboard_block_lists(b)
    assert (a, bb) == ref
    for lst, parity in ((a, 0), (bb, 1)):
        assert all(sum(b.blockCoordinates(x)) % 2 == parity for x in lst)


def test_checkerboard_odd_block_count_asserts():
    b = Blocking([0, 0, 0], [30, 30, 30], [10, 10, 10])
    with pytest.raises(AssertionError):
        vu.make_checkerboard_block_lists(b)


def test_checkerboard_large_grid_no_recursion_limit():
    b = Blocking([0, 0, 0], [32 * 64, 8 * 256, 8 * 256], [64, 256, 256])  # config 5: 2048 blocks
    a, bb = vu.make_checkerboard_block_lists(b)
    assert len(a) == len(bb) == 1024


@pytest.mark.parametrize('ext', ['n5', 'zr'])
def test_file_reader_roundtrip(tmp_path, ext):
    path = str(tmp_path / ('data.' + ext))
    x = np.random.RandomState(0).randint(0, 1 << 40, size=(37, 41, 23)).astype('uint64')
    with vu.file_reader(path) as f:
        ds = f.require_dataset('a/b', shape=x.shape, chunks=(8, 16, 8), compression='gzip', dtype='uint64')
        ds[:] = x
        ds[3:11, 5:40, 2:9] = 7
    x[3:11, 5:40, 2:9] = 7
    with vu.file_reader(path, 'r') as f:
        assert np.array_equal(f['a/b'][:], x)
        assert np.array_equal(f['a/b'][5:30, 1, :], x[5:30, 1, :])
    assert vu.get_shape(path, 'a/b') == x.shape


def test_n5_layout_is_standard(tmp_path):
    """attributes.json in F order and big-endian chunks with the n5 header."""
    import gzip
    path = str(tmp_path / 'd.n5')
    with vu.file_reader(path) as f:
        ds = f.create_dataset('x', shape=(3, 4, 5), chunks=(3, 4, 5), dtype='uint16', compression='gzip')
        ds[:] = np.arange(60, dtype='uint16').reshape(3, 4, 5)
    meta = json.load(open(os.path.join(path, 'x', 'attributes.json')))
    assert meta['dimensions'] == [5, 4, 3] and meta['dataType'] == 'uint16'
    raw = open(os.path.join(path, 'x', '0', '0', '0'), 'rb').read()
    assert list(np.frombuffer(raw[:4], '>u2')) == [0, 3] and list(np.frombuffer(raw[4:16], '>u4')) == [5, 4, 3]
    data = np.frombuffer(gzip.decompress(raw[16:]), '>u2')
    assert np.array_equal(data, np.arange(60))


@pytest.mark.parametrize('ext', ['n5', 'zr'])
def test_read_many_missing_chunks_and_overlaps(tmp_path, ext):
    """read_many: overlapping indices share chunks; chunks never written read as the fill."""
    path = str(tmp_path / ('d.' + ext))
    x = np.arange(20 * 30 * 40, dtype='float32').reshape(20, 30, 40)
    with vu.file_reader(path) as f:
        ds = f.create_dataset('x', shape=x.shape, chunks=(8, 8, 8), dtype='float32', compression='gzip')
        ds[0:8, :, :] = x[0:8]
        ds.n_threads = 3
        idx = [np.s_[2:19, 3:29, 5:33], np.s_[0:20, 0:30, 0:40], np.s_[7:9, 4, 1:39], np.s_[:, :, :]]
        got = ds.read_many(idx)
    exp = np.zeros_like(x)
    exp[0:8] = x[0:8]
    for i, g in zip(idx, got):
        assert np.array_equal(g, exp[i])
    # 4-D (channel-first) input with a channel range, as _read_block indexes it
    x4 = np.arange(3 * 9 * 20 * 21, dtype='float32').reshape(3, 9, 20, 21)
    with vu.file_reader(path) as f:
        ds = f.create_dataset('x4', shape=x4.shape, chunks=(1, 4, 8, 8), dtype='float32', compression='gzip')
        ds[:] = x4
        ds.n_threads = 4
        idx = [(slice(1, 3), slice(0, 9), slice(2, 18), slice(0, 21)), (slice(0, None), slice(3, 4), slice(5, 6), slice(7, 20))]
        got = ds.read_many(idx)
    for i, g in zip(idx, got):
        assert np.array_equal(g, x4[i])


@pytest.mark.parametrize('codec', ['libdeflate', 'zlib'])
@pytest.mark.parametrize('ext,comp', [('n5', 'gzip'), ('n5', 'zlib'), ('zr', 'gzip'), ('zr', 'zlib'), ('n5', 'raw')])
def test_chunk_codecs_interoperate(tmp_path, monkeypatch, codec, ext, comp):
    """Chunks written with either codec (libdeflate, or zlib when it is absent) read back with
    the other and with Python's zlib / gzip; float chunks come back native-endian."""
    import zlib
    from cluster_tools_amd.io import deflate
    if codec == 'libdeflate' and not deflate.available():
        pytest.skip('libdeflate.so.0 not installed')
    if codec == 'zlib':
        monkeypatch.setattr(deflate, '_lib', False)
    path = str(tmp_path / ('d.' + ext))
    rng = np.random.RandomState(1)
    x = rng.rand(19, 33, 21).astype('float32')
    lab = (np.arange(19 * 33 * 21, dtype='uint64') // 50 + (1 << 40)).reshape(19, 33, 21)
    with vu.file_reader(path) as f:
        f.create_dataset('x', shape=x.shape, chunks=(8, 16, 16), dtype='float32', compression=comp)[:] = x
        f.create_dataset('l', shape=x.shape, chunks=(8, 16, 16), dtype='uint64', compression=comp)[:] = lab
    monkeypatch.setattr(deflate, '_lib', None if codec == 'zlib' else False)
    with vu.file_reader(path, 'r') as f:
        rx = f['x'][:]
        assert rx.dtype == np.float32 and rx.dtype.isnative and np.array_equal(rx, x)
        assert np.array_equal(f['l'][:], lab)
    if comp != 'raw':
        # every chunk file is a plain gzip / zlib stream
        name = os.path.join(path, 'l', '0', '0', '0') if ext == 'n5' else os.path.join(path, 'l', '0.0.0')
        raw = open(name, 'rb').read()
        payload = raw[16:] if ext == 'n5' else raw
        assert (payload[:2] == b'\x1f\x8b') == (comp == 'gzip')
        zlib.decompress(payload, 47)


def test_tail(tmp_path):
    p = tmp_path / 'out.txt'
    p.write_text('abcd\n1234\n5678\nwxyz\n')
    assert tail(str(p), 3) == ['1234', '5678', 'wxyz']


def test_log_protocol_parsing(tmp_path):
    p = tmp_path / 'w_0.log'
    p.write_text('2020-01-01 10:00:00.000: start\n2020-01-01 10:00:01.000: processed block 3\n'
                 '2020-01-01 10:00:05.500: processed block 7\n2020-01-01 10:00:06.000: processed job 0\n')
    assert pu.parse_job(str(p), 0) and not pu.parse_job(str(p), 1)
    assert pu.parse_blocks(str(p)) == [3, 7]
    assert pu.parse_runtime(str(p)) == 6.0
    q = tmp_path / 'w_1.log'
    q.write_text('2020-01-01 10:00:00.000: processed block 1\n')
    assert not pu.parse_job(str(q), 1)
    assert pu.parse_blocks_task(str(tmp_path / 'w_'), 2, [0]) == [1]


def _configs(tmp_path, block_shape, **gc):
    cfg_dir = tmp_path / 'configs'
    cfg_dir.mkdir()
    from cluster_tools_amd.cluster_tasks import BaseClusterTask
    g = BaseClusterTask.default_global_config()
    g.update({'shebang': '#! ' + sys.executable, 'block_shape': list(block_shape)}, **gc)
    (cfg_dir / 'global.config').write_text(json.dumps(g))
    return str(cfg_dir)


def test_retry_reruns_failed_blocks(tmp_path):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from failing_task import FailingTaskLocal
    cfg = _configs(tmp_path, (10, 32, 32), max_num_retries=1)
    out = str(tmp_path / 'out.n5')
    task = FailingTaskLocal(output_path=out, output_key='data', shape=[40, 64, 64], config_dir=cfg,
                            tmp_folder=str(tmp_path / 'tmp'), max_jobs=4)
    assert luigi.build([task], local_scheduler=True)
    with vu.file_reader(out, 'r') as f:
        assert (f['data'][:] == 1).all()
    cfgs = sorted(os.listdir(str(tmp_path / 'tmp')))
    assert 'failing_task_job_0.config' in cfgs
    blocks = json.load(open(str(tmp_path / 'tmp' / 'failing_task_job_1.config')))['block_list']
    assert all(b % 4 == 1 for b in blocks)   # the retry re-ran exactly the failed blocks
    assert os.path.exists(str(tmp_path / 'tmp' / 'failing_task.log'))


def test_no_retry_without_budget_renames_log(tmp_path):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from failing_task import FailingTaskLocal
    cfg = _configs(tmp_path, (10, 32, 32), max_num_retries=0)
    task = FailingTaskLocal(output_path=str(tmp_path / 'o.n5'), output_key='data', shape=[40, 64, 64],
                            config_dir=cfg, tmp_folder=str(tmp_path / 'tmp'), max_jobs=4)
    assert not luigi.build([task], local_scheduler=True)
    assert os.path.exists(str(tmp_path / 'tmp' / 'failing_task_failed.log'))


@pytest.mark.parametrize('relabel_in_job', [True, False])
def test_watershed_task_writes_job_configs_and_fails_loudly_without_gpu(tmp_path, relabel_in_job):
    """Without a GPU the job processes die before 'processed job': the task raises, the
    workflow returns False and the task log is renamed (no silent CPU fallback).  With the
    relabel in the jobs (job_relabel.py) the jobs take consecutive blocks and fail together
    through their process group instead of waiting for each other."""
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    from cluster_tools_amd.synthetic import boundary_map
    from cluster_tools_amd.watershed import WatershedWorkflow
    cfg = _configs(tmp_path, (16, 32, 32))
    inp = str(tmp_path / 'in.n5')
    with vu.file_reader(inp) as f:
        f.create_dataset('raw', data=boundary_map((32, 64, 64), seed=2), chunks=(16, 32, 32))
    wf = WatershedWorkflow(input_path=inp, input_key='raw', output_path=str(tmp_path / 'ws.n5'), output_key='ws',
                           config_dir=cfg, tmp_folder=str(tmp_path / 'tmp'), target='local', max_jobs=2,
                           relabel_in_job=relabel_in_job)
    assert not luigi.build([wf], local_scheduler=True)
    tmp = tmp_path / 'tmp'
    job0 = json.load(open(str(tmp / 'watershed_job_0.config')))
    blocks0 = [0, 1, 2, 3] if relabel_in_job else [0, 2, 4, 6]
    assert job0['block_list'] == blocks0 and job0['threshold'] == .5 and job0['block_shape'] == [16, 32, 32]
    assert ('relabel' in job0) == relabel_in_job
    assert os.path.exists(str(tmp / 'watershed_failed.log'))
    assert os.path.exists(str(tmp / 'watershed.py'))
    assert open(str(tmp / 'watershed.py')).readline().strip() == '#! ' + sys.executable


def test_keep_on_device_divides_free_memory_across_the_jobs_of_a_gpu(monkeypatch):
    """watershed._keep_on_device: a job keeps its uint64 outputs in HBM only while they fit in
    its share of half the free memory -- the relabel's n_jobs spread over the visible GPUs."""
    import torch
    from cluster_tools_amd.watershed import watershed as ws
    blocking = Blocking([0, 0, 0], [64, 64, 64], [32, 32, 32])
    need = 8 * 8 * 32 ** 3                    # all 8 inner blocks, uint64
    cfg = {'block_shape': [32, 32, 32], 'halo': [4, 4, 4], 'relabel': {'n_jobs': 4}}
    monkeypatch.setattr(torch.cuda, 'device_count', lambda: 1)
    monkeypatch.setattr(torch.cuda, 'mem_get_info', lambda d=None: (2 * 4 * need, 1 << 40))
    assert ws._keep_on_device(blocking, list(range(8)), cfg)
    monkeypatch.setattr(torch.cuda, 'mem_get_info', lambda d=None: (2 * 4 * need - 1, 1 << 40))
    assert not ws._keep_on_device(blocking, list(range(8)), cfg)
    monkeypatch.setattr(torch.cuda, 'device_count', lambda: 2)   # 2 jobs per GPU now
    assert ws._keep_on_device(blocking, list(range(8)), cfg)
    assert not ws._keep_on_device(blocking, list(range(8)), dict(cfg, keep_on_device=False))


def test_split_blocks_consecutive_keeps_block_ids():
    """consecutive runs are runs of the block LIST (a ROI or a block_list_path
    gives ids that are not 0..N-1), the round-robin split is block_list[j::n_jobs]
    (cluster_tasks.py:328 of the reference)."""
    from cluster_tools_amd.cluster_tasks import split_blocks
    bl = [3, 4, 7, 8, 11, 12, 30]
    runs = split_blocks(bl, 3, consecutive=True)
    assert runs == [[3, 4, 7], [8, 11], [12, 30]]
    assert sum(runs, []) == bl
    assert split_blocks(bl, 3) == [[3, 8, 30], [4, 11], [7, 12]]


@pytest.mark.parametrize('retries', [0, 1])
def test_workflow_keeps_retry_with_max_num_retries(tmp_path, retries):
    """the in-job relabel numbers all blocks at once and cannot re-run one, so
    with max_num_retries > 0 WatershedWorkflow runs watershed + RelabelWorkflow, whose watershed
    task retries failed blocks as the reference's does (cluster_tasks.py:127-142)."""
    from cluster_tools_amd.watershed import WatershedWorkflow
    from cluster_tools_amd.relabel import RelabelWorkflow
    cfg = _configs(tmp_path, (16, 32, 32))
    g = json.load(open(os.path.join(cfg, 'global.config')))
    g['max_num_retries'] = retries
    json.dump(g, open(os.path.join(cfg, 'global.config'), 'w'))
    wf = WatershedWorkflow(input_path='in.n5', input_key='raw', output_path='ws.n5', output_key='ws',
                           config_dir=cfg, tmp_folder=str(tmp_path / 'tmp'), target='local', max_jobs=2)
    dep = wf.requires()
    if retries:
        assert isinstance(dep, RelabelWorkflow)
    else:
        assert not isinstance(dep, RelabelWorkflow) and dep.assignment_key == 'relabel_watershed'
