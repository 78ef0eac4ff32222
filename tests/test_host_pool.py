"""The host path's worker pool (cluster_tools_amd/csrc/host_pool.h): back-to-back parallel_for
calls run every index exactly once and return only after all of them (a worker could
carry a claim across generations).  Host code only: built with g++, once plain and once under
ThreadSanitizer when the toolchain has it."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, 'native', 'pool_stress.cpp')


def _build(tmp_path, flags):
    exe = str(tmp_path / 'pool_stress')
    r = subprocess.run(['g++', '-std=c++17', '-O1', '-g', '-pthread'] + flags + [SRC, '-o', exe],
                       capture_output=True, text=True)
    return exe if r.returncode == 0 else None


def test_pool_plain(tmp_path):
    exe = _build(tmp_path, [])
    assert exe, 'g++ failed'
    r = subprocess.run([exe, '20000'], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith('ok')


def test_pool_tsan(tmp_path):
    exe = _build(tmp_path, ['-fsanitize=thread'])
    if exe is None:
        pytest.skip('g++ has no ThreadSanitizer runtime here')
    r = subprocess.run([exe, '3000'], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, TSAN_OPTIONS='halt_on_error=1'))
    if 'FATAL: ThreadSanitizer' in r.stderr and 'unexpected memory mapping' in r.stderr:
        pytest.skip('ThreadSanitizer cannot run in this environment')
    assert r.returncode == 0, r.stderr[-3000:]
