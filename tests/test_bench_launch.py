"""bench.py --gpus N starts its N ranks itself: without WORLD_SIZE in the
environment the parent spawns N children with the torchrun environment (RANK, LOCAL_RANK,
WORLD_SIZE, MASTER_ADDR, MASTER_PORT) before anything touches a GPU, and they form one
process group.  --launch-check stops after the group's all-gather (gloo, no GPU)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, extra_env=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT')}
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', str(n), '--launch-check'],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    return r


def test_bench_launches_two_ranks():
    r = _run(2)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line['world_size'] == 2
    # every rank saw world size 2; ranks 0 and 1 with local ranks 0 and 1
    assert sorted(tuple(x) for x in line['ranks']) == [(0, 0, 2), (1, 1, 2)]


def test_bench_launches_four_ranks():
    r = _run(4)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line['world_size'] == 4 and len(line['ranks']) == 4


def test_failing_rank_fails_the_launch():
    # rank 1 dies before joining the group: the parent stops rank 0 (which would wait for it
    # in the rendezvous) and exits with rank 1's code
    r = _run(2, {'CTWS_BENCH_FAIL_RANK': '1'})
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert 'rank 1 exited with 3' in r.stderr
