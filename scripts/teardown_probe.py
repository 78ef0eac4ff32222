#!/usr/bin/env python
"""How long a watershed job process takes to exit after its last log line: a child does what a
relabel job does (HIP via libctws and torch, a gloo group, device tensors) and prints the time
of its last line; the parent measures when the child has exited."""
import subprocess
import sys
import time

CHILD = r'''
import time, os, numpy as np, torch, torch.distributed as dist
from datetime import timedelta
from cluster_tools_amd import ctws
t0 = time.time()
dist.init_process_group('gloo', init_method='tcp://127.0.0.1:%s' % os.environ['PORT'], rank=0, world_size=1,
                        timeout=timedelta(seconds=60))
with ctws.Handle(0) as h:
    x = torch.arange(1 << 24, device='cuda', dtype=torch.int64)
    u = h.unique_u64_device(x)
    y = x.cpu().numpy()
dist.barrier()
dist.destroy_process_group()
print('work %.3f' % (time.time() - t0))
print('last %.6f' % time.time(), flush=True)
if os.environ.get('FAST_EXIT') == '1':
    os._exit(0)
'''


def main():
    import os
    for fast in ('0', '1'):
        env = dict(os.environ, PORT='29533', FAST_EXIT=fast)
        t = time.time()
        p = subprocess.run([sys.executable, '-c', CHILD], env=env, capture_output=True, text=True)
        end = time.time()
        last = [float(line.split()[1]) for line in p.stdout.splitlines() if line.startswith('last ')]
        print('fast_exit %s rc %i: process %.3f s, exit after last line %.3f s; %s' % (
            fast, p.returncode, end - t, end - last[0] if last else -1, p.stdout.splitlines()[:1]))
        if p.returncode:
            print(p.stderr[-2000:])


if __name__ == '__main__':
    main()
