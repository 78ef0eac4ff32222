#!/usr/bin/env python
"""PCIe probe for the host path: pinned H2D / D2H copy rates alone, in 20 MB pieces, both
directions at once, and under concurrent host-memory load (numpy copies on CPU threads)."""
import json
import threading
import time

import numpy as np
import torch


def main():
    dev = torch.device('cuda', 0)
    nb = 1 << 30
    hin = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    hout = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    din = torch.empty(nb, dtype=torch.uint8, device=dev)
    dout = torch.empty(nb, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    piece = 20 << 20

    def run(h2d, d2h, pieces=False, reps=3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            if h2d:
                with torch.cuda.stream(s1):
                    if pieces:
                        for o in range(0, nb, piece):
                            din[o:o + piece].copy_(hin[o:o + piece], non_blocking=True)
                    else:
                        din.copy_(hin, non_blocking=True)
            if d2h:
                with torch.cuda.stream(s2):
                    hout.copy_(dout, non_blocking=True)
        torch.cuda.synchronize()
        return round(nb * reps / (time.perf_counter() - t0) / 1e9, 1)

    run(True, True)
    res = {'h2d': run(True, False), 'h2d_pieces': run(True, False, True), 'd2h': run(False, True),
           'duplex': run(True, True), 'duplex_pieces': run(True, True, True)}
    # host memory load: T threads each copying a 512 MB numpy array back and forth
    for T in (4, 8, 12):
        stop = [False]
        bufs = [(np.ones(64 << 20, np.float64), np.empty(64 << 20, np.float64)) for _ in range(T)]
        moved = [0] * T

        def load(k):
            a, b = bufs[k]
            while not stop[0]:
                np.copyto(b, a)
                moved[k] += 2 * a.nbytes

        th = [threading.Thread(target=load, args=(k,)) for k in range(T)]
        for t in th:
            t.start()
        time.sleep(0.2)
        m0, t0 = sum(moved), time.perf_counter()
        r = {'h2d': run(True, False), 'duplex': run(True, True)}
        r['cpu_copy_gbs'] = round((sum(moved) - m0) / (time.perf_counter() - t0) / 1e9, 1)
        stop[0] = True
        for t in th:
            t.join()
        res['load_%d_threads' % T] = r
    print(json.dumps(res))


if __name__ == '__main__':
    main()
