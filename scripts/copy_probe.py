"""H2D / D2H copy rate from pinned memory and its interference with a concurrent streaming
kernel (is the copy an SDMA transfer or a blit kernel?)."""
import time
import torch

n = 1 << 29  # 2 GiB of float32
host = torch.empty(n, dtype=torch.float32).pin_memory()
dev = torch.empty(n, dtype=torch.float32, device='cuda')
big = torch.rand(2 * n, device='cuda')
s_copy = torch.cuda.Stream()
torch.cuda.synchronize()


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


t_h2d = timed(lambda: dev.copy_(host, non_blocking=True))
t_d2h = timed(lambda: host.copy_(dev, non_blocking=True))
t_k = timed(lambda: big.sum())


def both():
    with torch.cuda.stream(s_copy):
        dev.copy_(host, non_blocking=True)
    for _ in range(20):
        big.sum()


t_both = timed(both, reps=2)
print('H2D %.1f GB/s, D2H %.1f GB/s, kernel %.2f ms, 20 kernels + concurrent H2D %.1f ms (alone %.1f / %.1f ms)'
      % (4 * n / t_h2d / 1e9, 4 * n / t_d2h / 1e9, t_k * 1e3, t_both * 1e3, 20 * t_k * 1e3, t_h2d * 1e3))
