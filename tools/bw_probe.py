"""HBM bandwidth probe: torch read-only (sum), copy and write (fill) rates on the box, as the
practical ceiling the memory-bound kernels are compared against."""
import torch

def t(fn, it=20):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it

for mb in (256, 1024):
    n = mb * 2 ** 20 // 4
    a = torch.randn(n, device="cuda")
    b = torch.empty_like(a)
    ms = t(lambda: a.sum())
    print(f"{mb:5d} MB read (sum)   {4 * n / ms / 1e6:7.0f} GB/s")
    ms = t(lambda: b.copy_(a))
    print(f"{mb:5d} MB copy (r+w)   {8 * n / ms / 1e6:7.0f} GB/s")
    ms = t(lambda: b.fill_(1.0))
    print(f"{mb:5d} MB write (fill) {4 * n / ms / 1e6:7.0f} GB/s")
