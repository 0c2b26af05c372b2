"""Practical HBM ceilings on this GPU: read-only (sum), write-only (fill), copy and in-place
read-modify-write of large bf16 buffers (torch kernels), in TB/s of bytes moved."""
import torch

n = 1 << 29                     # 1 GiB of bf16
a = torch.randn(n, dtype=torch.bfloat16, device="cuda")
b = torch.empty_like(a)


def timed(fn, bytes_moved, it=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    return bytes_moved / (ms * 1e-3) / 1e12


B = 2 * n
print(f"read (sum)        {timed(lambda: a.sum(dtype=torch.float32), B):.2f} TB/s")
print(f"write (fill)      {timed(lambda: b.fill_(1.0), B):.2f} TB/s")
print(f"copy              {timed(lambda: b.copy_(a), 2 * B):.2f} TB/s")
print(f"rmw (add_ scalar) {timed(lambda: b.add_(1.0), 2 * B):.2f} TB/s")
print(f"2 in 1 out (add)  {timed(lambda: torch.add(a, b, out=b), 3 * B):.2f} TB/s")
