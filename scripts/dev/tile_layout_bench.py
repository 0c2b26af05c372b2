"""Drive tile_layout_bench.hip: RMW bandwidth of row-strided vs contiguous 64x64 tiles."""
import ctypes
import os
import sys

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tile_layout_bench.so"))
lib.rmw_tiles_launch.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
for K in (256, 512, 1024):
    N = (1 << 27) // K      # 128 Mi elements per array (256 MB bf16)
    arrs = [torch.zeros(N * K, dtype=torch.int16, device="cuda") for _ in range(3)]
    s = torch.cuda.current_stream().cuda_stream
    for tiled in (0, 1):
        run = lambda: lib.rmw_tiles_launch(*[a.data_ptr() for a in arrs], N, K, tiled, s)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        tb = 3 * 2 * 2 * N * K / (ms * 1e-3) / 1e12
        print(f"K={K:5d} {'tiled  ' if tiled else 'strided'}: {ms * 1e3:8.1f} us  {tb:.2f} TB/s",
              flush=True)
