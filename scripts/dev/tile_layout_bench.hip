// Micro-benchmark: read-modify-write of three bf16 arrays (master hi, lo, momentum) by 64x64
// tiles, the fused MLP backward's access pattern, with the tiles (a) row-strided inside a
// row-major [N][K] matrix (128-B segments K * 2 bytes apart) or (b) stored contiguously (8 KB).
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {
__global__ __launch_bounds__(256) void rmw_tiles(uint16_t* a, uint16_t* b, uint16_t* c, int K,
                                                 int tiled, int n_tiles_k) {
  const int tile = blockIdx.x;
  const int tn = tile / n_tiles_k, tk = tile % n_tiles_k;
  const int tid = threadIdx.x;
  // 64 rows x 64 cols = 4096 elements = 512 uint4 -> 2 per thread
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c8 = tid + 256 * i, r = c8 >> 3, ch = c8 & 7;
    size_t o;
    if (tiled) o = (size_t)tile * 4096 + r * 64 + ch * 8;
    else o = (size_t)(tn * 64 + r) * K + tk * 64 + ch * 8;
    uint4 va = *(uint4*)(a + o), vb = *(uint4*)(b + o), vc = *(uint4*)(c + o);
    va.x += 1; vb.y += 1; vc.z += 1;
    *(uint4*)(a + o) = va;
    *(uint4*)(b + o) = vb;
    *(uint4*)(c + o) = vc;
  }
}
}  // namespace

extern "C" int rmw_tiles_launch(void* a, void* b, void* c, int N, int K, int tiled, void* stream) {
  const int nt = (N / 64) * (K / 64);
  hipLaunchKernelGGL(rmw_tiles, dim3(nt), dim3(256), 0, (hipStream_t)stream, (uint16_t*)a,
                     (uint16_t*)b, (uint16_t*)c, K, tiled, K / 64);
  return (int)hipGetLastError();
}
