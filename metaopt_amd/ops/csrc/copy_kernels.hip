// Batched device copies for the sweep's checkpoint pool (one launch per sync instead of one
// framework copy per tensor and member).
//
// A descriptor moves n f32 values src -> dst and optionally also writes their bf16 image to dst16
// (restoring a member's bf16 working weights in the same pass that restores its f32 master copy).
// Work is split into 4096-element chunks listed on the host, so a launch needs no per-descriptor
// grid sizing and stays balanced however ragged the member sizes are.
#include "common.h"

using namespace mopt;

extern "C" {

struct CopyDesc {       // 32 bytes, mirrored by metaopt_amd/ops/ckpt.py
  const float* src;
  float* dst;
  bf16_t* dst16;        // nullptr: no bf16 image
  int64_t n;            // multiple of 4
};

struct CopyChunk {      // 16 bytes
  int32_t desc;
  int32_t pad;
  int64_t start;        // element offset inside the descriptor
};

}  // extern "C"

namespace {

constexpr int kChunk = 4096;

__global__ __launch_bounds__(256) void multi_copy_kernel(const CopyDesc* __restrict__ descs,
                                                         const CopyChunk* __restrict__ chunks) {
  const CopyChunk c = chunks[blockIdx.x];
  const CopyDesc d = descs[c.desc];
  const int64_t end = min((int64_t)kChunk, d.n - c.start);
  for (int64_t i = 4 * threadIdx.x; i < end; i += 4 * 256) {
    const f32x4 v = *(const f32x4*)(d.src + c.start + i);
    *(f32x4*)(d.dst + c.start + i) = v;
    if (d.dst16) *(uint2*)(d.dst16 + c.start + i) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
  }
}

}  // namespace

extern "C" {

int mopt_multi_copy(const void* descs, const void* chunks, int n_chunks, void* stream) {
  if (n_chunks <= 0) return 0;
  hipLaunchKernelGGL(multi_copy_kernel, dim3(n_chunks), dim3(256), 0, (hipStream_t)stream,
                     (const CopyDesc*)descs, (const CopyChunk*)chunks);
  return (int)hipGetLastError();
}

}  // extern "C"
