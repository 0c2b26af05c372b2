// Batched device copies for the sweep's checkpoint pool (one launch per sync instead of one
// framework copy per tensor and member).
//
// A descriptor moves n values from an f32 (src) or bf16 (src16) source to an f32 destination
// (dst) and/or the bf16 image of the values (dst16): restoring a member's bf16 working weights in
// the same pass that restores its f32 master copy, and widening / narrowing a bf16 momentum
// buffer into / out of the f32 checkpoint pool (exact: the values are bf16), and joining /
// splitting split master weights (hi = bf16 working copy, lo = residual; common.h).
// Work is split into 4096-element chunks listed on the host, so a launch needs no per-descriptor
// grid sizing and stays balanced however ragged the member sizes are.
#include "common.h"

using namespace mopt;

extern "C" {

struct CopyDesc {       // 64 bytes, mirrored by metaopt_amd/ops/ckpt.py
  const float* src;     // f32 source, or nullptr when src16 is set
  float* dst;           // nullptr: no f32 copy
  bf16_t* dst16;        // nullptr: no bf16 image (with dst_lo: the hi half of a split master)
  int64_t n;            // multiple of 4
  const bf16_t* src16;  // bf16 source (widened exactly; with src_lo: hi half of a split master)
  const bf16_t* src_lo; // lo half of a split-master source
  bf16_t* dst_lo;       // lo half of a split-master destination
  int64_t pad;
};

struct CopyChunk {      // 16 bytes
  int32_t desc;
  int32_t pad;
  int64_t start;        // element offset inside the descriptor
};

}  // extern "C"

namespace {

constexpr int kChunk = 4096;

__device__ __forceinline__ f32x4 copy_load(const CopyDesc& d, int64_t e) {
  if (d.src_lo) return join4(*(const uint2*)(d.src16 + e), *(const uint2*)(d.src_lo + e));
  if (d.src16) return bf4_to_f32(*(const uint2*)(d.src16 + e));
  return *(const f32x4*)(d.src + e);
}

__device__ __forceinline__ void copy_store(const CopyDesc& d, int64_t e, const f32x4& v) {
  if (d.dst) *(f32x4*)(d.dst + e) = v;
  if (d.dst_lo) {
    uint2 hi, lo;
    split4(v, hi, lo);
    *(uint2*)(d.dst16 + e) = hi;
    *(uint2*)(d.dst_lo + e) = lo;
  } else if (d.dst16) {
    *(uint2*)(d.dst16 + e) = f32_to_bf4(v);
  }
}

// A chunk is kChunk / 1024 = 4 vectors per thread: all four loads are issued before the first
// store (the compiler cannot reorder them itself -- source and destination pointers may alias
// as far as it knows), so every thread keeps 4 loads in flight instead of one.
__global__ __launch_bounds__(256) void multi_copy_kernel(const CopyDesc* __restrict__ descs,
                                                         const CopyChunk* __restrict__ chunks) {
  constexpr int kPer = kChunk / 1024;
  const CopyChunk c = chunks[blockIdx.x];
  const CopyDesc d = descs[c.desc];
  const int64_t end = min((int64_t)kChunk, d.n - c.start);
  f32x4 v[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int64_t i = 4 * threadIdx.x + 1024 * u;
    if (i < end) v[u] = copy_load(d, c.start + i);
  }
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int64_t i = 4 * threadIdx.x + 1024 * u;
    if (i < end) copy_store(d, c.start + i, v[u]);
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
