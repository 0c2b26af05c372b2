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

// ------------------------------------------------------------------------------------------
// Member initialisation of a flat population (models/flatpop.py) in ONE launch: every
// parameter tensor of the member gets its f32 master (p32) and bf16 copy (p16) -- a constant or
// N(0, std) drawn from the counter-based RNG of common.h (Box-Muller over two uniforms keyed by
// (seed, tag, element)) -- and zeroed optimizer moments (m: f32 or bf16, v: f32 or absent);
// non-parameter state (running statistics) is filled by constant segments with only p32 set.
// Replaces 4 framework launches per tensor (~240 per ResNet-20 member).
extern "C" {

struct InitSeg {        // 64 bytes, mirrored by metaopt_amd/models/flatpop.py
  float* p32;           // f32 master, or (split) its 16-bit low halves
  bf16_t* p16;          // nullptr: no bf16 copy; split: the high halves
  void* m;              // nullptr: no first moment
  float* v;             // nullptr: no second moment
  int64_t n;            // multiple of 4
  int32_t kind;         // 0: constant val, 1: N(0, val)
  float val;
  uint32_t seed, tag;
  int32_t m16;          // m is bf16
  int32_t split;        // split master (common.h split4): p16 = hi, p32 = lo
};

}  // extern "C"

namespace {

__device__ __forceinline__ float normal_draw(uint32_t key, int64_t e) {
  const float u1 = fmaxf(rng_uniform(key, (uint32_t)(2 * e)), 1.0f / 16777216.0f);
  const float u2 = rng_uniform(key, (uint32_t)(2 * e + 1));
  return sqrtf(-2.f * __logf(u1)) * __cosf(6.283185307179586f * u2);
}

__global__ __launch_bounds__(256) void flat_init_kernel(const InitSeg* __restrict__ segs,
                                                        const CopyChunk* __restrict__ chunks) {
  const CopyChunk c = chunks[blockIdx.x];
  const InitSeg d = segs[c.desc];
  const int64_t end = min((int64_t)kChunk, d.n - c.start);
  const uint32_t key = rng_key(d.seed, d.tag, 0u);
  for (int64_t i = 4 * threadIdx.x; i < end; i += 1024) {
    const int64_t e = c.start + i;
    f32x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = d.kind == 1 ? d.val * normal_draw(key, e + r) : d.val;
    if (d.split) {           // p32 holds the 16-bit low halves of a split master
      uint2 hi, lo;
      split4(v, hi, lo);
      *(uint2*)(d.p16 + e) = hi;
      *(uint2*)((uint16_t*)d.p32 + e) = lo;
    } else {
      *(f32x4*)(d.p32 + e) = v;
      if (d.p16) *(uint2*)(d.p16 + e) = f32_to_bf4(v);
    }
    if (d.m) {
      if (d.m16) *(uint2*)((bf16_t*)d.m + e) = make_uint2(0u, 0u);
      else *(f32x4*)((float*)d.m + e) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (d.v) *(f32x4*)(d.v + e) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

}  // namespace

extern "C" {

int mopt_flat_init(const void* segs, const void* chunks, int n_chunks, void* stream) {
  if (n_chunks <= 0) return 0;
  hipLaunchKernelGGL(flat_init_kernel, dim3(n_chunks), dim3(256), 0, (hipStream_t)stream,
                     (const InitSeg*)segs, (const CopyChunk*)chunks);
  return (int)hipGetLastError();
}

}  // extern "C"
