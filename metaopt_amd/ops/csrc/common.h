// Shared device helpers for the metaopt_amd gfx950 (CDNA4) kernels.
//
// Conventions used by every kernel in this directory:
//   * wave = 64 lanes, workgroups of 256 threads (4 waves), one wave per 16x16 MFMA fragment set;
//   * bf16 tensors are stored as raw 16-bit words and moved 16 bytes per lane;
//   * MFMA = v_mfma_f32_16x16x32_bf16.  Lane l holds A[row l&15][k 8(l>>4)..+7],
//     B[k 8(l>>4)..+7][col l&15]; the f32 result C[row 4(l>>4)+r][col l&15] is register r.
//   * LDS tiles are [rows][64 + 8] bf16 (144-byte rows): 16-byte row reads at a fixed column are
//     conflict-free over 16 consecutive rows, and the rows stay 16-byte aligned for ds_read_b128
//     and 8-byte aligned for ds_read_b64_tr_b16.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mopt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t bf16_t;  // storage type of a bf16 element

constexpr int kLdsStride = 72;  // bf16 elements per LDS tile row (64 + 8 pad)

// Unpadded LDS tiles of 64-element (128-byte) rows with the 16-byte chunk c of row r stored at
// chunk c ^ swz128(r) (row bits 1 and 3 into chunk bits 1 and 2).  Conflict-free for the MFMA
// fragment reads of these tiles -- ds_read_b128 of 16 rows at one chunk, ds_read_b64_tr_b16 of
// 4 + 4 rows x 2 lane groups -- and for the 8-lanes-per-row staging stores (scripts/lds_banks.py
// searched every XOR map of the row bits; padding rows to 72 elements costs 4 extra cycles per
// fragment read and 2 per transposed read).  Rows r and r + 4 k + 32 m share the map, so a
// lane's fragment addresses differ by immediate offsets across those rows.
__device__ __forceinline__ int swz128(int r) { return (r & 2) | ((r & 8) >> 1); }
__device__ __forceinline__ int soff(int r, int c) {
  return r * 64 + (((c >> 3) ^ swz128(r)) << 3) + (c & 7);
}

// 64-column bf16 LDS tiles with 128-B rows whose 16-B chunks are XOR-swizzled by row:
// chunk' = chunk ^ swz_row(row), swz_row = (r0^r1^r2^r3^r4, r0^r1^r2^r3, r0^r3) over the row's
// low 5 bits.  Found by scripts/lds_banks.py: conflict-free for every LDS access of the
// population-MLP kernels -- 16-B staging stores, ds_read_b128 fragment reads (4 non-contiguous
// 16-lane groups), ds_read_b64_tr_b16 transposed reads (32-lane halves) and the 2-B epilogue
// stores -- where the 8-element row pad cost 2-4 extra cycles per fragment / transposed read.
__device__ __forceinline__ int swz_row(int r) {
  const int p = (r ^ (r >> 1) ^ (r >> 2) ^ (r >> 3)) & 1;
  return (p ^ ((r >> 4) & 1)) | (p << 1) | (((r ^ (r >> 3)) & 1) << 2);
}
// element offset of (row, col) in a swizzled 64-column tile
__device__ __forceinline__ int tile_off(int r, int c) {
  return r * 64 + ((((c >> 3) ^ swz_row(r)) & 7) << 3) + (c & 7);
}
// 64-column f32 tile, 256-B rows, 16-B chunks XOR-swizzled by (row & 15): conflict-free for
// column-fragment stores (rows = lanes) and row-contiguous reads
__device__ __forceinline__ int ftile_off(int r, int c) {
  return r * 64 + ((((c >> 2) ^ r) & 15) << 2) + (c & 3);
}

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // hipcc emits v_cvt_pk_bf16_f32 (RNE, NaN-preserving)
  return __builtin_bit_cast(bf16_t, b);
}

// two floats -> packed bf16x2 (RNE) in ONE v_cvt_pk_bf16_f32 with both sources: the scalar form
// (two converts, a shift and an OR -- hipcc does not merge them) cost 3 extra VALU per pair in
// every epilogue and softmax pack (round 5)
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, bf16x2_t));
}

// Split f32 master weights: hi = the bf16 working copy (round to nearest, ties toward the
// smaller magnitude), lo = a 16-bit residual such that (hi << 16) + lo - 0x7FFF is the f32 bit
// pattern again -- exact reconstruction of the master from 4 bytes, of which the forward reads
// only the 2 of hi.  Mirrored by metaopt_amd/ops/reference.py (split_f32 / join_f32).
__device__ __forceinline__ float join_hilo(uint32_t hi, uint32_t lo) {
  return __uint_as_float((hi << 16) + lo - 0x7FFFu);
}

__device__ __forceinline__ uint32_t split_hi(uint32_t u) { return (u + 0x7FFFu) >> 16; }

__device__ __forceinline__ uint32_t split_lo(uint32_t u, uint32_t hi) {
  return (u - (hi << 16) + 0x7FFFu) & 0xFFFFu;
}

// 4 (hi, lo) pairs (8 + 8 bytes) <-> 4 f32
__device__ __forceinline__ f32x4 join4(uint2 hi, uint2 lo) {
  return f32x4{join_hilo(hi.x & 0xFFFFu, lo.x & 0xFFFFu), join_hilo(hi.x >> 16, lo.x >> 16),
               join_hilo(hi.y & 0xFFFFu, lo.y & 0xFFFFu), join_hilo(hi.y >> 16, lo.y >> 16)};
}

__device__ __forceinline__ void split4(const f32x4& v, uint2& hi, uint2& lo) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t u = __float_as_uint(v[r]);
    h[r] = split_hi(u) & 0xFFFFu;
    l[r] = split_lo(u, h[r]);
  }
  hi = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
  lo = make_uint2(l[0] | (l[1] << 16), l[2] | (l[3] << 16));
}

// 4 packed bf16 <-> 4 f32 (bf16 optimizer state moved 8 bytes per lane)
__device__ __forceinline__ f32x4 bf4_to_f32(uint2 v) {
  return f32x4{__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xFFFF0000u),
               __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xFFFF0000u)};
}

__device__ __forceinline__ uint2 f32_to_bf4(const f32x4& v) {
  return make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ds_read_b64_tr_b16: the 16 lanes of a group each supply the address of row q = i>>2, columns
// 4(i&3)..+3 of a 4x16 block; lane i receives column i of the 4 rows.
__device__ __forceinline__ s16x4 lds_tr4(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}

__device__ __forceinline__ bf16x8 cat_frag(s16x4 lo, s16x4 hi) {
  s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 lds_frag(const bf16_t* p) {
  return __builtin_bit_cast(bf16x8, *(const uint4*)p);
}

// Bijective XCD-aware remap: consecutive work items land on the same XCD (blocks b, b+8, ... share
// one L2 under round-robin dispatch), so the k-strips / n-tiles of one trial share its operands in
// L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  if (nwg <= 8) return bid;
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// murmur3 finaliser: the counter-based RNG behind per-trial dropout.  Mirrored bit-for-bit by
// metaopt_amd/ops/reference.py so the HIP path and the PyTorch reference draw identical masks.
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ uint32_t rng_key(uint32_t seed, uint32_t layer, uint32_t step) {
  return fmix32(seed ^ fmix32(layer * 0x9E3779B9u + step * 0x7FEB352Du + 0x632BE5ABu));
}

__device__ __forceinline__ float rng_uniform(uint32_t key, uint32_t idx) {
  return (float)(fmix32(key ^ (idx * 0x9E3779B9u)) >> 8) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// -------------------------------------------------------------- bounds-checked debug build
// Compiled with -DMOPT_BOUNDS_CHECK (the "checked" library variant, lib/variants/checked/,
// loaded with MOPT_KERNEL_CHECKED=1), the kernels verify on the device the data-dependent
// indices that no host-side check can see -- token ids, class labels, sorted gather indices --
// before using them (the shapes and work tables are checked on the host before every launch).
// A violation increments this code object's counter, the first one prints the check, value
// and bound, and the offending access is skipped: a bad index is reported, never turned into
// a memory fault.  The host reads and clears the counters after each launch
// (metaopt_amd/ops/_lib.py) and raises naming the launch.  In the default build MOPT_IN_RANGE
// is the constant `true` and costs nothing.
#ifdef MOPT_BOUNDS_CHECK
static __device__ unsigned int g_violations;  // one per code object (internal linkage)

__device__ __noinline__ bool report_out_of_range(int64_t v, int64_t hi, const char* what) {
  if (atomicAdd(&g_violations, 1u) == 0)
    printf("[mopt bounds] %s: index %lld outside [0, %lld) (block %u thread %u)\n", what,
           (long long)v, (long long)hi, blockIdx.x, threadIdx.x);
  return false;
}

__device__ __forceinline__ bool in_range(int64_t v, int64_t hi, const char* what) {
  return (v >= 0 && v < hi) ? true : report_out_of_range(v, hi, what);
}
#define MOPT_IN_RANGE(v, hi, what) ::mopt::in_range((int64_t)(v), (int64_t)(hi), what)
// extern "C" reader of this code object's counter (reads and clears it; synchronises)
#define MOPT_VIOLATIONS_READER(name)                                                  \
  extern "C" unsigned int mopt_violations_##name() {                                  \
    unsigned int h = 0, z = 0;                                                        \
    if (hipDeviceSynchronize() != hipSuccess) return 0xFFFFFFFFu;                     \
    if (hipMemcpyFromSymbol(&h, HIP_SYMBOL(::mopt::g_violations), sizeof h) != hipSuccess) \
      return 0xFFFFFFFFu;                                                             \
    (void)hipMemcpyToSymbol(HIP_SYMBOL(::mopt::g_violations), &z, sizeof z);          \
    return h;                                                                         \
  }
#define MOPT_CHECKED_BUILD 1
#else
#define MOPT_IN_RANGE(v, hi, what) true
#define MOPT_VIOLATIONS_READER(name) \
  extern "C" unsigned int mopt_violations_##name() { return 0; }
#define MOPT_CHECKED_BUILD 0
#endif

}  // namespace mopt
