// Causal flash attention (forward + backward) for the population LM (north-star kernel K10).
//
// Layouts (head dim 64, bf16):
//   Q, K, V, dQ, dK, dV   [BH][T][64]            BH = population * batch * heads
//   O, dO                 [B'][T][H][64]        = the [rows, d_model] activation layout
//   LSE2, Dsum            [BH][T] f32           log2-domain logsumexp / rowsum(dO * O)
// T is a multiple of 64.  Softmax runs in the exp2 domain: s = (q.k) * scale * log2(e).
//
// Every MFMA is v_mfma_f32_16x16x32_bf16 with the fragment layout of common.h.  The trick that
// keeps P (and dS) in registers between the two GEMMs of each step: scores are computed
// TRANSPOSED (S^T = K Q^T, lane = one query) with the K rows fed to the MFMA in a permuted order,
// so that the 4+4 accumulator registers a lane holds for key tiles 2s and 2s+1 are exactly the 8
// consecutive keys 32s + 8g .. 32s + 8g + 7 that the B operand of the P.V MFMA wants in that lane.
// The row-max / row-sum of the online softmax are then a 4-lane reduction (lanes l, l^16, l^32,
// l^48), and the P.V product reads V through ds_read_b64_tr_b16 (no LDS transpose pass).
//
// Kernels: attn_fwd (one 64-query block per workgroup, 16 queries per wave), attn_bwd_dq (same
// decomposition, loops over key blocks; computes Dsum of its own query rows and stores it for
// attn_bwd_dkdv, launched after it) and attn_bwd_dkdv (one 64-key block per workgroup, 16 keys
// per wave, loops over query blocks).  No atomics anywhere.
#include "common.h"

using namespace mopt;

namespace {

constexpr int D = 64;          // head dim
constexpr int BQ = 64;         // queries per workgroup
constexpr int BKV = 64;        // keys per block
constexpr int LS = kLdsStride;
// LDS tile layouts: SW = common.h's XOR chunk swizzle of 64-element rows (soff; every fragment
// read conflict-free), else rows padded to LS = 72 elements (4 extra cycles per fragment read, 2
// per transposed read).  The forward uses SW (round 5: 109-114 -> 96-104 us per call at the same
// occupancy, bank conflicts 0).  The backward kernels keep the padded rows: swizzled, the extra
// per-lane addresses spill them at their 4 / 3 waves per SIMD, and at 3 / 2 waves (no spills, no
// conflicts) dQ + dK/dV ran 324 against 289 us (profiles/r5/attn_swizzle/).  (Round 4 measured
// another swizzle, chunk ^ (row >> 1) & 7, slower even in the forward: it mixed the rows that
// otherwise differ by immediate offsets; swz128 leaves row bits 0, 2, 4, 5 out.)
// The backward kernels' padded tiles (round 6): rows of LSB = 80 elements (40 dwords) and a key /
// query order within each 32-row step (row_of below) that gives every 32-lane half of a
// transposed read 8 CONSECUTIVE rows -- 8 x 8 dwords at multiples of 40 mod 64, all 64 banks --
// and every 16-lane group of a fragment read distinct banks: the scripts/lds_banks.py model goes
// from 4 / 2 extra cycles per fragment / transposed read (72-element rows, direct order: rows r
// and r + 8 of one half always share banks) to 0 / 0.
// (MOPT_ATTN_PERM=0: the direct order and 72-element rows, for A/B builds)
#ifndef MOPT_ATTN_PERM
#define MOPT_ATTN_PERM 1
#endif
constexpr int LSB = MOPT_ATTN_PERM ? 80 : LS;
template <bool SW>
__device__ __forceinline__ int toff(int r, int c) { return SW ? soff(r, c) : r * LSB + c; }
template <bool SW>
constexpr int tile_elems() { return SW ? 64 * D : 64 * LSB; }

// Row (key or query) of MFMA k index 8 g + j of 32-row step ks: the direct order (forward,
// PB = false), or the backward's (PB): 16 (g >> 1) + 8 (j >> 2) + 4 (g & 1) + (j & 3).
template <bool PB>
__device__ __forceinline__ int row_of(int ks, int g, int j) {
  return (PB && MOPT_ATTN_PERM) ? 32 * ks + 16 * (g >> 1) + 8 * (j >> 2) + 4 * (g & 1) + (j & 3)
                                : 32 * ks + 8 * g + j;
}

// Occupancy targets (waves per SIMD; 0 = the compiler's choice): the register cap that lets N
// workgroups share a CU.  Swept in round 4 on variant builds (scripts/attn_bench.py,
// profiles/r4/attn_sweep_r4q.log; fwd / dQ+dK/dV us, two runs): 0,4,3 117 / 257; 4,4,3 101 / 263;
// 3,4,3 109 / 267; 2,4,3 108 / 268; 0,3,3 117 / 261; 0,4,2 123 / 259; 0,5,3 123 / 350; 0,4,4
// 121 / 386.  The forward at 4 waves (since the native exp2 it compiles without spills) and
// dQ / dK/dV at 4 / 3 (round 3: 110.9 -> 99.5 / 179.8 -> 157.7 us per call).
#ifndef MOPT_ATTN_WAVES          // "fwd, dq, dkdv" -- variant builds of scripts/attn_bench.py sweeps
#define MOPT_ATTN_WAVES 4, 4, 3
#endif
constexpr int kAttnWaves[3] = {MOPT_ATTN_WAVES};
constexpr int kAttnFwdWaves = kAttnWaves[0], kAttnDqWaves = kAttnWaves[1],
              kAttnDkdvWaves = kAttnWaves[2];
// (Measured and rejected, round 4: two 16-query / 16-key sets per wave -- 128 queries or keys
// per workgroup, every LDS fragment feeding two MFMAs -- ran fwd 104 -> 157 us, dQ 98 -> 149,
// dK/dV 156 -> 250 on the 125M LM: the doubled register state cost the occupancy that hides
// this loop's latency; profiles/round4.md.)
#define MOPT_WAVES_ATTR(n) __attribute__((amdgpu_waves_per_eu((n) > 0 ? (n) : 1)))

// (position of this workgroup's sequence block within its head, head index bh) for a 1-D grid of
// nblk * n_bh workgroups.  All blocks of one (batch, head) run on ONE XCD -- they re-read the same
// K/V (or Q/dO) tiles, which then stay in that XCD's L2; with the 2-D (T/64, BH) grid the
// hardware's round-robin put the 8 blocks of a head on 8 different XCDs and every XCD fetched
// every head's tiles.  XCDs get contiguous shares of heads; within a head, rank 0 first.
__device__ __forceinline__ int2 head_block(int nblk, int n_bh) {
  const int t = xcd_remap((int)blockIdx.x, nblk * n_bh);
  return make_int2(t % nblk, t / nblk);
}

// Load a [64][64] bf16 tile (rows contiguous, row stride 64) into a swizzled LDS tile.
template <bool SW>
__device__ __forceinline__ void tile_to_lds(const bf16_t* __restrict__ g, bf16_t* s, int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + 256 * i, r = c >> 3, ch = c & 7;
    *(uint4*)(s + toff<SW>(r, ch * 8)) = *(const uint4*)(g + r * D + ch * 8);
  }
}

// The same tile in two steps, so the next key block's global loads are in flight while the current
// block is multiplied (register staging, T14): load into registers, store to LDS after the barrier.
__device__ __forceinline__ void tile_load(const bf16_t* __restrict__ g, uint4& r0, uint4& r1,
                                          int tid) {
  r0 = *(const uint4*)(g + (tid >> 3) * D + (tid & 7) * 8);
  r1 = *(const uint4*)(g + ((tid + 256) >> 3) * D + (tid & 7) * 8);
}
template <bool SW>
__device__ __forceinline__ void tile_store(const uint4& r0, const uint4& r1, bf16_t* s, int tid) {
  *(uint4*)(s + toff<SW>(tid >> 3, (tid & 7) * 8)) = r0;
  *(uint4*)(s + toff<SW>((tid + 256) >> 3, (tid & 7) * 8)) = r1;
}

// Key row of the permuted K/V fragment: tile j = 2s + h, fragment row m -- the row whose score
// lands in accumulator register (j, r) of lane group g where the P.V B operand wants key
// row_of(s, g, 4 h + r): m = 4 g + r
template <bool PB>
__device__ __forceinline__ int perm_row(int s, int h, int m) {
  if constexpr (PB) return row_of<true>(s, m >> 2, 4 * h + (m & 3));
  return 32 * s + 8 * (m >> 2) + 4 * h + (m & 3);   // (the forward's own expression: its code
}                                                   //  is register-tuned, 88 VGPRs)

// V^T (or K^T) A-fragment for keys 32s + 8g .. +7, head-dim columns 16 dt .. +15, from LDS [key][dh].
template <bool SW>
__device__ __forceinline__ bf16x8 tr_frag(const bf16_t* s, int ks, int g, int q, int pp, int dt) {
  if constexpr (SW) {
    const s16x4 lo = lds_tr4(s + toff<SW>(32 * ks + 8 * g + q, 16 * dt + 4 * pp));
    const s16x4 hi = lds_tr4(s + toff<SW>(32 * ks + 8 * g + 4 + q, 16 * dt + 4 * pp));
    return cat_frag(lo, hi);
  }
  const s16x4 lo = lds_tr4(s + toff<SW>(row_of<true>(ks, g, q), 16 * dt + 4 * pp));
  const s16x4 hi = lds_tr4(s + toff<SW>(row_of<true>(ks, g, 4 + q), 16 * dt + 4 * pp));
  return cat_frag(lo, hi);
}

__device__ __forceinline__ bf16x8 pack_frag(const f32x4& a, const f32x4& b) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 w = {pack2bf(a[0], a[1]), pack2bf(a[2], a[3]), pack2bf(b[0], b[1]), pack2bf(b[2], b[3])};
  return __builtin_bit_cast(bf16x8, w);
}

// v_exp_f32 alone: exp2f goes through the library's denormal-safe path (a compare, two selects,
// an add and a rescale around every v_exp_f32) -- about 5 VALU per score, a third of the
// backward kernels' VALU issue (round 4 PMC, profiles/round4.md).  Softmax terms below 2^-126
// flush to zero, which changes no bf16 probability.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Gradient outputs of the backward kernels: 4 consecutive head-dim columns col .. col + 3 of row
// t of head bh, to the head-major buffer `plain` -- or, when dqkv is set (the LM's fused QKV
// projection + RoPE, ops.qkv_rope_attention), straight into the QKV activation's gradient
// [B' T][3][H][64] (section sec: q, k, v) with the inverse interleaved-pair RoPE on q and k, so
// no separate RoPE-backward pass re-reads dQ / dK.
struct RopeOut {
  bf16_t* dqkv;
  const float* cosT;
  const float* sinT;
};

__device__ __forceinline__ void put_grad4(bf16_t* plain, const RopeOut& ro, int sec, int bh,
                                          int H, int T, int t, int col, float (&x)[4]) {
  if (ro.dqkv == nullptr) {
    *(uint2*)plain = make_uint2(pack2bf(x[0], x[1]), pack2bf(x[2], x[3]));
    return;
  }
  const int b = bh / H, hh = bh - b * H;
  if (sec < 2) {
    const float* cs = ro.cosT + (size_t)t * 32 + (col >> 1);
    const float* sn = ro.sinT + (size_t)t * 32 + (col >> 1);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float a = x[2 * j], bb = x[2 * j + 1], c = cs[j], sv = sn[j];
      x[2 * j] = a * c + bb * sv;
      x[2 * j + 1] = bb * c - a * sv;
    }
  }
  bf16_t* o = ro.dqkv + ((size_t)(b * T + t) * 3 + sec) * H * 64 + hh * 64 + col;
  *(uint2*)o = make_uint2(pack2bf(x[0], x[1]), pack2bf(x[2], x[3]));
}

// max / sum over the lanes l, l ^ 16, l ^ 32, l ^ 48 with gfx950's v_permlane16_swap /
// v_permlane32_swap (VALU, a few cycles): with both operands v, the pair the swap returns is
// {v[l], v[l ^ 16]} (or ^ 32) in some order, and max / + of the pair is order-free.  __shfl_xor
// compiled to ds_bpermute_b32 -- an LDS round trip on the softmax's critical path, 4 per key block.
__device__ __forceinline__ float xor16_pair_max(float v) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}
__device__ __forceinline__ float max4(float v) {
  v = xor16_pair_max(v);
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}
__device__ __forceinline__ float sum4(float v) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// S^T tiles for one 64-key block: st[j][r] = s(query li, key 32s + 8g + 4h + r), j = 2s + h.
template <bool SW>
__device__ __forceinline__ void scores_T(const bf16_t* Ks, const bf16x8 (&qf)[2], int li, int g,
                                         f32x4 (&st)[4]) {
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = 2 * s + h, row = perm_row<!SW>(s, h, li);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) acc = mfma16(lds_frag(Ks + toff<SW>(row, 32 * ks + 8 * g)), qf[ks], acc);
      st[j] = acc;
    }
}

// Forward: O = softmax(QK^T * scale, causal) V.   1-D grid of (T / 64 / NQB) * BH workgroups of
// NQB 64-query blocks (256 NQB threads, 16 queries per wave) sharing each staged K / V tile: with
// NQB = 2 the threads of the first block load the K tile, those of the second the V tile, and the
// first block's waves skip the multiply of the last key block (past their diagonal).  Measured
// (round 5, profiles/r5/attn_qb2/, 3 interleaved runs): NQB = 2 95-99 us per call against 90-95
// for NQB = 1 (LM-125M 38.4-38.9 vs 38.4-38.5 ms) -- half the K / V staging per query does not pay
// for the 8-wave barriers and the idle diagonal block; NQB = 1 stays the default.
#ifndef MOPT_ATTN_FWD_QB
#define MOPT_ATTN_FWD_QB 1
#endif
template <int NQB>
__global__ __launch_bounds__(256 * NQB) MOPT_WAVES_ATTR(kAttnFwdWaves) void attn_fwd_kernel(const bf16_t* __restrict__ Q,
                                                       const bf16_t* __restrict__ K,
                                                       const bf16_t* __restrict__ V,
                                                       bf16_t* __restrict__ O,
                                                       float* __restrict__ LSE2, int T, int H,
                                                       float c, int n_bh) {
  __shared__ __attribute__((aligned(16))) bf16_t Ks[tile_elems<true>()];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[tile_elems<true>()];
  const int nblk = T / (BQ * NQB);
  const int2 hb = head_block(nblk, n_bh);
  const int qb0 = (nblk - 1 - hb.x) * NQB;            // longest (most key blocks) first
  const int qb_last = qb0 + NQB - 1;
  const int bh = hb.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4, q = li >> 2, pp = li & 3;
  const size_t base = (size_t)bh * T * D;
  const int qb = qb0 + (wave >> 2);                    // this wave's query block
  const int qrow = qb * BQ + (wave & 3) * 16 + li;     // this lane's query
  // NQB = 2: waves 0-3 stage K, waves 4-7 V (wave-uniform pointers)
  const bf16_t* kvsrc = (NQB == 1 || tid < 256) ? K + base : V + base;
  bf16_t* kvdst = (NQB == 1 || tid < 256) ? Ks : Vs;
  const int ltid = tid & 255;

  bf16x8 qf[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) qf[ks] = lds_frag(Q + base + (size_t)qrow * D + 32 * ks + 8 * g);

  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  uint4 ka, kc, va, vc;   // key block kb + 1, fetched while block kb is multiplied
  tile_load(kvsrc, ka, kc, ltid);
  if (NQB == 1) tile_load(V + base, va, vc, tid);
  for (int kb = 0; kb <= qb_last; ++kb) {
    __syncthreads();
    tile_store<true>(ka, kc, kvdst, ltid);
    if (NQB == 1) tile_store<true>(va, vc, Vs, tid);
    __syncthreads();
    {
      const size_t nb = (size_t)min(kb + 1, qb_last) * BKV * D;   // clamped: no branch around loads
      tile_load(kvsrc + nb, ka, kc, ltid);
      if (NQB == 1) tile_load(V + base + nb, va, vc, tid);
    }
    if (NQB > 1 && kb > qb) continue;                  // wave-uniform: past this wave's diagonal
    f32x4 st[4];
    scores_T<true>(Ks, qf, li, g, st);
    // the row max on the raw scores (c > 0: max(s) c = max(s c)), the scale folded into the
    // exponent's fma -- 16 multiplies per key block less
    float mx = -INFINITY;
    if (kb == qb) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kb * BKV + 32 * (j >> 1) + 8 * g + 4 * (j & 1) + r;
          if (key > qrow) st[j][r] = -INFINITY;
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) mx = fmaxf(mx, st[j][r]);
    const float m_new = fmaxf(m, max4(mx) * c);
    const float alpha = fast_exp2(m - m_new);
    float ls = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = fast_exp2(fmaf(st[j][r], c, -m_new));
        st[j][r] = p;
        ls += p;
      }
    l = l * alpha + sum4(ls);
    m = m_new;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 pb = pack_frag(st[2 * s], st[2 * s + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] = mfma16(tr_frag<true>(Vs, s, g, q, pp, dt), pb, o[dt]);
    }
  }
  // o[dt][r] = O^T[dh 16 dt + 4 g + r][query li]
  const float inv = 1.f / l;
  const int b = bh / H, hh = bh % H;
  bf16_t* out = O + (((size_t)b * T + qrow) * H + hh) * D;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
    *(uint2*)(out + 16 * dt + 4 * g) =
        make_uint2(pack2bf(o[dt][0] * inv, o[dt][1] * inv), pack2bf(o[dt][2] * inv, o[dt][3] * inv));
  if (g == 0) LSE2[(size_t)bh * T + qrow] = m + log2f(l);
}

// Dsum[bh][t] = sum_d dO * O  (one thread per query row).  (Round 6: no longer launched -- the dQ
// kernel computes the Dsum of its query rows from the dO fragments it loads anyway; kept as the
// standalone form for MOPT_ATTN_PREP=1 A/B builds.)
__global__ __launch_bounds__(256) void attn_bwd_prep_kernel(const bf16_t* __restrict__ O,
                                                            const bf16_t* __restrict__ dO,
                                                            float* __restrict__ Dsum, int T, int H,
                                                            int n_rows) {
  const int i = blockIdx.x * 256 + threadIdx.x;     // i = bh * T + t
  if (i >= n_rows) return;
  const int bh = i / T, t = i % T, b = bh / H, hh = bh % H;
  const size_t off = (((size_t)b * T + t) * H + hh) * D;
  float acc = 0.f;
#pragma unroll
  for (int c8 = 0; c8 < D / 8; ++c8) {
    const uint4 a = *(const uint4*)(O + off + 8 * c8);
    const uint4 d = *(const uint4*)(dO + off + 8 * c8);
    const uint32_t aw[4] = {a.x, a.y, a.z, a.w}, dw[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      acc += bf2f(aw[e] & 0xFFFF) * bf2f(dw[e] & 0xFFFF) + bf2f(aw[e] >> 16) * bf2f(dw[e] >> 16);
  }
  Dsum[i] = acc;
}

// dQ = scale * sum_k dS K, dS = P * (dP - Dsum), dP = dO V^T.   grid (T/64, BH).
// DSUM: Dsum of the lane's query = sum_d dO O from its two dO fragments and the matching O
// fragments (16 of the 64 products per lane, summed over the 4 lanes of the query), stored for
// the dK/dV kernel -- the separate prep pass (O and dO read once more) goes.
__global__ __launch_bounds__(256) MOPT_WAVES_ATTR(kAttnDqWaves) void attn_bwd_dq_kernel(const bf16_t* __restrict__ Q,
                                                          const bf16_t* __restrict__ K,
                                                          const bf16_t* __restrict__ V,
                                                          const bf16_t* __restrict__ dO,
                                                          const float* __restrict__ LSE2,
                                                          float* __restrict__ Dsum,
                                                          bf16_t* __restrict__ dQ, int T, int H,
                                                          float c, float scale, int n_bh,
                                                          const RopeOut ro,
                                                          const bf16_t* __restrict__ O) {
  __shared__ __attribute__((aligned(16))) bf16_t Ks[tile_elems<false>()];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[tile_elems<false>()];
  const int nqb = T / BQ;
  const int2 hb = head_block(nqb, n_bh);
  const int qb = nqb - 1 - hb.x;
  const int bh = hb.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4, q = li >> 2, pp = li & 3;
  const size_t base = (size_t)bh * T * D;
  const int qrow = qb * BQ + wave * 16 + li;
  const int b = bh / H, hh = bh % H;
  const size_t orow = (((size_t)b * T + qrow) * H + hh) * D;

  bf16x8 qf[2], df[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    qf[ks] = lds_frag(Q + base + (size_t)qrow * D + 32 * ks + 8 * g);
    df[ks] = lds_frag(dO + orow + 32 * ks + 8 * g);
  }
  const float lse = LSE2[(size_t)bh * T + qrow];
  float dsum;
  if (O != nullptr) {
    float part = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 of = lds_frag(O + orow + 32 * ks + 8 * g);
#pragma unroll
      for (int e = 0; e < 8; ++e) part = fmaf((float)df[ks][e], (float)of[e], part);
    }
    dsum = sum4(part);
    if (g == 0) Dsum[(size_t)bh * T + qrow] = dsum;
  } else {
    dsum = Dsum[(size_t)bh * T + qrow];
  }
  f32x4 acc[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ka, kc, va, vc;
  tile_load(K + base, ka, kc, tid);
  tile_load(V + base, va, vc, tid);
  for (int kb = 0; kb <= qb; ++kb) {
    __syncthreads();
    tile_store<false>(ka, kc, Ks, tid);
    tile_store<false>(va, vc, Vs, tid);
    __syncthreads();
    {
      const size_t nb = (size_t)min(kb + 1, qb) * BKV * D;
      tile_load(K + base + nb, ka, kc, tid);
      tile_load(V + base + nb, va, vc, tid);
    }
    f32x4 st[4], dpt[4];
    scores_T<false>(Ks, qf, li, g, st);
    scores_T<false>(Vs, df, li, g, dpt);     // dP^T = V dO^T, same permuted key order
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float p = fast_exp2(st[j][r] * c - lse);
        if (kb == qb) {
          const int key = kb * BKV + row_of<true>(j >> 1, g, 4 * (j & 1) + r);
          if (key > qrow) p = 0.f;
        }
        st[j][r] = p * (dpt[j][r] - dsum);   // dS (without the scale)
      }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 sb = pack_frag(st[2 * s], st[2 * s + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) acc[dt] = mfma16(tr_frag<false>(Ks, s, g, q, pp, dt), sb, acc[dt]);
    }
  }
  bf16_t* out = dQ + base + (size_t)qrow * D;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    float x[4] = {acc[dt][0] * scale, acc[dt][1] * scale, acc[dt][2] * scale, acc[dt][3] * scale};
    put_grad4(out + 16 * dt + 4 * g, ro, 0, bh, H, T, qrow, 16 * dt + 4 * g, x);
  }
}

// dV = sum_q P^T dO,  dK = scale * sum_q dS^T Q.   grid (T/64, BH); one 64-key block per WG.
// Scores are computed un-transposed here (S = Q K^T, lane = one key) with the Q / dO rows fed in
// the permuted order, so P^T and dS^T land in A-fragment order for the two accumulating MFMAs.
__global__ __launch_bounds__(256) MOPT_WAVES_ATTR(kAttnDkdvWaves) void attn_bwd_dkdv_kernel(const bf16_t* __restrict__ Q,
                                                            const bf16_t* __restrict__ K,
                                                            const bf16_t* __restrict__ V,
                                                            const bf16_t* __restrict__ dO,
                                                            const float* __restrict__ LSE2,
                                                            const float* __restrict__ Dsum,
                                                            bf16_t* __restrict__ dK,
                                                            bf16_t* __restrict__ dV, int T, int H,
                                                            float c, float scale, int n_bh,
                                                            const RopeOut ro) {
  __shared__ __attribute__((aligned(16))) bf16_t Qs[tile_elems<false>()];
  __shared__ __attribute__((aligned(16))) bf16_t dOs[tile_elems<false>()];
  __shared__ __attribute__((aligned(16))) float lse_s[BQ];
  __shared__ __attribute__((aligned(16))) float dsum_s[BQ];
  const int2 hb = head_block(T / BKV, n_bh);
  const int kb = hb.x;                            // blocks with more query blocks are early ids
  const int bh = hb.y;
  const int nqb = T / BQ;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4, q = li >> 2, pp = li & 3;
  const size_t base = (size_t)bh * T * D;
  const int krow = kb * BKV + wave * 16 + li;    // this lane's key
  const int b = bh / H, hh = bh % H;

  bf16x8 kf[2], vf[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    kf[ks] = lds_frag(K + base + (size_t)krow * D + 32 * ks + 8 * g);
    vf[ks] = lds_frag(V + base + (size_t)krow * D + 32 * ks + 8 * g);
  }
  f32x4 dk[4], dv[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dk[dt] = dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // query block qb + 1 (Q tile, dO rows in the [B'][T][H][64] layout, LSE2 / Dsum) is fetched
  // into registers while block qb is multiplied (T14 register staging)
  uint4 qa, qc, da, dc;
  float lse_r = 0.f, dsum_r = 0.f;
  const int r0 = tid >> 3, r1 = (tid + 256) >> 3, ch = tid & 7;
  // per-thread bases of the query-block loads (block qb_ adds qb_ * BQ rows): 32-bit offsets
  // from them, no 64-bit index arithmetic inside the loop
  const bf16_t* qbase = Q + base + (tid >> 3) * D + (tid & 7) * 8;
  const bf16_t* dob = dO + (((size_t)b * T + r0) * H + hh) * D + ch * 8;
  const int dorow = 32 * H * D;                                   // rows r1 - r0 = 32
  const float* lseb = LSE2 + (size_t)bh * T + tid;
  const float* dsb = Dsum + (size_t)bh * T + tid;
#define MOPT_DKDV_LOAD(QB)                                                                   \
  {                                                                                          \
    const int qb_ = (QB);                                                                    \
    const uint32_t qo_ = (uint32_t)(qb_ * BQ * D), do_ = (uint32_t)(qb_ * BQ * H * D);       \
    qa = *(const uint4*)(qbase + qo_);                                                       \
    qc = *(const uint4*)(qbase + qo_ + 32 * D);                                              \
    da = *(const uint4*)(dob + do_);                                                         \
    dc = *(const uint4*)(dob + do_ + dorow);                                                 \
    if (tid < BQ) {                                                                          \
      lse_r = lseb[qb_ * BQ];                                                                \
      dsum_r = dsb[qb_ * BQ];                                                                \
    }                                                                                        \
  }
  MOPT_DKDV_LOAD(kb)
  for (int qb = kb; qb < nqb; ++qb) {
    __syncthreads();
    tile_store<false>(qa, qc, Qs, tid);
    *(uint4*)(dOs + toff<false>(r0, ch * 8)) = da;
    *(uint4*)(dOs + toff<false>(r1, ch * 8)) = dc;
    if (tid < BQ) {
      lse_s[tid] = lse_r;
      dsum_s[tid] = dsum_r;
    }
    __syncthreads();
    MOPT_DKDV_LOAD(min(qb + 1, nqb - 1))
    // S and dP tiles j = 2s + h: rows = queries 32s + 8g + 4h + r (C layout), column = key li.
    f32x4 st[4], dp[4];
    scores_T<false>(Qs, kf, li, g, st);
    scores_T<false>(dOs, vf, li, g, dp);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // the 4 queries of register r = 0..3 are consecutive: one 16-byte LDS read each for LSE2
      // and Dsum (instead of 8 4-byte reads)
      const int q0 = row_of<true>(j >> 1, g, 4 * (j & 1));
      const f32x4 l4 = *(const f32x4*)(lse_s + q0), d4 = *(const f32x4*)(dsum_s + q0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float p = fast_exp2(st[j][r] * c - l4[r]);
        if (qb == kb && qb * BQ + q0 + r < krow) p = 0.f;
        st[j][r] = p;
        dp[j][r] = p * (dp[j][r] - d4[r]);
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 pa = pack_frag(st[2 * s], st[2 * s + 1]);
      const bf16x8 sa = pack_frag(dp[2 * s], dp[2 * s + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        // dV^T[dh][key] += dO^T P^T : A = dO^T (tr-read), B = P^T fragment (this lane's key)
        dv[dt] = mfma16(tr_frag<false>(dOs, s, g, q, pp, dt), pa, dv[dt]);
        dk[dt] = mfma16(tr_frag<false>(Qs, s, g, q, pp, dt), sa, dk[dt]);
      }
    }
  }
  // dv[dt][r] = dV^T[dh 16 dt + 4 g + r][key li]
  bf16_t* okp = dK + base + (size_t)krow * D;
  bf16_t* ovp = dV + base + (size_t)krow * D;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    float xk[4] = {dk[dt][0] * scale, dk[dt][1] * scale, dk[dt][2] * scale, dk[dt][3] * scale};
    float xv[4] = {dv[dt][0], dv[dt][1], dv[dt][2], dv[dt][3]};
    put_grad4(okp + 16 * dt + 4 * g, ro, 1, bh, H, T, krow, 16 * dt + 4 * g, xk);
    put_grad4(ovp + 16 * dt + 4 * g, ro, 2, bh, H, T, krow, 16 * dt + 4 * g, xv);
  }
#undef MOPT_DKDV_LOAD
}

}  // namespace

extern "C" {

int mopt_attn_fwd(const void* q, const void* k, const void* v, void* o, void* lse2, int bh, int T,
                  int H, float scale, void* stream) {
  if (T % 64 || bh <= 0) return 1;
  const float c = scale * 1.4426950408889634f;
  constexpr int NQB = MOPT_ATTN_FWD_QB;
  if (NQB > 1 && T % (64 * NQB) == 0)
    hipLaunchKernelGGL(attn_fwd_kernel<NQB>, dim3((T / (64 * NQB)) * bh), dim3(256 * NQB), 0,
                       (hipStream_t)stream, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                       (bf16_t*)o, (float*)lse2, T, H, c, bh);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<1>, dim3((T / 64) * bh), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o,
                       (float*)lse2, T, H, c, bh);
  return (int)hipGetLastError();
}

// dqkv (optional): the gradient of the QKV activation [B' T][3][H][64] with the inverse
// interleaved RoPE applied to its q / k sections (cos / sin [T][32]) -- written instead of dq,
// dk, dv (which may then be null)
int mopt_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                  const void* lse2, void* dsum, void* dq, void* dk, void* dv, int bh, int T, int H,
                  float scale, void* dqkv, const void* cosT, const void* sinT, void* stream) {
  if (T % 64 || bh <= 0 || (dqkv != nullptr && (cosT == nullptr || sinT == nullptr))) return 1;
  const float c = scale * 1.4426950408889634f;
  const int rows = bh * T;
  const RopeOut ro{(bf16_t*)dqkv, (const float*)cosT, (const float*)sinT};
  hipStream_t st = (hipStream_t)stream;
  // dQ first: it computes Dsum (MOPT_ATTN_PREP=1: the separate prep pass, for A/B builds)
#ifndef MOPT_ATTN_PREP
#define MOPT_ATTN_PREP 0
#endif
  if (MOPT_ATTN_PREP)
    hipLaunchKernelGGL(attn_bwd_prep_kernel, dim3((rows + 255) / 256), dim3(256), 0, st,
                       (const bf16_t*)o, (const bf16_t*)dout, (float*)dsum, T, H, rows);
  hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3((T / 64) * bh), dim3(256), 0, st, (const bf16_t*)q,
                     (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, (const float*)lse2,
                     (float*)dsum, (bf16_t*)dq, T, H, c, scale, bh, ro,
                     MOPT_ATTN_PREP ? nullptr : (const bf16_t*)o);
  hipLaunchKernelGGL(attn_bwd_dkdv_kernel, dim3((T / 64) * bh), dim3(256), 0, st,
                     (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout,
                     (const float*)lse2, (const float*)dsum, (bf16_t*)dk, (bf16_t*)dv, T, H, c,
                     scale, bh, ro);
  return (int)hipGetLastError();
}

}  // extern "C"
