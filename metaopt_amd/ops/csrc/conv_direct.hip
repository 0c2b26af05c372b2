// Direct 3x3 convolutions of the population ResNet (north-star kernel K3) for the narrow
// channel counts of CIFAR ResNets (8..64): halo-tiled in LDS, weights register-resident.
//
// Why not the implicit GEMM of pgemm.hip: with C <= 64 the GEMM's K = 9 C is gathered tap by
// tap, so every input pixel is fetched 9 times (from L2) and every workgroup re-derives its
// addresses per 16-byte chunk; the layers ran at ~4x their HBM time.  Here a workgroup owns a
// band of NPX output pixels (TR output rows of one image, or IMGS whole images when an image is
// smaller than the band), stages the input halo band ((TR-1)*S + 3 rows x (OW-1)*S + 3 columns
// x CI, zero-padded) in LDS ONCE, and runs all 9 taps against it.  Workgroups are persistent
// over the bands of one trial, so each wave loads its slice of that trial's weights into
// registers once (as MFMA B fragments: one 16-column slice of CO per wave) and streams bands.
//
//   dconv_fwd_kernel    y = conv(x, w)    (+ per (trial, channel) sum / sum^2 of the bf16 output
//                       accumulated across bands and added once per wave: the BatchNorm batch
//                       statistics, so the BN forward skips its reduction pass)
//                       also the stride-1 data gradient dx = conv(dy, flip(w)^T) (DG mode: the
//                       B fragments are the tap-flipped, channel-transposed weights)
//   dconv_wgrad_kernel  partial dW = sum over a trial's bands of im2col(x)^T . dy, both operands
//                       read from LDS with the transposing ds_read_b64_tr_b16, f32 partials per
//                       persistent workgroup, summed + rounded by dconv_reduce_kernel.
//
// MFMA v_mfma_f32_16x16x32_bf16: lane l holds A[row l&15][k 8(l>>4)..+7], B[k ..][col l&15],
// C[row 4(l>>4)+r][col l&15] (common.h).  Forward: rows = output pixels, k = tap*CI + c, cols =
// output channels.  Weight gradient: rows = tap*CI + c, k = output pixels, cols = CO.
// Preconditions (host-checked): square power-of-two images, OW <= NPX, CI in {8,16,32,64},
// CO in {16,32,64}, stride 1 or 2.
#include "common.h"

#include <algorithm>

using namespace mopt;

namespace {

enum Mode { kFwd = 0, kDgrad = 1, kDgrad2 = 2 };

struct Geom {
  int Bn;          // images per trial
  int H, OH;       // input / output side (square)
  int owl;         // log2 OW
  int TR, IMGS;    // output rows per band, images per band
  int TRI, WI;     // halo rows / columns
  int rpil;        // log2 (pixels per image in a band) = log2(TR * OW)
  int tpi;         // bands per image
  int tiles;       // bands per trial
  int nb;          // persistent workgroups per trial
  float inv_wi, inv_tri;  // 1 / WI, 1 / TRI: exact quotients of small integers via (t + .5) / d
  int lds_elems;          // bf16 elements of the workgroup's LDS allocation
  int cs_off;             // forward: element offset of the output tile (0: it aliases the halo)
  int x_shared;           // every trial reads the same input x (the stem over the shared batch)
};

__device__ __forceinline__ int fdiv(int t, float inv) { return (int)(((float)t + 0.5f) * inv); }

// LDS pixel stride of the halo band (elements).  An A fragment's ds_read_b128 is serviced in four
// 16-lane groups, e.g. {0-3, 12-15, 20-27}: fragment rows (pixels) li in {0-3, 12-15} at chunk
// g and li in {4-11} at chunk g + 1.  With a = the stride between consecutive fragment pixels in
// 16-byte bank slots, the 16 slots a li (+1) are distinct mod 16 exactly when a = 2 mod 4: so
// a = 2 (8 <= CI <= 16), 6 (CI 32), 10 (CI 64) at stride 1 (pixels adjacent), and odd pixel
// strides at stride 2 (fragment pixels two apart): CI + 8 for CI >= 16.
template <int CI, int S>
constexpr int pstride() {
  if (S == 2) return CI >= 16 ? CI + 8 : CI;
  // (CI = 8: the 4 chunks of a fragment row are 4 different taps -- unpadded measured best)
  if (CI == 8) return 8;
  return CI / 8 % 4 == 2 ? CI : CI + 16;
}

// halo band: input rows row0 .. row0 + TRI, columns -1 .. WI - 2 of images b0 .. b0 + IMGS,
// in 16-byte chunks c = (halo pixel) * CI / 8 + channel chunk.
// BNIN: x is a BatchNorm's raw input and the convolution's operand is relu(x sc + sh) -- applied
// as the band is staged (bn_apply_kernel's arithmetic, rounded to bf16), so the BatchNorm output
// is never written to HBM; tab = LDS [2][CI] f32 (scale, shift); the zero padding stays 0.
//
// Staging is software-pipelined (round 5): the band a workgroup multiplies next is fetched into
// registers (Halo::fetch, NPF 16-byte chunks per thread, every load unconditional -- padding
// chunks read the trial's first pixel and are zeroed at the store -- so the compiler's counted
// waits stay exact) while the current band's MFMAs run, and written to LDS (Halo::put) once the
// band is done.  Without it a workgroup's band loads were exposed at the top of every band and
// the 2-4 resident workgroups per CU kept too few bytes in flight (~3.3 TB/s).

// an opaque copy of v: keeps the per-chunk geometry derived from it inside the band loop (hoisted
// out of it, the chunks' band-invariant index arithmetic held ~60 VGPRs across the MFMAs)
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// global element offset (from the trial's base) of halo chunk c, -1 for zero padding
template <int CI>
__device__ __forceinline__ int halo_src(const Geom& g, int b0, int row0, int c) {
  constexpr int CC = CI / 8;
  const int cc = c % CC;
  const int t = c / CC;
  const int t2 = fdiv(t, g.inv_wi);
  const int hc = t - t2 * g.WI;
  const int img = fdiv(t2, g.inv_tri);
  const int hr = t2 - img * g.TRI;
  const int iy = row0 + hr, ix = hc - 1, b = b0 + img;
  return (b < g.Bn && iy >= 0 && iy < g.H && ix >= 0 && ix < g.H)
             ? ((b * g.H + iy) * g.H + ix) * CI + 8 * cc
             : -1;
}

// relu(x sc + sh) of one chunk (8 channels starting at 8 cc), tab = [2][CI] (scale, shift)
template <int CI>
__device__ __forceinline__ uint4 bnin_chunk(uint4 v, const float* tab, int cc) {
  const f32x4 sa = *(const f32x4*)(tab + 8 * cc), sb = *(const f32x4*)(tab + 8 * cc + 4);
  const f32x4 ha = *(const f32x4*)(tab + CI + 8 * cc);
  const f32x4 hb = *(const f32x4*)(tab + CI + 8 * cc + 4);
  const float sc[8] = {sa[0], sa[1], sa[2], sa[3], sb[0], sb[1], sb[2], sb[3]};
  const float sh[8] = {ha[0], ha[1], ha[2], ha[3], hb[0], hb[1], hb[2], hb[3]};
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float lo = fmaxf(bf2f(w[e] & 0xFFFF) * sc[2 * e] + sh[2 * e] + 0.f, 0.f);
    const float hi = fmaxf(bf2f(w[e] >> 16) * sc[2 * e + 1] + sh[2 * e + 1] + 0.f, 0.f);
    w[e] = pack2bf(lo, hi);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ int halo_chunks(const Geom& g, int cc) {
  return g.IMGS * g.TRI * g.WI * cc;
}

// NPF: halo chunks per thread held in registers -- enough for a band of the image side this
// shape has in a CIFAR ResNet (16 channels at 32 x 32, 32 at 16 x 16, 64 at 8 x 8; make_geom's
// arithmetic); other sides stage the chunks past NPF synchronously.  Capped at 10 (40 VGPRs).
template <int CI, int CO, int S, int NPX, int MODE>
constexpr int halo_pf() {
  // kDgrad2: H is the (full-resolution) output side, the output has CO channels
  const int c = MODE == 2 ? CO : CI;
  const int H = c <= 16 ? 32 : 512 / c;
  const int OH = MODE == 2 ? H : H / S;
  const int px = OH * OH;
  const int imgs = px >= NPX ? 1 : NPX / px;
  const int tr = px >= NPX ? NPX / OH : OH;
  const int tri = MODE == 2 ? tr / 2 + 2 : (tr - 1) * S + 3;
  const int wi = MODE == 2 ? OH / 2 + 2 : (OH - 1) * S + 3;
  const int n = (imgs * tri * wi * (CI / 8) + 255) / 256;
  const int cap = CI >= 64 || CO >= 64 ? 3 : 10;
  return n < 1 ? 1 : (n > cap ? cap : n);
}

// the register half of the pipelined halo staging (plain arrays in the kernel, passed by
// reference into these force-inlined helpers)
template <int CI, int NPF>
__device__ __forceinline__ void halo_fetch(uint4 (&v)[NPF], uint32_t& ok, const bf16_t* x,
                                           const Geom& g, int b0, int row0) {
  const int n = halo_chunks(g, CI / 8);
  ok = 0;
#pragma unroll
  for (int i = 0; i < NPF; ++i) {
    const int c = opaque(threadIdx.x + 256 * i);
    const int o = halo_src<CI>(g, b0, row0, min(c, n - 1));
    ok |= (c < n && o >= 0) ? (1u << i) : 0u;
    v[i] = *(const uint4*)(x + (uint32_t)(o < 0 ? 0 : o));
  }
}

template <int CI, int S, int NPF, int BNIN>
__device__ __forceinline__ void halo_put(bf16_t* hs, const uint4 (&v)[NPF], uint32_t ok,
                                         const bf16_t* x, const Geom& g, int b0, int row0,
                                         const float* tab) {
  constexpr int CC = CI / 8;
  const int n = halo_chunks(g, CC);
#pragma unroll
  for (int i = 0; i < NPF; ++i) {
    const int c = opaque(threadIdx.x + 256 * i);
    if (c < n) {
      uint4 w = make_uint4(0, 0, 0, 0);
      if ((ok >> i) & 1u) w = BNIN ? bnin_chunk<CI>(v[i], tab, c % CC) : v[i];
      *(uint4*)(hs + (c / CC) * pstride<CI, S>() + 8 * (c % CC)) = w;
    }
  }
  for (int c = threadIdx.x + 256 * NPF; c < n; c += 256) {   // past the registers: synchronous
    const int o = halo_src<CI>(g, b0, row0, c);
    uint4 w = make_uint4(0, 0, 0, 0);
    if (o >= 0) {
      w = *(const uint4*)(x + o);
      if (BNIN) w = bnin_chunk<CI>(w, tab, c % CC);
    }
    *(uint4*)(hs + (c / CC) * pstride<CI, S>() + 8 * (c % CC)) = w;
  }
}

// BNIN prologue: the workgroup's trial's (scale, shift) = (gamma rstd, beta - mean scale) into
// the LDS table (published by the caller's next barrier)
struct BnIn {
  const float* stat;     // [P][2][C] mean, rstd
  const bf16_t* gamma;   // [P][C]
  const bf16_t* beta;    // [P][C]
  const bf16_t* x;       // BNB data gradients: the BatchNorm's input, shaped like the output
  const bf16_t* y;       // BNB 2: the BatchNorm's (post-ReLU) output, relu' read off it
  // BNIN 2 (a block output relu(BN(x) + shortcut) as the operand): the shortcut -- shaped like x
  // (res_c = 0) or the option-A shortcut of a block input at twice the side with res_c channels
  // (res_c > 0: pixel (2i, 2j), channels >= res_c zero); rmul 0: no shortcut (the stem's
  // relu(BN(x)); res then points at x) -- and the materialised output `out`, shaped like x
  const bf16_t* res;
  bf16_t* out;
  int res_c;
  float rmul;
  // BNIN forwards that finalize the BatchNorm themselves (round 6: one bn_finalize_kernel launch
  // less per BatchNorm): xsums [P][2][C] the batch sums of x, from which every workgroup derives
  // its table; the trial's first workgroup also stores stat (mean, rstd, for the backward) and
  // the running-statistics update -- bn_finalize_kernel's arithmetic, operation for operation
  const float* xsums;
  float* stat_w;
  float* running;
  float Mf, Mm1f, eps, momentum;
};

// BNIN 2 staging: relu(fma(x, sc, sh) + shortcut) of one chunk (bn_apply_kernel's arithmetic:
// the materialised block output is bit-identical to the separate pass's)
template <int CI>
__device__ __forceinline__ uint4 bnres_chunk(uint4 v, uint4 r, bool rz, float rmul,
                                             const float* tab, int cc) {
  const f32x4 sa = *(const f32x4*)(tab + 8 * cc), sb = *(const f32x4*)(tab + 8 * cc + 4);
  const f32x4 ha = *(const f32x4*)(tab + CI + 8 * cc);
  const f32x4 hb = *(const f32x4*)(tab + CI + 8 * cc + 4);
  const float sc[8] = {sa[0], sa[1], sa[2], sa[3], sb[0], sb[1], sb[2], sb[3]};
  const float sh[8] = {ha[0], ha[1], ha[2], ha[3], hb[0], hb[1], hb[2], hb[3]};
  const bool use = !rz && rmul != 0.f;   // (a select, not 0 * r: r may be non-finite)
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
  const uint32_t rw[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float lo = fmaxf(fmaf(bf2f(w[e] & 0xFFFF), sc[2 * e], sh[2 * e]) +
                               (use ? bf2f(rw[e] & 0xFFFF) : 0.f), 0.f);
    const float hi = fmaxf(fmaf(bf2f(w[e] >> 16), sc[2 * e + 1], sh[2 * e + 1]) +
                               (use ? bf2f(rw[e] >> 16) : 0.f), 0.f);
    w[e] = pack2bf(lo, hi);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// element offset of the shortcut chunk matching x's chunk at offset o (trial-relative, x of side
// 1 << hl with CI channels); rz: the chunk's channels are past an option-A shortcut's res_c
template <int CI, int RK>
__device__ __forceinline__ int res_off(int o, int hl, int res_c, bool& rz) {
  if constexpr (RK == 0) {   // shortcut shaped like x (or none)
    rz = false;
    return o;
  }
  const int pix = o / CI, c8 = o % CI, side = 1 << hl;
  const int ix = pix & (side - 1), iy = (pix >> hl) & (side - 1), b = pix >> (2 * hl);
  rz = c8 >= res_c;
  return ((b * 2 * side + 2 * iy) * 2 * side + 2 * ix) * res_c + (rz ? 0 : c8);
}

// BNIN 2 fetch: x and the shortcut of the halo chunks (every load unconditional, as halo_fetch)
template <int CI, int NPF, int RK>
__device__ __forceinline__ void halo_fetch_res(uint4 (&v)[NPF], uint4 (&r)[NPF], uint32_t& ok,
                                               const bf16_t* x, const bf16_t* rp,
                                               const BnIn& bn, const Geom& g, int b0, int row0,
                                               int hl) {
  const int n = halo_chunks(g, CI / 8);
  ok = 0;
#pragma unroll
  for (int i = 0; i < NPF; ++i) {
    const int c = opaque(threadIdx.x + 256 * i);
    const int o = halo_src<CI>(g, b0, row0, min(c, n - 1));
    ok |= (c < n && o >= 0) ? (1u << i) : 0u;
    const int oo = o < 0 ? 0 : o;
    bool rz;
    const int ro = res_off<CI, RK>(oo, hl, bn.res_c, rz);
    v[i] = *(const uint4*)(x + (uint32_t)oo);
    r[i] = *(const uint4*)(rp + (uint32_t)ro);
  }
}

// is halo chunk c an interior pixel of the band (its own output rows' input pixels -- the bands
// tile the input exactly) rather than a halo row / column shared with a neighbour
template <int CI, int S>
__device__ __forceinline__ bool halo_interior(const Geom& g, int c) {
  const int t = c / (CI / 8);
  const int t2 = fdiv(t, g.inv_wi);
  const int hc = t - t2 * g.WI;
  const int img = fdiv(t2, g.inv_tri);
  const int hr = t2 - img * g.TRI;
  constexpr int E = S == 1 ? 2 : 1;
  return hr >= 1 && hr <= g.TRI - E && hc >= 1 && hc <= g.WI - E;
}

// BNIN 2 put: the block output into the LDS band and, for the band's interior pixels, to HBM
template <int CI, int S, int NPF, int RK>
__device__ __forceinline__ void halo_put_res(bf16_t* hs, const uint4 (&v)[NPF],
                                             const uint4 (&r)[NPF], uint32_t ok, const bf16_t* x,
                                             const bf16_t* rp, bf16_t* op, const BnIn& bn,
                                             const Geom& g, int b0, int row0, int hl,
                                             const float* tab) {
  constexpr int CC = CI / 8;
  const int n = halo_chunks(g, CC);
#pragma unroll
  for (int i = 0; i < NPF; ++i) {
    const int c = opaque(threadIdx.x + 256 * i);
    if (c < n) {
      uint4 w = make_uint4(0, 0, 0, 0);
      if ((ok >> i) & 1u) {
        const int o = halo_src<CI>(g, b0, row0, c);
        bool rz;
        res_off<CI, RK>(o, hl, bn.res_c, rz);
        w = bnres_chunk<CI>(v[i], r[i], rz, bn.rmul, tab, c % CC);
        if (halo_interior<CI, S>(g, c)) *(uint4*)(op + o) = w;
      }
      *(uint4*)(hs + (c / CC) * pstride<CI, S>() + 8 * (c % CC)) = w;
    }
  }
  for (int c = threadIdx.x + 256 * NPF; c < n; c += 256) {   // past the registers: synchronous
    const int o = halo_src<CI>(g, b0, row0, c);
    uint4 w = make_uint4(0, 0, 0, 0);
    if (o >= 0) {
      bool rz;
      const int ro = res_off<CI, RK>(o, hl, bn.res_c, rz);
      w = bnres_chunk<CI>(*(const uint4*)(x + o), *(const uint4*)(rp + ro), rz, bn.rmul, tab,
                          c % CC);
      if (halo_interior<CI, S>(g, c)) *(uint4*)(op + o) = w;
    }
    *(uint4*)(hs + (c / CC) * pstride<CI, S>() + 8 * (c % CC)) = w;
  }
}

template <int CI>
__device__ __forceinline__ void bnin_table(float* tab, const BnIn& bn, int p, bool first) {
  for (int i = threadIdx.x; i < CI; i += 256) {
    float mean, rstd;
    if (bn.xsums != nullptr) {
      mean = bn.xsums[(2 * p) * CI + i] / bn.Mf;
      const float var = fmaxf(bn.xsums[(2 * p + 1) * CI + i] / bn.Mf - mean * mean, 0.f);
      rstd = rsqrtf(var + bn.eps);
      if (first) {
        float* rm = bn.running + (int64_t)p * 2 * CI;
        rm[i] = (1.f - bn.momentum) * rm[i] + bn.momentum * mean;
        rm[CI + i] = (1.f - bn.momentum) * rm[CI + i] + bn.momentum * var * bn.Mf / bn.Mm1f;
        bn.stat_w[(2 * p) * CI + i] = mean;
        bn.stat_w[(2 * p + 1) * CI + i] = rstd;
      }
    } else {
      mean = bn.stat[(2 * p) * CI + i];
      rstd = bn.stat[(2 * p + 1) * CI + i];
    }
    const float sc = bf2f(bn.gamma[(int64_t)p * CI + i]) * rstd;
    tab[i] = sc;
    tab[CI + i] = bf2f(bn.beta[(int64_t)p * CI + i]) - mean * sc;
  }
}

// The band pixel of MFMA fragment row m (0..15) under PIXP: bits (0, 1, 2, 3) of m move to bits
// (1, 2, 0, 3) -- the scripts/lds_banks.py search's conflict-free order for 16 pixels spanning two
// 8-pixel rows of a 80-element-stride halo (MOPT_FWD_PIXP=0: the direct order, A/B builds).
#ifndef MOPT_FWD_PIXP
#define MOPT_FWD_PIXP 1
#endif
template <bool PIXP>
__device__ __forceinline__ int frag_pix(int m) {
  return PIXP ? (((m & 1) << 1) | (((m >> 1) & 1) << 2) | ((m >> 2) & 1) | (m & 8)) : m;
}

// halo offset of output pixel pl of a band (tap (0, 0), channel 0)
template <int CI, int S>
__device__ __forceinline__ int pix_base(const Geom& g, int pl) {
  const int img = pl >> g.rpil, rem = pl & ((1 << g.rpil) - 1);
  const int ly = rem >> g.owl, ox = rem & ((1 << g.owl) - 1);
  return ((img * g.TRI + ly * S) * g.WI + ox * S) * pstride<CI, S>();
}

// halo offset of tap k / CI, channel k % CI (tap clamped to 8: padded k rows meet zero weights)
template <int CI, int S>
__device__ __forceinline__ int tap_off(const Geom& g, int k) {
  const int tap = min(k / CI, 8), c = k % CI;
  const int kh = tap / 3, kw = tap - 3 * kh;
  return (kh * g.WI + kw) * pstride<CI, S>() + c;
}

// ADD: data-gradient epilogue addend -- 0 none, 1 same layout as the output (identity shortcut),
// 2 half-resolution option-A shortcut gradient (compile-time: the epilogue code otherwise costs
// the forward kernels registers and a wave per SIMD)
// BNB (stride-1 data gradient whose output dy feeds a BatchNorm -> ReLU backward, the first
// BatchNorm of a basic block under _BNReluConv3x3): the epilogue also accumulates that backward's
// reductions sums[p][0][c] += dz, sums[p][1][c] += dz xhat (dz = dy relu'(x sc + sh), xhat =
// (x - mean) rstd, x = bn.x) from the stored bf16 dy -- the BatchNorm backward then skips its
// reduction pass (bn_reduce_kernel<true>: both tensors read once more).
// BNB 2 (data gradient of the conv that consumes a block output relu(BN(x) + shortcut), with the
// next block's shortcut gradient as ADD 1 / 2): the stored value is dz = (dgrad + addend) *
// relu'(bn.y) -- the gradient BEHIND that ReLU, which is also the previous block's shortcut
// gradient -- and the epilogue accumulates sum dz, sum dz xhat (xhat from bn.x) as BNB 1 does.
// The BatchNorm backward then runs its apply pass alone without a mask and writes no copy of dz:
// of its reduce (3 tensors), apply (3 read, 2 written) and this epilogue's store, 3 passes and
// a launch go.
// BNIN 2 (forward of the conv that consumes a block output): the operand relu(fma(x, sc, sh) +
// shortcut) is formed while staging (x = the block's last BatchNorm input, bn.res the shortcut),
// and the band's interior pixels of it are also written to bn.out -- the materialised block
// output the next shortcut, the relu' mask of the backward and this conv's weight gradient read:
// bn_apply_kernel's pass (x and shortcut read, output written) is folded into this conv's own
// operand read.
template <int CI, int CO, int NPX, int MODE, int S, int ADD, int BNIN = 0, int BNB = 0>
__global__ __launch_bounds__(256) void dconv_fwd_kernel(const bf16_t* __restrict__ x,
                                                        const bf16_t* __restrict__ w,
                                                        bf16_t* __restrict__ y,
                                                        float* __restrict__ sums,
                                                        const bf16_t* __restrict__ addend,
                                                        const Geom g, int addend_c,
                                                        const BnIn bn) {
  static_assert(BNIN == 0 || MODE == kFwd, "the BatchNorm input is applied by forwards only");
  static_assert(BNB != 1 || (MODE == kDgrad && ADD == 0), "BNB 1: plain stride-1 data gradients");
  static_assert(BNB != 2 || (MODE != kFwd && ADD != 0), "BNB 2: data gradients with an addend");
  constexpr int mode = MODE;
  constexpr int KS = (9 * CI + 31) / 32;  // 32-wide k steps (k = tap * CI + c)
  constexpr int WN = CO / 16, WM = 4 / WN;
  constexpr int MFW = NPX / 16 / WM;      // 16-pixel fragments per wave
  constexpr int LSC = CO + 8;
  // 64 channels at stride 1 (8 x 8 images: a fragment's 16 pixels are two image rows): fragment
  // row li multiplies band pixel frag_pix(li) -- with the direct order the two rows' halo pixels
  // met the same banks (4 extra cycles per A-fragment read on every pixel stride, 2.9 measured);
  // the epilogue stores C row m at tile row frag_pix(m), so the copy-out is unchanged
  constexpr bool PIXP = MOPT_FWD_PIXP && CI >= 64 && S == 1 && MODE != kDgrad2;
  // (64-channel data gradients with an addend: one prefetched chunk -- the addend registers on
  //  top of a full prefetch cost the kernel its second workgroup per CU, 51 -> 72 us in situ)
  // (BNIN 2 / 3: x and the shortcut in flight -- at most 3 chunks of each, the rest of a band
  //  staged synchronously, so the 16-channel stride-2 and 32-channel kernels keep 2 workgroups
  //  per CU)
  constexpr int NPF = (CO >= 64 && ADD != 0) ? 1
                      : BNIN >= 2 ? (halo_pf<CI, CO, S, NPX, MODE>() < 3 ? halo_pf<CI, CO, S, NPX, MODE>() : 3)
                                  : halo_pf<CI, CO, S, NPX, MODE>();
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  bf16_t* hs = smem;
  // the output tile: its own LDS region when the launch found room (cs_off > 0: the band's
  // copy-out overlaps the next band), else restaged over the halo band once the MFMAs are done
  bf16_t* cs = smem + g.cs_off;
  const bool alias = g.cs_off == 0;

  const int p = blockIdx.x / g.nb, blk = blockIdx.x % g.nb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, gq = lane >> 4;
  const int wm = wave / WN, wn = wave % WN;
  const int n = 16 * wn + li;
  const int64_t wbatch = (int64_t)9 * CI * CO;
  const bf16_t* wp = w + p * wbatch;
  const int64_t x_batch = (int64_t)g.Bn * g.H * g.H * CI;
  const bf16_t* xp = x + (g.x_shared ? 0 : p * x_batch);
  auto band_row0 = [&](int t) {
    const int oy = (t % g.tpi) * g.TR;
    return mode == kDgrad2 ? oy / 2 - 1 : oy * S - 1;
  };

  // the first band's halo is in flight during the weight prologue
  uint4 hv[NPF];
  uint32_t hok;
  // BNIN 2: the shortcut chunks beside x's, the trial's shortcut / output bases
  constexpr bool BR = BNIN >= 2;
  constexpr int RK = BNIN == 3 ? 1 : 0;
  uint4 rv[BR ? NPF : 1];
  const int hl = 31 - __builtin_clz(g.H);
  const bf16_t* rp = !BR ? nullptr
                     : RK ? bn.res + p * ((int64_t)g.Bn * 4 * g.H * g.H * bn.res_c)
                          : bn.res + p * x_batch;
  bf16_t* op = BR ? bn.out + p * x_batch : nullptr;
  if constexpr (BR)
    halo_fetch_res<CI, NPF, RK>(hv, rv, hok, xp, rp, bn, g, (blk / g.tpi) * g.IMGS, band_row0(blk),
                            hl);
  else
    halo_fetch<CI, NPF>(hv, hok, xp, g, (blk / g.tpi) * g.IMGS, band_row0(blk));

  // this wave's B fragments for every k step
  bf16x8 wr[KS];
  if constexpr (MODE == kFwd) {
    // W [9 CI][CO] is n-contiguous: staged through LDS in k chunks and read back transposed
    // (ds_read_b64_tr_b16), so neither a transposed copy nor 2-byte gathers are needed
    static_assert((NPX * LSC / CO) / 32 >= 1, "weight chunk");
    const int KCH = min(KS * 32, (g.lds_elems / CO) / 32 * 32);  // k rows per chunk
    const int q = li >> 2, pp = li & 3;
    for (int c0 = 0; c0 < KS * 32; c0 += KCH) {
      for (int c = threadIdx.x; c < KCH * (CO / 8); c += 256) {
        const int r = c / (CO / 8), cc = c % (CO / 8);
        uint4 v = make_uint4(0, 0, 0, 0);
        if (c0 + r < 9 * CI) v = *(const uint4*)(wp + (int64_t)(c0 + r) * CO + 8 * cc);
        *(uint4*)(smem + r * CO + 8 * cc) = v;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < KS; ++j) {
        if (32 * j < c0 || 32 * j >= c0 + KCH) continue;
        const int r = 32 * j - c0 + 8 * gq + q;
        wr[j] = cat_frag(lds_tr4(smem + r * CO + 16 * wn + 4 * pp),
                         lds_tr4(smem + (r + 4) * CO + 16 * wn + 4 * pp));
      }
      __syncthreads();
    }
  } else {
#pragma unroll
    for (int j = 0; j < KS; ++j) {
      const int k0 = 32 * j + 8 * gq;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (k0 < 9 * CI) {
        const int tp = k0 / CI, c = k0 % CI;
        const int64_t off = mode == kDgrad
                                ? ((int64_t)(8 - tp) * CO + n) * CI + c  // flip, W [9 CO][CI]
                                : ((int64_t)tp * CO + n) * CI + c;       // kDgrad2: unflipped
        v = *(const uint4*)(wp + off);
      }
      wr[j] = __builtin_bit_cast(bf16x8, v);
    }
  }

  const int64_t y_batch = (int64_t)g.Bn * g.OH * (1 << g.owl) * CO;
  bf16_t* yp = y + p * y_batch;
  const int ppi = 1 << g.rpil;  // band pixels per image

  // this lane's pixel of each of its fragments (the band geometry is the same for every band)
  int pb[MFW], ply[MFW], pox[MFW];
#pragma unroll
  for (int i = 0; i < MFW; ++i) {
    const int pl = (wm * MFW + i) * 16 + li;
    pb[i] = pix_base<CI, S>(g, (wm * MFW + i) * 16 + frag_pix<PIXP>(li));
    const int rem = pl & ((1 << g.rpil) - 1);
    ply[i] = ((pl >> g.rpil) * g.TRI) * 2 + (rem >> g.owl);  // kDgrad2: 2 img TRI + ly
    pox[i] = rem & ((1 << g.owl) - 1);
  }

  float s1 = 0.f, s2 = 0.f;
  float* bntab = (float*)(smem + g.lds_elems);  // BNIN: [2][CI] past the halo / output tile
  // output chunks (8 channels) per thread and band; BNB: a thread's chunk is the same in every
  // band (CO / 8 | 256), so it keeps that chunk's relu' constants and raw sums (sum dz, sum dz
  // x -- turned into sum dz xhat once, at the end: 32 registers instead of 48)
  constexpr int CPR = CO / 8;
  constexpr int XCH = (NPX * CPR + 255) / 256;
  float bsc[8], bsh[8], ba[8], bb[8];
  // BNB: the band's BatchNorm input; ADD: the band's addend -- loaded before the next band's
  // halo fetch and used by the band's copy-out (one band later)
  uint4 xr[(BNB != 0 || ADD != 0) ? XCH : 1];
  // BNB 2: the BatchNorm's output (relu' mask) and input (xhat) of the band, loaded beside the
  // addend -- except at 64 channels, where the 32 more registers cost the second workgroup per
  // CU: loaded by the copy-out itself
  constexpr bool BPF = BNB == 2 && CO < 64;
  uint4 yr[BPF ? XCH : 1], cr[BPF ? XCH : 1];
  if constexpr (BNB != 0) {
    const int c0 = 8 * (threadIdx.x % CPR);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if constexpr (BNB == 1) {
        const float mean = bn.stat[(2 * p) * CO + c0 + e];
        bsc[e] = bf2f(bn.gamma[(int64_t)p * CO + c0 + e]) * bn.stat[(2 * p + 1) * CO + c0 + e];
        bsh[e] = bf2f(bn.beta[(int64_t)p * CO + c0 + e]) - mean * bsc[e];
      }
      ba[e] = bb[e] = 0.f;
    }
  }
  if constexpr (BNIN != 0) {
    bnin_table<CI>(bntab, bn, p, blk == 0);
    __syncthreads();
  }
  // Band loop, one band behind on the copy-out: put(t) -> barrier -> copy-out(t - 1) -> loads
  // of t's addend / BatchNorm input and of band t + nb's halo -> MFMAs(t) -> barrier -> C(t) to
  // LDS.  Aliased output tile: the copy-out of t - 1 finishes before put(t) overwrites it.
  int pt = -1;                 // the band whose output tile is in LDS
  for (int t = blk;; t += g.nb) {
    const bool have = t < g.tiles;
    const int b0 = (t / g.tpi) * g.IMGS, oy0 = (t % g.tpi) * g.TR;
    if (have && !alias) {
      if constexpr (BR)
        halo_put_res<CI, S, NPF, RK>(hs, hv, rv, hok, xp, rp, op, bn, g, b0, band_row0(t), hl, bntab);
      else
        halo_put<CI, S, NPF, BNIN>(hs, hv, hok, xp, g, b0, band_row0(t), bntab);
    }
    __syncthreads();
    if (pt >= 0) {
      // ---- copy-out of band pt: contiguous (b0, oy0 .. oy0 + TR) or whole images b0 .. ----
      const int pb0 = (pt / g.tpi) * g.IMGS, poy0 = (pt % g.tpi) * g.TR;
      const int valid = min(NPX, (g.Bn - pb0) * ppi);
      bf16_t* yt = yp + ((int64_t)pb0 * g.OH + poy0) * (1 << g.owl) * CO;
#pragma unroll
      for (int k = 0; k < XCH; ++k) {
        const int c = threadIdx.x + 256 * k;
        if (c >= valid * CPR) break;
        const int row = c / CPR, cc = c % CPR;
        uint4 v = *(const uint4*)(cs + row * LSC + 8 * cc);
        bool add = ADD == 1;
        if constexpr (ADD == 2) {   // option-A shortcut: its gradient lands on even pixels
          const int rem = row & ((1 << g.rpil) - 1);
          const int oy = poy0 + (rem >> g.owl), ox = rem & ((1 << g.owl) - 1);
          add = ((oy | ox) & 1) == 0;
        }
        if (ADD != 0 && add) {  // data gradient + the shortcut branch's gradient
          const uint4 a = xr[k];
          const uint32_t vw[4] = {v.x, v.y, v.z, v.w}, aw[4] = {a.x, a.y, a.z, a.w};
          uint32_t o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            o[e] = pack2bf(bf2f(vw[e] & 0xFFFF) + bf2f(aw[e] & 0xFFFF),
                           bf2f(vw[e] >> 16) + bf2f(aw[e] >> 16));
          v = make_uint4(o[0], o[1], o[2], o[3]);
        }
        if constexpr (BNB == 2) {  // dz = g relu'(y); sum dz, sum dz x (bn_reduce relu mode 1)
          uint4 yq, xq;
          if constexpr (BPF) {
            yq = yr[k];
            xq = cr[k];
          } else {
            const int64_t o = (yt - y) + (int64_t)row * CO + 8 * cc;
            yq = *(const uint4*)(bn.y + o);
            xq = *(const uint4*)(bn.x + o);
          }
          const uint32_t yw[4] = {yq.x, yq.y, yq.z, yq.w}, xw[4] = {xq.x, xq.y, xq.z, xq.w};
          uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float lo = bf2f(yw[e] & 0xFFFF) <= 0.f ? 0.f : bf2f(vw[e] & 0xFFFF);
            const float hi = bf2f(yw[e] >> 16) <= 0.f ? 0.f : bf2f(vw[e] >> 16);
            vw[e] = (bf2f(yw[e] & 0xFFFF) <= 0.f ? 0u : (vw[e] & 0xFFFFu)) |
                    (bf2f(yw[e] >> 16) <= 0.f ? 0u : (vw[e] & 0xFFFF0000u));
            ba[2 * e] += lo;
            bb[2 * e] += lo * bf2f(xw[e] & 0xFFFF);
            ba[2 * e + 1] += hi;
            bb[2 * e + 1] += hi * bf2f(xw[e] >> 16);
          }
          v = make_uint4(vw[0], vw[1], vw[2], vw[3]);
        }
        *(uint4*)(yt + (int64_t)row * CO + 8 * cc) = v;
        if constexpr (BNB == 1) {
          const uint4 xq = xr[k];
          const uint32_t vw[4] = {v.x, v.y, v.z, v.w}, xw[4] = {xq.x, xq.y, xq.z, xq.w};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = bf2f(e & 1 ? vw[e >> 1] >> 16 : vw[e >> 1] & 0xFFFF);
            const float xv = bf2f(e & 1 ? xw[e >> 1] >> 16 : xw[e >> 1] & 0xFFFF);
            // bn_reduce_kernel<true>'s relu mode 2 arithmetic
            const float dz = xv * bsc[e] + bsh[e] + 0.f <= 0.f ? 0.f : d;
            ba[e] += dz;
            bb[e] += dz * xv;
          }
        }
      }
    }
    if (alias) {
      __syncthreads();   // the copy-out is done with the tile the halo overwrites
      if (have) {
        if constexpr (BR)
          halo_put_res<CI, S, NPF, RK>(hs, hv, rv, hok, xp, rp, op, bn, g, b0, band_row0(t), hl,
                                   bntab);
        else
          halo_put<CI, S, NPF, BNIN>(hs, hv, hok, xp, g, b0, band_row0(t), bntab);
      }
      __syncthreads();
    }
    if (!have) break;
    const int valid = min(NPX, (g.Bn - b0) * ppi);
    if constexpr (BNB != 0 || ADD != 0) {   // (row clamped: every load unconditional)
      const bf16_t* yt = yp + ((int64_t)b0 * g.OH + oy0) * (1 << g.owl) * CO;
#pragma unroll
      for (int k = 0; k < XCH; ++k) {
        const int c = min(threadIdx.x + 256 * k, valid * CPR - 1);
        const int row = c / CPR, cc = c % CPR;
        const bf16_t* src;
        if constexpr (BPF) {
          const int64_t o = (yt - y) + (int64_t)row * CO + 8 * cc;
          yr[k] = *(const uint4*)(bn.y + o);
          cr[k] = *(const uint4*)(bn.x + o);
        }
        if constexpr (BNB == 1) {
          src = bn.x + (yt - y) + (int64_t)row * CO + 8 * cc;
        } else if constexpr (ADD == 1) {  // identity shortcut: same layout as the output
          src = addend + (yt - y) + (int64_t)row * CO + 8 * cc;
        } else {   // option-A shortcut [P Bn][OH / 2][OH / 2][addend_c], even pixels only
          const int b = b0 + (row >> g.rpil), rem = row & ((1 << g.rpil) - 1);
          const int oy = oy0 + (rem >> g.owl), ox = rem & ((1 << g.owl) - 1);
          const int hs2 = g.OH >> 1;
          src = addend + ((((int64_t)p * g.Bn + b) * hs2 + (oy >> 1)) * hs2 + (ox >> 1)) *
                             addend_c + 8 * cc;
        }
        xr[k] = *(const uint4*)src;
      }
    }
    {   // the next band's halo (the current one again past the last: loads stay unconditional)
      const int tn = t + g.nb < g.tiles ? t + g.nb : t;
      if constexpr (BR)
        halo_fetch_res<CI, NPF, RK>(hv, rv, hok, xp, rp, bn, g, (tn / g.tpi) * g.IMGS,
                                band_row0(tn), hl);
      else
        halo_fetch<CI, NPF>(hv, hok, xp, g, (tn / g.tpi) * g.IMGS, band_row0(tn));
    }

    f32x4 acc[MFW];
#pragma unroll
    for (int i = 0; i < MFW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (MODE != kDgrad2) {
#pragma unroll
      for (int j = 0; j < KS; ++j) {
        const int to = tap_off<CI, S>(g, 32 * j + 8 * gq);
#pragma unroll
        for (int i = 0; i < MFW; ++i) acc[i] = mfma16(lds_frag(hs + pb[i] + to), wr[j], acc[i]);
      }
    } else {
      // stride-2 data gradient (transposed convolution): output pixel (ly, ox) takes dy at
      // ((ly + 1 - kh) / 2, (ox + 1 - kw) / 2) for the taps whose divisions are exact (oy0 even)
#pragma unroll
      for (int j = 0; j < KS; ++j) {
        const int k0 = 32 * j + 8 * gq;
        const int tap = min(k0 / CI, 8), c = k0 % CI;
        const int kh = tap / 3, kw = tap - 3 * kh;
#pragma unroll
        for (int i = 0; i < MFW; ++i) {
          // ply = 2 img TRI + ly: parity and halving act on ly alone
          const int ny = ply[i] + 1 - kh, nx = pox[i] + 1 - kw;
          const bf16x8 f = lds_frag(hs + (((ny >> 1) + 1) * g.WI +
                                          (nx >> 1) + 1) * pstride<CI, S>() + c);
          const bf16x8 z = __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0));
          acc[i] = mfma16(((ny | nx) & 1) ? z : f, wr[j], acc[i]);
        }
      }
    }

    __syncthreads();  // every wave is done with the halo band (and with the previous copy-out)
#pragma unroll
    for (int i = 0; i < MFW; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = (wm * MFW + i) * 16 + frag_pix<PIXP>(4 * gq + r);
        const bf16_t v = f2bf(acc[i][r]);
        cs[row * LSC + n] = v;
        if (row < valid) {
          const float f = bf2f(v);
          s1 += f;
          s2 += f * f;
        }
      }
    pt = t;
  }
  if constexpr (BNB != 0) {
    // threads of one chunk: lanes equal mod CPR (xor over the lane bits above log2 CPR), then
    // the 4 waves through LDS (the tile is free after the last barrier), one atomic per channel
    for (int off = 32; off >= CPR; off >>= 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        ba[e] += __shfl_xor(ba[e], off, 64);
        bb[e] += __shfl_xor(bb[e], off, 64);
      }
    }
    float* red = (float*)smem;   // [4 waves][2][CO]
    if (lane < CPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(wave * 2) * CO + 8 * lane + e] = ba[e];
        red[(wave * 2 + 1) * CO + 8 * lane + e] = bb[e];
      }
    }
    __syncthreads();
    if (threadIdx.x < CO) {     // sum dz xhat = rstd (sum dz x - mean sum dz)
      const int c = threadIdx.x;
      const float a = red[c] + red[2 * CO + c] + red[4 * CO + c] + red[6 * CO + c];
      const float bx = red[CO + c] + red[3 * CO + c] + red[5 * CO + c] + red[7 * CO + c];
      const float mean = bn.stat[(2 * p) * CO + c], rstd = bn.stat[(2 * p + 1) * CO + c];
      atomicAdd(sums + (2 * p) * CO + c, a);
      atomicAdd(sums + (2 * p + 1) * CO + c, rstd * (bx - mean * a));
    }
  }
  if (BNB == 0 && sums != nullptr) {   // (BNB: sums holds the backward reductions above)
    s1 += __shfl_xor(s1, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 16, 64);
    s2 += __shfl_xor(s2, 32, 64);
    if (gq == 0) {
      atomicAdd(sums + (2 * p) * CO + n, s1);
      atomicAdd(sums + (2 * p + 1) * CO + n, s2);
    }
  }
}

// weight-gradient dy tile row stride (elements): with 8 consecutive pixel rows per transposed
// read (below) a row stride of 8 dwords x an odd number spreads them over all 64 banks
// (MOPT_WGRAD_PERM=0: the direct pixel order and CO + 8 rows, for A/B builds)
#ifndef MOPT_WGRAD_PERM
#define MOPT_WGRAD_PERM 1
#endif
// (64 channels: 72, 0.2-0.4 modelled extra cycles where 80 has none -- 80 pushes the stride-2
//  32 -> 64 kernel's halo + tile past the 64 KB per workgroup)
constexpr int wgrad_lsd(int co) {
  return !MOPT_WGRAD_PERM ? co + 8 : co == 16 ? 16 : co == 32 ? 48 : co + 8;
}

template <int CI, int CO, int NPX, int S, int BNIN = 0>
__global__ __launch_bounds__(256) void dconv_wgrad_kernel(const bf16_t* __restrict__ x,
                                                          const bf16_t* __restrict__ dy,
                                                          float* __restrict__ part,
                                                          const Geom g, int P, const BnIn bn) {
  constexpr int M = 9 * CI;
  constexpr int MFT = (M + 15) / 16, NFT = CO / 16, MFW = (MFT + 3) / 4;
  constexpr int LSD = wgrad_lsd(CO);
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  const int halo = g.IMGS * g.TRI * g.WI * pstride<CI, S>();
  bf16_t* hs = smem;
  bf16_t* ds = smem + halo;   // (halo: a multiple of 8 elements)
  bf16_t* zs = ds + NPX * LSD;  // 8 zero bytes: source of the padded rows m >= 9 CI
  float* bntab = (float*)(zs + 8);  // BNIN: [2][CI] (scale, shift)

  const int p = blockIdx.x / g.nb, blk = blockIdx.x % g.nb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, gq = lane >> 4, q = li >> 2, pp = li & 3;
  if (threadIdx.x == 0) *(uint2*)zs = make_uint2(0, 0);
  if constexpr (BNIN != 0) {
    bnin_table<CI>(bntab, bn, p, false);   // (stat read: finalized by the forward)
    __syncthreads();
  }

  // this lane's A column chunk (m = 16 mi + 4 pp .. + 3) of each of the wave's M fragments
  int co_off[MFW];
  bool mvalid[MFW];
#pragma unroll
  for (int i = 0; i < MFW; ++i) {
    const int m = 16 * (wave + 4 * i) + 4 * pp;
    mvalid[i] = m < M;
    co_off[i] = tap_off<CI, S>(g, m);
  }
  f32x4 acc[MFW][NFT];
#pragma unroll
  for (int i = 0; i < MFW; ++i)
#pragma unroll
    for (int j = 0; j < NFT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int NKS = NPX / 32;
  const int ow = 1 << g.owl, ppi = 1 << g.rpil;
  const bf16_t* xp = x + (g.x_shared ? 0 : p * ((int64_t)g.Bn * g.H * g.H * CI));
  const bf16_t* dyp = dy + p * ((int64_t)g.Bn * g.OH * ow * CO);
  // pipelined staging (see Halo): band t + nb's halo and dy tile are loaded into registers while
  // band t is multiplied (the dy rows past a partial band's end re-read its last row, zeroed at
  // the store, so every load is unconditional)
  constexpr int NPF = halo_pf<CI, CO, S, NPX, kFwd>();
  // 64 output channels: the 144 accumulator registers leave no room for a band in flight (one
  // workgroup per CU with it, 43 -> 62 us in situ): fetched at the top of the band instead
  constexpr bool PFW = CO < 64;
  constexpr int CPR = CO / 8;
  constexpr int DYC = (NPX * CPR + 255) / 256;
  uint4 hv[NPF], dv[DYC];
  uint32_t hok;
  auto fetch = [&](int t) {
    const int b0 = (t / g.tpi) * g.IMGS, oy0 = (t % g.tpi) * g.TR;
    halo_fetch<CI, NPF>(hv, hok, xp, g, b0, oy0 * S - 1);
    const int valid = min(NPX, (g.Bn - b0) * ppi);
    const bf16_t* dyt = dyp + ((int64_t)b0 * g.OH + oy0) * ow * CO;
#pragma unroll
    for (int k = 0; k < DYC; ++k) {
      const int c = min(threadIdx.x + 256 * k, valid * CPR - 1);
      dv[k] = *(const uint4*)(dyt + (int64_t)(c / CPR) * CO + 8 * (c % CPR));
    }
  };
  if (PFW) fetch(blk);
  for (int t = blk; t < g.tiles; t += g.nb) {
    const int b0 = (t / g.tpi) * g.IMGS, oy0 = (t % g.tpi) * g.TR;
    if (!PFW) fetch(t);
    halo_put<CI, S, NPF, BNIN>(hs, hv, hok, xp, g, b0, oy0 * S - 1, bntab);
    const int valid = min(NPX, (g.Bn - b0) * ppi);
#pragma unroll
    for (int k = 0; k < DYC; ++k) {
      const int c = threadIdx.x + 256 * k;
      if (c < NPX * CPR) {
        const int row = c / CPR, cc = c % CPR;
        *(uint4*)(ds + row * LSD + 8 * cc) = row < valid ? dv[k] : make_uint4(0, 0, 0, 0);
      }
    }
    __syncthreads();
    if (PFW) fetch(t + g.nb < g.tiles ? t + g.nb : t);
    // (offsets recomputed per step: hoisting all NKS of them and unrolling fully doubled the
    //  VGPRs of the 16-channel kernel and cost more in occupancy than the ALU saved)
#pragma unroll 2
    for (int ks = 0; ks < NKS; ++ks) {
      // the lane's two pixel rows: k = 8 gq + j of the MFMA (j < 4 from the first transposed
      // read, j >= 4 from the second) is pixel 16 (gq >> 1) + 8 (j >> 2) + 4 (gq & 1) + (j & 3)
      // of the k-step -- any bijection works (A and B share it); this one gives each 32-lane
      // half of a transposed read 8 CONSECUTIVE pixels, 8 x 32 B of distinct banks (the direct
      // order, rows r and r + 8 in one half, conflicted 2-way on every layout: 2.0 extra cycles
      // per read, scripts/lds_banks.py model; 1.8-2.5 measured, profiles/r6/resnet_pmc/)
      const int ka = MOPT_WGRAD_PERM ? 32 * ks + 16 * (gq >> 1) + 4 * (gq & 1) + q
                                     : 32 * ks + 8 * gq + q;
      const int kb = ka + (MOPT_WGRAD_PERM ? 8 : 4);
      const int pa = pix_base<CI, S>(g, ka), pb = pix_base<CI, S>(g, kb);
      bf16x8 b[NFT];
#pragma unroll
      for (int j = 0; j < NFT; ++j)
        b[j] = cat_frag(lds_tr4(ds + ka * LSD + 16 * j + 4 * pp),
                        lds_tr4(ds + kb * LSD + 16 * j + 4 * pp));
#pragma unroll
      for (int i = 0; i < MFW; ++i) {
        if (wave + 4 * i >= MFT) continue;  // wave-uniform
        const bf16x8 a = cat_frag(lds_tr4(mvalid[i] ? hs + pa + co_off[i] : zs),
                                  lds_tr4(mvalid[i] ? hs + pb + co_off[i] : zs));
#pragma unroll
        for (int j = 0; j < NFT; ++j) acc[i][j] = mfma16(a, b[j], acc[i][j]);
      }
    }
    __syncthreads();
  }
  // partial [blk][p][m][n]
  float* out = part + ((int64_t)blk * P + p) * M * CO;
#pragma unroll
  for (int i = 0; i < MFW; ++i) {
    const int mi = wave + 4 * i;
    if (mi >= MFT) continue;
#pragma unroll
    for (int j = 0; j < NFT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * mi + 4 * gq + r;
        if (m < M) out[(int64_t)m * CO + 16 * j + li] = acc[i][j][r];
      }
  }
}

// out[p][i] (bf16, batch stride sO) = sum over the nb partials [nb][P][MN]; 4 elements per
// thread (16-byte partial loads, MN % 4 == 0), the nb loads of a thread issued 4 at a time
__global__ __launch_bounds__(256) void dconv_reduce_kernel(const float* __restrict__ part,
                                                           bf16_t* __restrict__ out, int64_t sO,
                                                           int P, int MN, int nb) {
  const int64_t total = (int64_t)P * MN;
  const int64_t i = 4 * ((int64_t)blockIdx.x * 256 + threadIdx.x);
  if (i >= total) return;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  int k = 0;
  for (; k + 4 <= nb; k += 4) {
    const f32x4 a = *(const f32x4*)(part + k * total + i);
    const f32x4 b = *(const f32x4*)(part + (k + 1) * total + i);
    const f32x4 c = *(const f32x4*)(part + (k + 2) * total + i);
    const f32x4 d = *(const f32x4*)(part + (k + 3) * total + i);
    s += (a + b) + (c + d);
  }
  for (; k < nb; ++k) s += *(const f32x4*)(part + k * total + i);
  bf16_t* o = out + (i / MN) * sO + i % MN;  // 4 | MN: the 4 elements share a trial
  *(uint2*)o = f32_to_bf4(s);
}

int ilog2i(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return (1 << l) == v ? l : -1;
}

constexpr int npx_for(int co) { return co >= 64 ? 128 : 256; }
// persistent weight-gradient workgroups in all: ResNet-20 (32 trials) at 512 / 768 / 1024 / 2048
// / 4096: 5.75 / 5.58 / 5.52 / 5.60 / 5.66 ms per step (fewer workgroups: fewer f32 partials for
// the reduce to read; too few: bands no longer hide each other's loads); profiles/r5/conv_blocks
#ifndef MOPT_WGRAD_BLOCKS
#define MOPT_WGRAD_BLOCKS 1024
#endif
// forward / data-gradient workgroups in all (64-wide outputs: half); 512 / 2048: 5.73 / 5.67 ms
#ifndef MOPT_FWD_BLOCKS
#define MOPT_FWD_BLOCKS 1024
#endif
// weight gradient: halo and dy tile live together, so wide outputs take half bands
constexpr int npx_wgrad(int co) { return co >= 32 ? 128 : 256; }

// band geometry: input side H (power of two), stride S, NPX output pixels per band; kDgrad2:
// H is the side of the (full-resolution) output, the input dy is H / 2
bool make_geom(Geom& g, int Bn, int H, int S, int npx, int target_blocks, int P, int mode) {
  const int hl = ilog2i(H);
  if (hl < 0 || Bn < 1 || (S != 1 && S != 2) || (S == 2 && H < 2)) return false;
  // halo offsets are 32-bit element offsets from a trial's base (64 channels at most)
  if ((int64_t)Bn * H * H * 64 >= ((int64_t)1 << 31)) return false;
  g.Bn = Bn;
  g.H = mode == kDgrad2 ? H / 2 : H;
  g.OH = mode == kDgrad2 ? H : H / S;
  const int OW = g.OH;
  g.owl = ilog2i(OW);
  if (OW > npx) return false;
  const int px_img = g.OH * OW;
  g.IMGS = px_img >= npx ? 1 : npx / px_img;
  g.TR = px_img >= npx ? npx / OW : g.OH;
  g.rpil = ilog2i(g.TR * OW);
  g.TRI = mode == kDgrad2 ? g.TR / 2 + 2 : (g.TR - 1) * S + 3;
  g.WI = mode == kDgrad2 ? OW / 2 + 2 : (OW - 1) * S + 3;
  g.inv_wi = 1.f / (float)g.WI;
  g.inv_tri = 1.f / (float)g.TRI;
  g.tpi = g.OH / g.TR;
  g.tiles = ((Bn + g.IMGS - 1) / g.IMGS) * g.tpi;
  int nb = (target_blocks + P - 1) / P;
  g.nb = nb < 1 ? 1 : (nb > g.tiles ? g.tiles : nb);
  return true;
}

template <int CI, int S>
size_t halo_bytes(const Geom& g) { return (size_t)g.IMGS * g.TRI * g.WI * pstride<CI, S>() * 2; }

// S: the stride of the halo layout (kDgrad2 reads its half-resolution dy band at layout S = 1)
template <int CI, int CO, int MODE, int S, int ADD = 0, int BNIN = 0, int BNB = 0>
int launch_fwd(const void* x, const void* w, void* y, void* sums, int P, int Bn, int H,
               hipStream_t st, const void* addend = nullptr, int addend_c = 0,
               const BnIn& bn = BnIn{}, int x_shared = 0) {
  // (the stride-2 data gradient of a 64-channel dy: 128-pixel bands -- at 256 its 18 weight
  //  fragments and 8 accumulator fragments per wave held one workgroup per CU, 0.7 TB/s)
  constexpr int NPX = (MODE == kDgrad2 && CI >= 32) ? 128 : npx_for(CO);
  Geom g{};
  // (64-wide outputs: half the workgroups, twice the bands each -- their weight prologue is long)
  // (the 16-channel BNIN 2 forward holds 3 workgroups per CU, not 4: one wave of them)
  const int blocks = CO >= 64 ? MOPT_FWD_BLOCKS / 2
                     : (BNIN >= 2 && CO == 16) ? MOPT_FWD_BLOCKS * 3 / 4 : MOPT_FWD_BLOCKS;
  if (!make_geom(g, Bn, H, MODE == kDgrad2 ? 2 : S, NPX, blocks, P, MODE))
    return (int)hipErrorInvalidValue;
  const size_t hb = halo_bytes<CI, S>(g), ob = (size_t)NPX * (CO + 8) * 2;
  const size_t tab = BNIN ? (size_t)2 * CI * sizeof(float) : 0;
  // the output tile gets its own region (copy-out overlapped with the next band) when the two
  // fit the 64 KB per workgroup; else it aliases the halo band
  const bool sep = hb + ob + tab <= 64 * 1024;
  const size_t lds = sep ? hb + ob : std::max(hb, ob);
  const size_t lds_all = lds + tab;
  if (lds_all > 64 * 1024) return (int)hipErrorNotSupported;
  g.lds_elems = (int)(lds / 2);
  g.cs_off = sep ? (int)(hb / 2) : 0;
  g.x_shared = x_shared;
  hipLaunchKernelGGL((dconv_fwd_kernel<CI, CO, NPX, MODE, S, ADD, BNIN, BNB>), dim3(P * g.nb),
                     dim3(256), lds_all, st,
                     (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, (float*)sums,
                     (const bf16_t*)addend, g, addend_c, bn);
  return (int)hipGetLastError();
}

template <int CI, int CO, int S, int BNIN = 0>
int launch_wgrad(const void* x, const void* dy, void* dw, void* part, int P, int Bn, int H,
                 hipStream_t st, int* nb_out, const BnIn& bn = BnIn{}, int x_shared = 0) {
  constexpr int NPX = npx_wgrad(CO);
  // persistent workgroups per trial: MOPT_WGRAD_BLOCKS in all, <= 64 MB of f32 partials, >= 4
  // bands each
  constexpr int64_t kPartBytes = 64 << 20;
  const int64_t per = (int64_t)P * 9 * CI * CO * 4;
  const int by_bytes = (int)(kPartBytes / per > 0 ? kPartBytes / per : 1);
  Geom g{};
  if (!make_geom(g, Bn, H, S, NPX, MOPT_WGRAD_BLOCKS, P, kFwd)) return (int)hipErrorInvalidValue;
  g.x_shared = x_shared;
  g.nb = min(g.nb, max(1, min(by_bytes, g.tiles / 4)));
  if (nb_out != nullptr) {  // size query
    *nb_out = g.nb;
    return 0;
  }
  const size_t lds = halo_bytes<CI, S>(g) + (size_t)NPX * wgrad_lsd(CO) * 2 + 16 +
                     (BNIN ? (size_t)2 * CI * sizeof(float) : 0);
  if (lds > 64 * 1024) return (int)hipErrorNotSupported;
  hipLaunchKernelGGL((dconv_wgrad_kernel<CI, CO, NPX, S, BNIN>), dim3(P * g.nb), dim3(256), lds,
                     st, (const bf16_t*)x, (const bf16_t*)dy, (float*)part, g, P, bn);
  const int MN = 9 * CI * CO;
  const int64_t total = (int64_t)P * MN;
  hipLaunchKernelGGL(dconv_reduce_kernel, dim3((unsigned)((total / 4 + 255) / 256)), dim3(256), 0, st,
                     (const float*)part, (bf16_t*)dw, (int64_t)MN, P, MN, g.nb);
  return (int)hipGetLastError();
}

#define MOPT_DCONV_SHAPES(X) X(8, 16) X(16, 16) X(16, 32) X(32, 32) X(32, 64) X(64, 64)
// data gradients run the forward kernel with the channel counts swapped (dy -> dx)
#define MOPT_DCONV_DGRAD_SHAPES(X) X(16, 16) X(32, 16) X(32, 32) X(64, 32) X(64, 64)

}  // namespace

extern "C" {

// Direct 3x3 convolution (pad 1) of a population, NHWC bf16, square power-of-two images:
//   kind 0 forward   y [P*Bn, H/S, H/S, Co] = conv(x [P*Bn, H, H, Ci], w [P, 9 Ci, Co]);
//                    aux = f32 sums [P][2][Co] (zeroed by the caller; += sum, sum^2 of y) or 0
//   kind 1 dgrad     dx [P*Bn, H, H, Ci] from dy [P*Bn, H/S, H/S, Co] and w [P, 9 Ci, Co];
//                    aux = bf16 addend (added in the epilogue) or 0: shaped like dx (aux_c = 0)
//                    or, aux_c > 0, [P*Bn, H/2, H/2, aux_c] added at dx's even pixels to
//                    channels < Ci (the gradient of an option-A shortcut)
//   kind 2 wgrad     dw [P, 9 Ci, Co] (bf16) from x and dy; aux = f32 partials
//                    [nb][P][9 Ci][Co], nb from mopt_dconv_wgrad_splits
// Returns hipErrorNotSupported (801) for shapes without an instantiation: the caller falls
// back to the implicit GEMM (mopt_pconv).
int mopt_dconv(int kind, const void* a, const void* b, void* out, void* aux, int P, int Bn, int H,
               int Ci, int Co, int stride, int aux_c, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (kind == 0) {
#define X(ci, co) \
    if (Ci == ci && Co == co) \
      return stride == 1 ? launch_fwd<ci, co, kFwd, 1>(a, b, out, aux, P, Bn, H, st) \
                         : launch_fwd<ci, co, kFwd, 2>(a, b, out, aux, P, Bn, H, st);
    MOPT_DCONV_SHAPES(X)
#undef X
    return (int)hipErrorNotSupported;
  }
  if (kind == 1) {  // the forward kernel over dy (Co channels) with flipped transposed weights
#define X(ci, co) \
    if (Co == ci && Ci == co) \
      return stride == 1 \
          ? (aux ? launch_fwd<ci, co, kDgrad, 1, 1>(a, b, out, nullptr, P, Bn, H, st, aux) \
                 : launch_fwd<ci, co, kDgrad, 1, 0>(a, b, out, nullptr, P, Bn, H, st)) \
          : (aux ? launch_fwd<ci, co, kDgrad2, 1, 2>(a, b, out, nullptr, P, Bn, H, st, aux, \
                                                     aux_c) \
                 : launch_fwd<ci, co, kDgrad2, 1, 0>(a, b, out, nullptr, P, Bn, H, st));
    MOPT_DCONV_DGRAD_SHAPES(X)
#undef X
    return (int)hipErrorNotSupported;
  }
  if (kind == 2) {
#define X(ci, co) \
    if (Ci == ci && Co == co) \
      return stride == 1 ? launch_wgrad<ci, co, 1>(a, b, out, aux, P, Bn, H, st, nullptr) \
                         : launch_wgrad<ci, co, 2>(a, b, out, aux, P, Bn, H, st, nullptr);
    MOPT_DCONV_SHAPES(X)
#undef X
    return (int)hipErrorNotSupported;
  }
  return (int)hipErrorInvalidValue;
}

// mopt_dconv kinds 0 (forward) and 2 (weight gradient) of a stride-1 convolution whose operand
// is relu(BatchNorm(x)) of the raw BatchNorm input x, applied while the halo bands are staged
// (stat [P][2][Ci] mean / rstd, gamma / beta [P][Ci] bf16): the BatchNorm output is never
// materialised.  Ci == Co in {16, 32, 64} (the second convolution of a ResNet basic block).
// fin (kind 0): xsums [P][2][Ci] the batch sums of x, running [P][2][Ci]; the forward finalizes
// the statistics itself -- stat is written (and the running statistics updated) by the kernel,
// no bn_finalize launch (null: stat holds them already).
int mopt_dconv_bnin(int kind, const void* a, const void* b, void* out, void* aux, int P, int Bn,
                    int H, int Ci, int Co, const void* stat, const void* gamma, const void* beta,
                    const void* xsums, void* running, int64_t M, float eps, float momentum,
                    void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (stat == nullptr || gamma == nullptr || beta == nullptr || (xsums && (kind != 0 || !running)))
    return (int)hipErrorInvalidValue;
  BnIn bn{(const float*)stat, (const bf16_t*)gamma, (const bf16_t*)beta, nullptr};
  if (xsums != nullptr) {
    bn.xsums = (const float*)xsums;
    bn.stat_w = (float*)stat;
    bn.running = (float*)running;
    bn.Mf = (float)M;
    bn.Mm1f = (float)(M - 1 > 1 ? M - 1 : 1);
    bn.eps = eps;
    bn.momentum = momentum;
  }
#define X(c) \
  if (Ci == c && Co == c) \
    return kind == 0 ? launch_fwd<c, c, kFwd, 1, 0, 1>(a, b, out, aux, P, Bn, H, st, nullptr, 0, bn) \
         : kind == 2 ? launch_wgrad<c, c, 1, 1>(a, b, out, aux, P, Bn, H, st, nullptr, bn) \
                     : (int)hipErrorInvalidValue;
  X(16) X(32) X(64)
#undef X
  return (int)hipErrorNotSupported;
}

// Stride-1 data gradient dbn [P*Bn, H, H, Ci] = dgrad(dy [.., Co], w) whose output is the
// gradient of relu(BatchNorm(x)) (x shaped like dbn; stat / gamma / beta of that BatchNorm):
// the epilogue also adds the BatchNorm backward's reductions (sum dz, sum dz xhat, relu'
// recomputed from x) into sums [P][2][Ci] (zeroed by the caller).  Ci == Co in {16, 32, 64}.
int mopt_dconv_dgrad_bnsums(const void* dy, const void* w, void* dbn, void* sums, int P, int Bn,
                            int H, int Ci, int Co, const void* x, const void* stat,
                            const void* gamma, const void* beta, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (sums == nullptr || x == nullptr || stat == nullptr || gamma == nullptr || beta == nullptr)
    return (int)hipErrorInvalidValue;
  const BnIn bn{(const float*)stat, (const bf16_t*)gamma, (const bf16_t*)beta, (const bf16_t*)x};
  // (the data gradient runs the forward kernel with the channel counts swapped: CO = Ci)
#define X(c) \
  if (Ci == c && Co == c) \
    return launch_fwd<c, c, kDgrad, 1, 0, 0, 1>(dy, w, dbn, sums, P, Bn, H, st, nullptr, 0, bn);
  X(16) X(32) X(64)
#undef X
  return (int)hipErrorNotSupported;
}

// Forward of a convolution whose input is a block output relu(BatchNorm(x) + shortcut), formed
// while the input bands are staged: y [P*Bn, H/S, H/S, Co] = conv(relu(fma(x, sc, sh) + res), w)
// with sc = gamma rstd, sh = beta - mean sc (stat [P][2][Ci] mean / rstd, gamma / beta [P][Ci]),
// res shaped like x (res_c = 0), the option-A shortcut of a [P*Bn, 2H, 2H, res_c] block input
// (res_c > 0), or none (res null: the stem's relu(BN(x))); the block output itself is written to
// out (shaped like x) and y's batch sums are added into sums [P][2][Co] (zeroed by the caller).
// xsums / running / M / eps / momentum: as mopt_dconv_bnin's (the statistics finalized here).
int mopt_dconv_bnres_fwd(const void* x, const void* w, void* y, void* sums, void* out,
                         const void* res, int res_c, const void* stat, const void* gamma,
                         const void* beta, int P, int Bn, int H, int Ci, int Co, int stride,
                         const void* xsums, void* running, int64_t M, float eps, float momentum,
                         void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (out == nullptr || stat == nullptr || gamma == nullptr || beta == nullptr ||
      sums == nullptr || (res == nullptr && res_c != 0) || (res_c % 8) || res_c > Ci ||
      (xsums != nullptr && running == nullptr))
    return (int)hipErrorInvalidValue;
  BnIn bn{(const float*)stat, (const bf16_t*)gamma, (const bf16_t*)beta, nullptr, nullptr,
          (const bf16_t*)(res != nullptr ? res : x), (bf16_t*)out, res_c,
          res != nullptr ? 1.f : 0.f};
  if (xsums != nullptr) {
    bn.xsums = (const float*)xsums;
    bn.stat_w = (float*)stat;
    bn.running = (float*)running;
    bn.Mf = (float)M;
    bn.Mm1f = (float)(M - 1 > 1 ? M - 1 : 1);
    bn.eps = eps;
    bn.momentum = momentum;
  }
  // (BNIN 2: shortcut shaped like x or none; 3: option-A -- the block outputs whose block
  //  changed its width, at the two widths a CIFAR ResNet changes to)
#define X(ci, co, s) \
  if (Ci == ci && Co == co && stride == s && res_c == 0) \
    return launch_fwd<ci, co, kFwd, s, 0, 2>(x, w, y, sums, P, Bn, H, st, nullptr, 0, bn);
  X(16, 16, 1) X(16, 32, 2) X(32, 32, 1) X(32, 64, 2) X(64, 64, 1)
#undef X
#define X(c) \
  if (Ci == c && Co == c && stride == 1 && res_c > 0) \
    return launch_fwd<c, c, kFwd, 1, 0, 3>(x, w, y, sums, P, Bn, H, st, nullptr, 0, bn);
  X(32) X(64)
#undef X
  return (int)hipErrorNotSupported;
}

// Data gradient of a convolution (stride 1: identity shortcut addend shaped like dx; stride 2:
// option-A addend [P*Bn, H/2, H/2, addend_c] at the even pixels) whose input is a block output
// bn_y = relu(BatchNorm(bn_x) + shortcut): dz = (dgrad + addend) relu'(bn_y) is stored into dx
// and the BatchNorm backward's reductions (sum dz, sum dz xhat) are added into sums [P][2][Ci]
// (zeroed by the caller; stat [P][2][Ci] mean / rstd of that BatchNorm).  Ci == Co at stride 1,
// Co == 2 Ci at stride 2 (a CIFAR ResNet's block entries).
int mopt_dconv_dgrad_bnres(const void* dy, const void* w, void* dx, const void* addend,
                           void* sums, int P, int Bn, int H, int Ci, int Co, int stride,
                           int addend_c, const void* bn_x, const void* bn_y, const void* stat,
                           void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (addend == nullptr || sums == nullptr || bn_x == nullptr || bn_y == nullptr ||
      stat == nullptr || (stride == 2 && addend_c <= 0))
    return (int)hipErrorInvalidValue;
  const BnIn bn{(const float*)stat, nullptr, nullptr, (const bf16_t*)bn_x, (const bf16_t*)bn_y};
  // (the data gradient runs the forward kernel with the channel counts swapped: CI = Co)
#define X1(c) \
  if (stride == 1 && Ci == c && Co == c) \
    return launch_fwd<c, c, kDgrad, 1, 1, 0, 2>(dy, w, dx, sums, P, Bn, H, st, addend, 0, bn);
#define X2(co, ci) \
  if (stride == 2 && Co == co && Ci == ci) \
    return launch_fwd<co, ci, kDgrad2, 1, 2, 0, 2>(dy, w, dx, sums, P, Bn, H, st, addend, \
                                                   addend_c, bn);
  X1(16) X1(32) X1(64) X2(32, 16) X2(64, 32)
#undef X1
#undef X2
  return (int)hipErrorNotSupported;
}

// mopt_dconv kinds 0 (forward, with the output's batch sums) and 2 (weight gradient) of a
// convolution whose input is the SAME for every trial: x [Bn, H, H, Ci] (the stem over the shared
// minibatch -- no P-fold copy of the batch, and its reads are L2 hits after the first trials).
int mopt_dconv_shared_x(int kind, const void* a, const void* b, void* out, void* aux, int P,
                        int Bn, int H, int Ci, int Co, int stride, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (stride != 1) return (int)hipErrorNotSupported;
#define X(ci, co) \
  if (Ci == ci && Co == co) \
    return kind == 0 ? launch_fwd<ci, co, kFwd, 1>(a, b, out, aux, P, Bn, H, st, nullptr, 0, \
                                                   BnIn{}, 1) \
         : kind == 2 ? launch_wgrad<ci, co, 1>(a, b, out, aux, P, Bn, H, st, nullptr, BnIn{}, 1) \
                     : (int)hipErrorInvalidValue;
  X(8, 16) X(16, 16)
#undef X
  return (int)hipErrorNotSupported;
}

// number of partial slices the weight-gradient kernel writes (0 when unsupported)
int mopt_dconv_wgrad_splits(int P, int Bn, int H, int Ci, int Co, int stride) {
  int nb = 0;
#define X(ci, co) \
  if (Ci == ci && Co == co) \
    return (stride == 1 \
                ? launch_wgrad<ci, co, 1>(nullptr, nullptr, nullptr, nullptr, P, Bn, H, 0, &nb) \
                : launch_wgrad<ci, co, 2>(nullptr, nullptr, nullptr, nullptr, P, Bn, H, 0, &nb)) \
               ? 0 : nb;
  MOPT_DCONV_SHAPES(X)
#undef X
  return 0;
}

}  // extern "C"
