// Forward-mode hypergradient step through SGD-momentum (north-star kernel K11).
//
// Inner update with per-trial learning rate eta_p and momentum mu_p:
//     v' = mu v + g            w' = w - eta v'
// Tangents w.r.t. h = (eta, mu) are propagated alongside (Z = dw/dh, Y = dv/dh), given the
// Hessian-vector products H Z_eta, H Z_mu of the training loss at w (computed by the caller with
// one forward-over-reverse pass per direction):
//     Y_eta' = mu Y_eta + H Z_eta               Z_eta' = Z_eta - eta Y_eta' - v'
//     Y_mu'  = mu Y_mu  + H Z_mu + v            Z_mu'  = Z_mu  - eta Y_mu'
// After K steps dL_val/dh = <grad L_val(w_K), Z_h> (hyper_dot_kernel, per trial).
// All buffers are flat f32 [P][n]; one pass reads 9 and writes 6 streams (memory bound).
#include "common.h"

using namespace mopt;

namespace {

__global__ __launch_bounds__(256) void hyper_sgdm_kernel(float* __restrict__ w,
                                                         float* __restrict__ v,
                                                         float* __restrict__ ze,
                                                         float* __restrict__ zm,
                                                         float* __restrict__ ye,
                                                         float* __restrict__ ym,
                                                         const float* __restrict__ g,
                                                         const float* __restrict__ he,
                                                         const float* __restrict__ hm,
                                                         const float* __restrict__ eta,
                                                         const float* __restrict__ mu,
                                                         int64_t n, int64_t total) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= total) return;
  const int p = (int)(i / n);
  const float et = eta[p], m = mu[p];
  f32x4 W = *(f32x4*)(w + i), Vv = *(f32x4*)(v + i), ZE = *(f32x4*)(ze + i),
        ZM = *(f32x4*)(zm + i), YE = *(f32x4*)(ye + i), YM = *(f32x4*)(ym + i);
  const f32x4 G = *(const f32x4*)(g + i), HE = *(const f32x4*)(he + i),
              HM = *(const f32x4*)(hm + i);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float vn = m * Vv[e] + G[e];
    const float yen = m * YE[e] + HE[e];
    const float ymn = m * YM[e] + HM[e] + Vv[e];
    ZE[e] = ZE[e] - et * yen - vn;
    ZM[e] = ZM[e] - et * ymn;
    W[e] = W[e] - et * vn;
    Vv[e] = vn;
    YE[e] = yen;
    YM[e] = ymn;
  }
  *(f32x4*)(w + i) = W;
  *(f32x4*)(v + i) = Vv;
  *(f32x4*)(ze + i) = ZE;
  *(f32x4*)(zm + i) = ZM;
  *(f32x4*)(ye + i) = YE;
  *(f32x4*)(ym + i) = YM;
}

// out[p][0] = <a, b0>_p, out[p][1] = <a, b1>_p over trial p's n elements.  grid (chunks, P).
__global__ __launch_bounds__(256) void hyper_dot_kernel(const float* __restrict__ a,
                                                        const float* __restrict__ b0,
                                                        const float* __restrict__ b1,
                                                        float* __restrict__ out, int64_t n) {
  __shared__ float red[2][4];
  const int p = blockIdx.y;
  const int64_t base = (int64_t)p * n;
  float s0 = 0.f, s1 = 0.f;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n;
       i += (int64_t)gridDim.x * 256 * 4) {
    const f32x4 A = *(const f32x4*)(a + base + i), B0 = *(const f32x4*)(b0 + base + i),
                B1 = *(const f32x4*)(b1 + base + i);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s0 += A[e] * B0[e];
      s1 += A[e] * B1[e];
    }
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    red[0][wave] = s0;
    red[1][wave] = s1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(out + 2 * p, red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    atomicAdd(out + 2 * p + 1, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

}  // namespace

extern "C" {

int mopt_hyper_sgdm(void* w, void* v, void* ze, void* zm, void* ye, void* ym, const void* g,
                    const void* he, const void* hm, const void* eta, const void* mu, int64_t n,
                    int P, void* stream) {
  if (n % 4) return 1;
  const int64_t total = n * P;
  hipLaunchKernelGGL(hyper_sgdm_kernel, dim3((unsigned)((total / 4 + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (float*)w, (float*)v, (float*)ze, (float*)zm,
                     (float*)ye, (float*)ym, (const float*)g, (const float*)he, (const float*)hm,
                     (const float*)eta, (const float*)mu, n, total);
  return (int)hipGetLastError();
}

int mopt_hyper_dot(const void* a, const void* b0, const void* b1, void* out, int64_t n, int P,
                   void* stream) {
  if (n % 4) return 1;
  (void)hipMemsetAsync(out, 0, sizeof(float) * 2 * P, (hipStream_t)stream);
  // every block ends in two float atomics on its trial's pair: 1024 blocks per trial serialised
  // on those addresses (222 us for 3.7 M-element trials, 1.6 TB/s); 192 blocks per trial still
  // fill the chip at 8 trials and each thread keeps several 16-byte loads per stream in flight
#ifndef MOPT_HYDOT_CHUNKS
#define MOPT_HYDOT_CHUNKS 192
#endif
  const int chunks = (int)min((int64_t)MOPT_HYDOT_CHUNKS, (n / 4 + 255) / 256);
  hipLaunchKernelGGL(hyper_dot_kernel, dim3(chunks, P), dim3(256), 0, (hipStream_t)stream,
                     (const float*)a, (const float*)b0, (const float*)b1, (float*)out, n);
  return (int)hipGetLastError();
}

}  // extern "C"

// ==============================================================================================
// Stacked operators of the hand-derived forward-over-reverse step (models/hyper_step.py).
//
// Every activation is a STACK of S <= 3 slices stored [P][S * R][cols]: slice 0 the primal rows
// of trial p, slices 1.. the rows of its tangents (one per hyper-parameter).  Each kernel reads
// the primal slice once and produces every slice, so the tangent propagation costs no extra
// pass over the primal.  All f32.  Parameter pointers (a0..a2, E0..E2, G0..G2) address one
// parameter inside the flat [P][pstride] run state (weights, weight tangents, gradients).
// ==============================================================================================
namespace {

constexpr int kMaxS = 3;

struct Ptr3 {
  const float* p[kMaxS];
};
struct MPtr3 {
  float* p[kMaxS];
};

// ---------------------------------------------------------------------------- embedding
// out[p][s R + r][:] = E_s[p][tok[p][r]][:]           one wave per (p, r)
__global__ __launch_bounds__(64) void hy_embed_fwd_kernel(const int* __restrict__ tok,
                                                          int64_t tok_stride, Ptr3 E,
                                                          float* __restrict__ out, int P, int R,
                                                          int d, int V, int64_t pstride, int S) {
  const int row = blockIdx.x;  // p * R + r
  const int p = row / R, r = row - p * R;
  const int v = tok[(int64_t)p * tok_stride + r];
  if (!MOPT_IN_RANGE(v, V, "hyper embedding token id")) return;
  for (int s = 0; s < S; ++s) {
    const float* src = E.p[s] + (int64_t)p * pstride + (int64_t)v * d;
    float* dst = out + ((int64_t)p * S * R + (int64_t)s * R + r) * d;
    for (int c = 4 * threadIdx.x; c < d; c += 256) *(f32x4*)(dst + c) = *(const f32x4*)(src + c);
  }
}

// G_s[p][tok[p][r]][:] += GX[p][s R + r][:]           one wave per (p, r), f32 atomics
__global__ __launch_bounds__(64) void hy_embed_bwd_kernel(const int* __restrict__ tok,
                                                          int64_t tok_stride,
                                                          const float* __restrict__ GX, MPtr3 G,
                                                          int P, int R, int d, int V,
                                                          int64_t pstride, int S) {
  const int row = blockIdx.x;
  const int p = row / R, r = row - p * R;
  const int v = tok[(int64_t)p * tok_stride + r];
  if (!MOPT_IN_RANGE(v, V, "hyper embedding token id")) return;
  for (int s = 0; s < S; ++s) {
    const float* src = GX + ((int64_t)p * S * R + (int64_t)s * R + r) * d;
    float* dst = G.p[s] + (int64_t)p * pstride + (int64_t)v * d;
    for (int c = threadIdx.x; c < d; c += 64) atomicAdd(dst + c, src[c]);
  }
}

// ---------------------------------------------------------------------------- RMSNorm
// One wave per row; lane holds columns lane + 64 k, k < NK (d = 64 NK).
template <int NK>
__global__ __launch_bounds__(256) void hy_norm_fwd_kernel(const float* __restrict__ X, Ptr3 a,
                                                          float* __restrict__ Y,
                                                          float* __restrict__ rstd, int P, int R,
                                                          int S, int64_t pstride, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= P * R) return;
  const int p = row / R, r = row - p * R;
  constexpr int d = 64 * NK;
  const float* a0 = a.p[0] + (int64_t)p * pstride;
  const int64_t base = (int64_t)p * S * R * d;
  float n[NK], w0[NK];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    n[k] = X[base + (int64_t)r * d + lane + 64 * k];
    w0[k] = a0[lane + 64 * k];
    ss += n[k] * n[k];
  }
  const float rs = rsqrtf(wave_sum(ss) / d + eps);
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    n[k] *= rs;
    Y[base + (int64_t)r * d + lane + 64 * k] = n[k] * w0[k];
  }
  if (lane == 0) rstd[row] = rs;
  for (int t = 1; t < S; ++t) {
    const float* at = a.p[t] + (int64_t)p * pstride;
    const int64_t o = base + ((int64_t)t * R + r) * d;
    float xd[NK];
    float cx = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      xd[k] = X[o + lane + 64 * k];
      cx += n[k] * xd[k];
    }
    cx = wave_sum(cx) / d;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const float nd = rs * (xd[k] - n[k] * cx);
      Y[o + lane + 64 * k] = nd * w0[k] + n[k] * at[lane + 64 * k];
    }
  }
}

// Adjoint (and its tangents) of the RMSNorm stack; GX (+)= the input adjoints, the weight
// gradients G_s are summed over the block's rows in registers and LDS, then added atomically.
// Block: 4 waves x RPW rows of one trial.
constexpr int kNormRPW = 2;  // 8 rows per block: >= 2 blocks per CU at 4096 rows
template <int NK>
__global__ __launch_bounds__(256) void hy_norm_bwd_kernel(const float* __restrict__ X,
                                                          const float* __restrict__ GY, Ptr3 a,
                                                          const float* __restrict__ rstd,
                                                          float* __restrict__ GX, MPtr3 G, int P,
                                                          int R, int S, int64_t pstride,
                                                          int accumulate) {
  constexpr int d = 64 * NK;
  __shared__ float red[4][kMaxS][d];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int blocks_per_trial = (R + 4 * kNormRPW - 1) / (4 * kNormRPW);
  const int p = blockIdx.x / blocks_per_trial;
  const int r0 = (blockIdx.x - p * blocks_per_trial) * 4 * kNormRPW + wave * kNormRPW;
  const float* a0 = a.p[0] + (int64_t)p * pstride;
  const int64_t base = (int64_t)p * S * R * d;
  float w0[NK], gacc[kMaxS][NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    w0[k] = a0[lane + 64 * k];
#pragma unroll
    for (int s = 0; s < kMaxS; ++s) gacc[s][k] = 0.f;
  }
  for (int rr = 0; rr < kNormRPW; ++rr) {
    const int r = r0 + rr;
    if (r >= R) break;
    const float rs = rstd[(int64_t)p * R + r];
    float n[NK], gy[NK], gn[NK];
    float c = 0.f;
    const int64_t o0 = base + (int64_t)r * d;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      n[k] = X[o0 + lane + 64 * k] * rs;
      gy[k] = GY[o0 + lane + 64 * k];
      gn[k] = gy[k] * w0[k];
      c += n[k] * gn[k];
      gacc[0][k] += gy[k] * n[k];
    }
    c = wave_sum(c) / d;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const float gx = rs * (gn[k] - n[k] * c);
      float* dst = GX + o0 + lane + 64 * k;
      *dst = accumulate ? *dst + gx : gx;
    }
#pragma unroll
    for (int t = 1; t < kMaxS; ++t) {
      if (t >= S) break;
      const float* at = a.p[t] + (int64_t)p * pstride;
      const int64_t ot = base + ((int64_t)t * R + r) * d;
      float xd[NK], gyd[NK];
      float cx = 0.f;
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        xd[k] = X[ot + lane + 64 * k];
        gyd[k] = GY[ot + lane + 64 * k];
        cx += n[k] * xd[k];
      }
      cx = wave_sum(cx) / d;
      float nd[NK], gnd[NK];
      float cd = 0.f;
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        nd[k] = rs * (xd[k] - n[k] * cx);
        gnd[k] = gyd[k] * w0[k] + gy[k] * at[lane + 64 * k];
        cd += nd[k] * gn[k] + n[k] * gnd[k];
        gacc[t][k] += gyd[k] * n[k] + gy[k] * nd[k];
      }
      cd = wave_sum(cd) / d;
      const float rd = -rs * rs * cx;
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        const float g = rd * (gn[k] - n[k] * c) + rs * (gnd[k] - nd[k] * c - n[k] * cd);
        float* dst = GX + ot + lane + 64 * k;
        *dst = accumulate ? *dst + g : g;
      }
    }
  }
#pragma unroll
  for (int s = 0; s < kMaxS; ++s)
#pragma unroll
    for (int k = 0; k < NK; ++k) red[wave][s][lane + 64 * k] = gacc[s][k];
  __syncthreads();
  for (int i = threadIdx.x; i < S * d; i += 256) {
    const int s = i / d, col = i - s * d;
    const float v = red[0][s][col] + red[1][s][col] + red[2][s][col] + red[3][s][col];
    atomicAdd(G.p[s] + (int64_t)p * pstride + col, v);
  }
}

// ---------------------------------------------------------------------------- RoPE + heads
// dir 0: QKV [P][S R][3 d] (cols q | k | v, head-major) -> Qh/Kh/Vh [P B H][S T][64], q and k
//        rotated by (cos, sin);  dir 1: the adjoint (heads -> QKV, rotation by -sin).
// One thread per (p, s, b, i, which, h, j < 32) pair of rotated columns (j, j + 32).
__global__ __launch_bounds__(256) void hy_rope_kernel(float* __restrict__ QKV,
                                                      const float* __restrict__ cs,
                                                      const float* __restrict__ sn,
                                                      float* __restrict__ Qh,
                                                      float* __restrict__ Kh,
                                                      float* __restrict__ Vh, int P, int B,
                                                      int T, int H, int S, int dir) {
  const int64_t total = (int64_t)P * S * B * T * 3 * H * 32;
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (id >= total) return;
  int64_t q = id;
  const int j = (int)(q % 32); q /= 32;
  const int h = (int)(q % H); q /= H;
  const int which = (int)(q % 3); q /= 3;
  const int i = (int)(q % T); q /= T;
  const int b = (int)(q % B); q /= B;
  const int s = (int)(q % S);
  const int p = (int)(q / S);
  const int d = 64 * H, R = B * T;
  float* row = QKV + ((int64_t)p * S * R + (int64_t)s * R + (int64_t)b * T + i) * 3 * d +
               which * d + h * 64;
  float* hd = (which == 0 ? Qh : which == 1 ? Kh : Vh) +
              ((((int64_t)p * B + b) * H + h) * S * T + (int64_t)s * T + i) * 64;
  const float c = which < 2 ? cs[i * 32 + j] : 1.f;
  const float sg = which < 2 ? sn[i * 32 + j] : 0.f;
  if (dir == 0) {
    const float t1 = row[j], t2 = row[j + 32];
    hd[j] = t1 * c - t2 * sg;
    hd[j + 32] = t2 * c + t1 * sg;
  } else {
    const float t1 = hd[j], t2 = hd[j + 32];
    row[j] = t1 * c + t2 * sg;
    row[j + 32] = t2 * c - t1 * sg;
  }
}

// dir 1: Oh [P B H][S T][64] -> O [P][S R][H 64];  dir 0: the inverse permutation.
// One thread per 4 columns.
__global__ __launch_bounds__(256) void hy_heads_kernel(float* __restrict__ O,
                                                       float* __restrict__ Oh, int P, int B,
                                                       int T, int H, int S, int dir) {
  const int64_t total = (int64_t)P * S * B * T * H * 16;
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (id >= total) return;
  int64_t q = id;
  const int c4 = (int)(q % 16); q /= 16;
  const int h = (int)(q % H); q /= H;
  const int i = (int)(q % T); q /= T;
  const int b = (int)(q % B); q /= B;
  const int s = (int)(q % S);
  const int p = (int)(q / S);
  const int R = B * T;
  float* o = O + (((int64_t)p * S * R + (int64_t)s * R + (int64_t)b * T + i) * H + h) * 64 + 4 * c4;
  float* oh = Oh + ((((int64_t)p * B + b) * H + h) * S * T + (int64_t)s * T + i) * 64 + 4 * c4;
  if (dir == 1) *(f32x4*)o = *(const f32x4*)oh;
  else *(f32x4*)oh = *(const f32x4*)o;
}

// ---------------------------------------------------------------------------- causal softmax
// One wave per (n, query row i); lane holds keys lane + 64 k, k < TK (T = 64 TK).
// S1 [N][S T][T] = [q; q_1; ..] k0^T, S2 [N][T][(S-1) T] = q0 [k_1; ..]^T.
template <int TK>
__global__ __launch_bounds__(256) void hy_softmax_fwd_kernel(const float* __restrict__ S1,
                                                             const float* __restrict__ S2,
                                                             float* __restrict__ Pm, int N,
                                                             int S, float scale) {
  constexpr int T = 64 * TK;
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wid >= N * T) return;
  const int n = wid / T, i = wid - n * T;
  const float* s1 = S1 + (int64_t)n * S * T * T;
  float* pm = Pm + (int64_t)n * S * T * T;
  float pr[TK];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < TK; ++k) {
    const int j = lane + 64 * k;
    pr[k] = j <= i ? scale * s1[(int64_t)i * T + j] : -INFINITY;
    mx = fmaxf(mx, pr[k]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  float l = 0.f;
#pragma unroll
  for (int k = 0; k < TK; ++k) {
    pr[k] = lane + 64 * k <= i ? __expf(pr[k] - mx) : 0.f;
    l += pr[k];
  }
  const float inv = 1.f / wave_sum(l);
#pragma unroll
  for (int k = 0; k < TK; ++k) {
    pr[k] *= inv;
    pm[(int64_t)i * T + lane + 64 * k] = pr[k];
  }
  for (int t = 1; t < S; ++t) {
    float sd[TK];
    float m = 0.f;
#pragma unroll
    for (int k = 0; k < TK; ++k) {
      const int j = lane + 64 * k;
      sd[k] = j <= i ? scale * (s1[((int64_t)t * T + i) * T + j] +
                                S2[((int64_t)n * T + i) * (S - 1) * T + (t - 1) * T + j])
                     : 0.f;
      m += pr[k] * sd[k];
    }
    m = wave_sum(m);
#pragma unroll
    for (int k = 0; k < TK; ++k)
      pm[((int64_t)t * T + i) * T + lane + 64 * k] = pr[k] * (sd[k] - m);
  }
}

// Score adjoints GS = scale * [P (gP - D); Ṗ_t (gP - D) + P (ġP_t - Ḋ_t)], D = <go, o>,
// Ḋ_t = <ġo_t, o> + <go, ȯ_t>;  GP1 [N][S T][T] = GO v0^T, GP2 [N][T][(S-1) T] = go0 v_t^T.
template <int TK>
__global__ __launch_bounds__(256) void hy_softmax_bwd_kernel(
    const float* __restrict__ Pm, const float* __restrict__ GP1, const float* __restrict__ GP2,
    const float* __restrict__ Oh, const float* __restrict__ GOh, float* __restrict__ GS, int N,
    int S, float scale) {
  constexpr int T = 64 * TK;
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wid >= N * T) return;
  const int n = wid / T, i = wid - n * T;
  const int64_t mt = (int64_t)n * S * T * T;   // [S T][T] matrices of head n
  const int64_t vt = (int64_t)n * S * T * 64;  // [S T][64] matrices of head n
  const float o0 = Oh[vt + (int64_t)i * 64 + lane];
  const float go0 = GOh[vt + (int64_t)i * 64 + lane];
  const float D = wave_sum(o0 * go0);
  float p[TK], gpd[TK];
#pragma unroll
  for (int k = 0; k < TK; ++k) {
    const int64_t e = (int64_t)i * T + lane + 64 * k;
    p[k] = Pm[mt + e];
    gpd[k] = GP1[mt + e] - D;
    GS[mt + e] = scale * p[k] * gpd[k];
  }
  for (int t = 1; t < S; ++t) {
    const int64_t rt = (int64_t)t * T + i;
    const float Dd = wave_sum(GOh[vt + rt * 64 + lane] * o0 + go0 * Oh[vt + rt * 64 + lane]);
#pragma unroll
    for (int k = 0; k < TK; ++k) {
      const int j = lane + 64 * k;
      const float gP = GP1[mt + rt * T + j] + GP2[((int64_t)n * T + i) * (S - 1) * T +
                                                  (t - 1) * T + j];
      GS[mt + rt * T + j] = scale * (Pm[mt + rt * T + j] * gpd[k] + p[k] * (gP - Dd));
    }
  }
}

// ---------------------------------------------------------------------------- SwiGLU
// GGU == nullptr: forward A = silu(g) u (+ tangents); else backward GGU from GA.
// One thread per (p, r, f).
__global__ __launch_bounds__(256) void hy_swiglu_kernel(const float* __restrict__ GU,
                                                        const float* __restrict__ A_or_GA,
                                                        float* __restrict__ GGU,
                                                        float* __restrict__ A, int P, int R,
                                                        int F, int S) {
  const int64_t total = (int64_t)P * R * F;
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (id >= total) return;
  const int f = (int)(id % F);
  const int64_t pr = id / F;
  const int r = (int)(pr % R);
  const int p = (int)(pr / R);
  const int64_t row0 = (int64_t)p * S * R + r;  // row of slice 0
  const float g = GU[row0 * 2 * F + f], u = GU[row0 * 2 * F + F + f];
  const float sg = 1.f / (1.f + __expf(-g));
  const float f0 = g * sg, d1 = sg * (1.f + g * (1.f - sg));
  if (GGU == nullptr) {
    A[row0 * F + f] = f0 * u;
    for (int t = 1; t < S; ++t) {
      const int64_t rt = row0 + (int64_t)t * R;
      A[rt * F + f] = d1 * GU[rt * 2 * F + f] * u + f0 * GU[rt * 2 * F + F + f];
    }
    return;
  }
  const float d2 = sg * (1.f - sg) * (2.f + g * (1.f - 2.f * sg));
  const float ga = A_or_GA[row0 * F + f];
  GGU[row0 * 2 * F + f] = ga * u * d1;
  GGU[row0 * 2 * F + F + f] = ga * f0;
  for (int t = 1; t < S; ++t) {
    const int64_t rt = row0 + (int64_t)t * R;
    const float gd = GU[rt * 2 * F + f], ud = GU[rt * 2 * F + F + f], gad = A_or_GA[rt * F + f];
    GGU[rt * 2 * F + f] = (gad * u + ga * ud) * d1 + ga * u * d2 * gd;
    GGU[rt * 2 * F + F + f] = gad * f0 + ga * d1 * gd;
  }
}

// ---------------------------------------------------------------------------- cross-entropy
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

__device__ __forceinline__ float block_max(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// In place over the logits stack Z [P][S R][V]: slice 0 -> (pi - onehot) / R, slice t ->
// pi (z_t - <pi, z_t>) / R; losses[p] += nll / R.  One workgroup per (p, r); the primal row is
// read from HBM once and kept in LDS (V floats of dynamic shared memory) for every later pass.
__global__ __launch_bounds__(256) void hy_ce_kernel(float* __restrict__ Z,
                                                    const int* __restrict__ tgt,
                                                    int64_t tgt_stride,
                                                    float* __restrict__ losses, int P, int R,
                                                    int V, int S) {
  extern __shared__ float zrow[];
  __shared__ float red[4];
  const int row = blockIdx.x;
  const int p = row / R, r = row - p * R;
  float* z = Z + ((int64_t)p * S * R + r) * V;
  const int y = tgt[(int64_t)p * tgt_stride + r];
  float mx = -INFINITY;
  for (int c = 4 * threadIdx.x; c < V; c += 1024) {
    const f32x4 v = *(const f32x4*)(z + c);
    *(f32x4*)(zrow + c) = v;
    mx = fmaxf(fmaxf(mx, fmaxf(v[0], v[1])), fmaxf(v[2], v[3]));
  }
  mx = block_max(mx, red);  // (its barriers also publish zrow)
  float se = 0.f;
  for (int c = 4 * threadIdx.x; c < V; c += 1024) {
    f32x4 v = *(const f32x4*)(zrow + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = __expf(v[e] - mx);
      se += v[e];
    }
    *(f32x4*)(zrow + c) = v;  // unnormalised softmax, own chunk
  }
  const float sum = block_sum(se, red);
  const float lse = mx + __logf(sum), inv = 1.f / sum;
  const float invR = 1.f / R;
  const bool ok = MOPT_IN_RANGE(y, V, "hyper target id");
  if (threadIdx.x == 0 && ok) atomicAdd(losses + p, (lse - z[y]) * invR);
  for (int t = 1; t < S; ++t) {
    float* zt = z + (int64_t)t * R * V;
    float m = 0.f;
    for (int c = 4 * threadIdx.x; c < V; c += 1024) {
      const f32x4 e = *(const f32x4*)(zrow + c), w = *(const f32x4*)(zt + c);
      m += e[0] * w[0] + e[1] * w[1] + e[2] * w[2] + e[3] * w[3];
    }
    m = block_sum(m, red) * inv;
    for (int c = 4 * threadIdx.x; c < V; c += 1024) {
      const f32x4 e = *(const f32x4*)(zrow + c);
      f32x4 w = *(const f32x4*)(zt + c);
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = e[k] * inv * (w[k] - m) * invR;
      *(f32x4*)(zt + c) = w;
    }
  }
  __syncthreads();  // the read of z[y] above is done before the row is overwritten
  for (int c = 4 * threadIdx.x; c < V; c += 1024) {
    f32x4 v = *(const f32x4*)(zrow + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (v[e] * inv - (c + e == y ? 1.f : 0.f)) * invR;
    *(f32x4*)(z + c) = v;
  }
}

// ---------------------------------------------------------------------------- zero segments
constexpr int kMaxSegs = 32;
struct Segs {
  int64_t off[kMaxSegs], len[kMaxSegs];
  int n;
};

__global__ __launch_bounds__(256) void hy_zero_kernel(MPtr3 bufs, int nbuf, int64_t pstride,
                                                      Segs segs) {
  const int sp = blockIdx.y;  // (buffer, segment, trial)
  const int seg = sp % segs.n;
  const int rest = sp / segs.n;
  const int b = rest % nbuf;
  const int p = rest / nbuf;
  float* dst = bufs.p[b] + (int64_t)p * pstride + segs.off[seg];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < segs.len[seg];
       i += (int64_t)gridDim.x * 256)
    dst[i] = 0.f;
}

template <typename K1, typename K2, typename K4, typename K8>
int pick_nk(int nk, K1 k1, K2 k2, K4 k4, K8 k8) {
  switch (nk) {
    case 1: k1(); return 0;
    case 2: k2(); return 0;
    case 4: k4(); return 0;
    case 8: k8(); return 0;
    default: return (int)hipErrorInvalidValue;
  }
}

int nslices(const void* p1, const void* p2) { return 1 + (p1 != nullptr) + (p2 != nullptr); }

}  // namespace

extern "C" {

int mopt_hy_embed_fwd(const void* tok, int64_t tok_stride, const void* E0, const void* E1,
                      const void* E2, void* out, int P, int R, int d, int V, int64_t pstride,
                      void* stream) {
  if (d % 4) return (int)hipErrorInvalidValue;
  Ptr3 E{{(const float*)E0, (const float*)E1, (const float*)E2}};
  hipLaunchKernelGGL(hy_embed_fwd_kernel, dim3(P * R), dim3(64), 0, (hipStream_t)stream,
                     (const int*)tok, tok_stride, E, (float*)out, P, R, d, V, pstride,
                     nslices(E1, E2));
  return (int)hipGetLastError();
}

int mopt_hy_embed_bwd(const void* tok, int64_t tok_stride, const void* GX, void* G0, void* G1,
                      void* G2, int P, int R, int d, int V, int64_t pstride, void* stream) {
  MPtr3 G{{(float*)G0, (float*)G1, (float*)G2}};
  hipLaunchKernelGGL(hy_embed_bwd_kernel, dim3(P * R), dim3(64), 0, (hipStream_t)stream,
                     (const int*)tok, tok_stride, (const float*)GX, G, P, R, d, V, pstride,
                     nslices(G1, G2));
  return (int)hipGetLastError();
}

int mopt_hy_norm_fwd(const void* X, const void* a0, const void* a1, const void* a2, void* Y,
                     void* rstd, int P, int R, int d, int S, int64_t pstride, float eps,
                     void* stream) {
  if (d % 64 || S != nslices(a1, a2)) return (int)hipErrorInvalidValue;
  Ptr3 a{{(const float*)a0, (const float*)a1, (const float*)a2}};
  const dim3 grid((P * R + 3) / 4);
  hipStream_t st = (hipStream_t)stream;
#define HY_NF(NK)                                                                       \
  [&] {                                                                                 \
    hipLaunchKernelGGL(hy_norm_fwd_kernel<NK>, grid, dim3(256), 0, st, (const float*)X, a, \
                       (float*)Y, (float*)rstd, P, R, S, pstride, eps);                 \
  }
  const int e = pick_nk(d / 64, HY_NF(1), HY_NF(2), HY_NF(4), HY_NF(8));
#undef HY_NF
  return e ? e : (int)hipGetLastError();
}

int mopt_hy_norm_bwd(const void* X, const void* GY, const void* a0, const void* a1,
                     const void* a2, const void* rstd, void* GX, void* G0, void* G1, void* G2,
                     int P, int R, int d, int S, int64_t pstride, int accumulate, void* stream) {
  if (d % 64 || S != nslices(a1, a2) || S != nslices(G1, G2)) return (int)hipErrorInvalidValue;
  Ptr3 a{{(const float*)a0, (const float*)a1, (const float*)a2}};
  MPtr3 G{{(float*)G0, (float*)G1, (float*)G2}};
  const int bpt = (R + 4 * kNormRPW - 1) / (4 * kNormRPW);
  const dim3 grid(P * bpt);
  hipStream_t st = (hipStream_t)stream;
#define HY_NB(NK)                                                                          \
  [&] {                                                                                    \
    hipLaunchKernelGGL(hy_norm_bwd_kernel<NK>, grid, dim3(256), 0, st, (const float*)X,    \
                       (const float*)GY, a, (const float*)rstd, (float*)GX, G, P, R, S,     \
                       pstride, accumulate);                                               \
  }
  const int e = pick_nk(d / 64, HY_NB(1), HY_NB(2), HY_NB(4), HY_NB(8));
#undef HY_NB
  return e ? e : (int)hipGetLastError();
}

int mopt_hy_rope(void* QKV, const void* cs, const void* sn, void* Qh, void* Kh, void* Vh, int P,
                 int B, int T, int H, int S, int dir, void* stream) {
  const int64_t total = (int64_t)P * S * B * T * 3 * H * 32;
  hipLaunchKernelGGL(hy_rope_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (float*)QKV, (const float*)cs, (const float*)sn,
                     (float*)Qh, (float*)Kh, (float*)Vh, P, B, T, H, S, dir);
  return (int)hipGetLastError();
}

int mopt_hy_heads(void* O, void* Oh, int P, int B, int T, int H, int S, int dir, void* stream) {
  const int64_t total = (int64_t)P * S * B * T * H * 16;
  hipLaunchKernelGGL(hy_heads_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (float*)O, (float*)Oh, P, B, T, H, S, dir);
  return (int)hipGetLastError();
}

int mopt_hy_softmax_fwd(const void* S1, const void* S2, void* Pm, int N, int T, int S,
                        float scale, void* stream) {
  if (T % 64 || (S > 1 && S2 == nullptr)) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)(((int64_t)N * T + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
#define HY_SF(TK)                                                                        \
  [&] {                                                                                  \
    hipLaunchKernelGGL(hy_softmax_fwd_kernel<TK>, grid, dim3(256), 0, st, (const float*)S1, \
                       (const float*)S2, (float*)Pm, N, S, scale);                       \
  }
  const int e = pick_nk(T / 64, HY_SF(1), HY_SF(2), HY_SF(4), HY_SF(8));
#undef HY_SF
  return e ? e : (int)hipGetLastError();
}

int mopt_hy_softmax_bwd(const void* Pm, const void* GP1, const void* GP2, const void* Oh,
                        const void* GOh, void* GS, int N, int T, int S, float scale,
                        void* stream) {
  if (T % 64 || (S > 1 && GP2 == nullptr)) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)(((int64_t)N * T + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
#define HY_SB(TK)                                                                          \
  [&] {                                                                                    \
    hipLaunchKernelGGL(hy_softmax_bwd_kernel<TK>, grid, dim3(256), 0, st, (const float*)Pm, \
                       (const float*)GP1, (const float*)GP2, (const float*)Oh,              \
                       (const float*)GOh, (float*)GS, N, S, scale);                        \
  }
  const int e = pick_nk(T / 64, HY_SB(1), HY_SB(2), HY_SB(4), HY_SB(8));
#undef HY_SB
  return e ? e : (int)hipGetLastError();
}

// GGU == nullptr: A_or_GA is the output A of the forward; else the adjoint GA (backward).
int mopt_hy_swiglu(const void* GU, void* A_or_GA, void* GGU, int P, int R, int F, int S,
                   void* stream) {
  const int64_t total = (int64_t)P * R * F;
  hipLaunchKernelGGL(hy_swiglu_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const float*)GU, (const float*)A_or_GA, (float*)GGU,
                     (float*)A_or_GA, P, R, F, S);
  return (int)hipGetLastError();
}

int mopt_hy_ce(void* Z, const void* tgt, int64_t tgt_stride, void* losses, int P, int R, int V,
               int S, void* stream) {
  if (V % 4 || V > 16384) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  (void)hipMemsetAsync(losses, 0, sizeof(float) * P, st);
  hipLaunchKernelGGL(hy_ce_kernel, dim3(P * R), dim3(256), sizeof(float) * V, st, (float*)Z,
                     (const int*)tgt,
                     tgt_stride, (float*)losses, P, R, V, S);
  return (int)hipGetLastError();
}

// zero the segments [off, off + len) of every trial of up to 3 flat [P][pstride] buffers;
// off / len are HOST arrays (copied into the kernel arguments)
int mopt_hy_zero(void* b0, void* b1, void* b2, int P, int64_t pstride, const int64_t* off,
                 const int64_t* len, int nseg, void* stream) {
  if (nseg <= 0) return 0;
  if (nseg > kMaxSegs) return (int)hipErrorInvalidValue;
  MPtr3 bufs{{(float*)b0, (float*)b1, (float*)b2}};
  const int nbuf = nslices(b1, b2);
  Segs s{};
  int64_t mx = 0;
  for (int i = 0; i < nseg; ++i) {
    s.off[i] = off[i];
    s.len[i] = len[i];
    mx = len[i] > mx ? len[i] : mx;
  }
  s.n = nseg;
  const unsigned gx = (unsigned)((mx + 255) / 256 < 64 ? (mx + 255) / 256 : 64);
  hipLaunchKernelGGL(hy_zero_kernel, dim3(gx, nseg * nbuf * P), dim3(256), 0,
                     (hipStream_t)stream, bufs, nbuf, pstride, s);
  return (int)hipGetLastError();
}

}  // extern "C"
