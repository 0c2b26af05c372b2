// Elementwise / normalisation / loss / optimizer kernels of the population LM (north-star
// kernels K4, K6, K9).  Every tensor carries a leading population dimension: rows of trial p are
// rows [p * rows_per_trial, (p + 1) * rows_per_trial) and per-trial parameters are indexed by p.
//
//   rmsnorm_fwd / rmsnorm_bwd_dx / rmsnorm_bwd_dw   y = x * rsqrt(mean(x^2) + eps) * w[p]
//   rope_fwd / rope_bwd       split qkv [rows][3 H 64] into head-major Q/K/V [B'][H][T][64] with
//                             rotate-half RoPE on q and k (and the inverse for the gradients)
//   swiglu_fwd / swiglu_bwd   h = silu(gate) * up on a fused [rows][2F] projection
//   ce_fwd_bwd                row softmax cross-entropy over the vocabulary, dlogits in place
//   embed_fwd / embed_bwd     token gather / f32 atomic scatter-add into the per-trial table
//   grad_sumsq / adamw_multi  per-trial global grad norm (clipping) and the fused AdamW update
//                             over the flat parameter buffers, per-trial lr / betas / wd / step
#include "common.h"

using namespace mopt;

extern "C" {

struct LmHP {          // per-trial optimizer hyper-parameters, 32 bytes (mirrored in lm.py)
  float lr, b1, b2, eps, wd, max_norm;
  int32_t t, pad;
};

struct Segment {       // one parameter tensor of the flat buffers: [P][numel] at offset off
  int64_t off;
  int64_t numel;       // per trial, multiple of 8
};

struct SegChunk {      // <= 2048 elements of ONE trial inside a segment
  int32_t seg, trial;
  int64_t start;       // element offset inside the segment ([P * numel])
};

}  // extern "C"

namespace {

constexpr int kAdamChunk = 2048;

__device__ __forceinline__ void unpack8(const uint4& u, float (&f)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[2 * e] = bf2f(w[e] & 0xFFFF);
    f[2 * e + 1] = bf2f(w[e] >> 16);
  }
}

__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]),
                    pack2bf(f[6], f[7]));
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float s = 0.f;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
  return s;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------------------------- RMSNorm
constexpr int kMaxChunks = 4;  // d <= 64 lanes * 8 * 4 = 2048

// One wave per row, 4 rows per workgroup.  RES: the pre-norm residual add is fused in --
// xs = x + res (rounded to bf16, as the unfused add would) is written out as the new residual
// stream and normalised, so the transformer block's residual add costs no pass of its own.
template <bool RES>
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(const bf16_t* __restrict__ x,
                                                          const bf16_t* __restrict__ res,
                                                          bf16_t* __restrict__ xs,
                                                          const bf16_t* __restrict__ w,
                                                          bf16_t* __restrict__ y,
                                                          float* __restrict__ rstd, int rows,
                                                          int d, int rows_per_trial, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int p = row / rows_per_trial, nc = d >> 3;
  const bf16_t* xr = x + (size_t)row * d;
  float v[kMaxChunks][8];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxChunks; ++k) {
    const int c = lane + 64 * k;
    if (c < nc) {
      unpack8(*(const uint4*)(xr + 8 * c), v[k]);
      if (RES) {
        float rv[8];
        unpack8(*(const uint4*)(res + (size_t)row * d + 8 * c), rv);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[k][e] = bf2f(f2bf(v[k][e] + rv[e]));
        *(uint4*)(xs + (size_t)row * d + 8 * c) = pack8(v[k]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += v[k][e] * v[k][e];
    }
  }
  const float r = rsqrtf(wave_sum(ss) / d + eps);
  const bf16_t* wr = w + (size_t)p * d;
#pragma unroll
  for (int k = 0; k < kMaxChunks; ++k) {
    const int c = lane + 64 * k;
    if (c < nc) {
      float wv[8], o[8];
      unpack8(*(const uint4*)(wr + 8 * c), wv);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = v[k][e] * r * wv[e];
      *(uint4*)(y + (size_t)row * d + 8 * c) = pack8(o);
    }
  }
  if (lane == 0) rstd[row] = r;
}

// dx = r * (g - xhat * mean(g * xhat)) (+ dres),  g = dy * w,  xhat = x * r.  RES: the
// gradient reaching the residual stream directly is added in the same pass (the fused
// add + norm's backward: both summands of the residual get this dx).
template <bool RES>
__global__ __launch_bounds__(256) void rmsnorm_bwd_dx_kernel(const bf16_t* __restrict__ x,
                                                             const bf16_t* __restrict__ w,
                                                             const bf16_t* __restrict__ dy,
                                                             const bf16_t* __restrict__ dres,
                                                             const float* __restrict__ rstd,
                                                             bf16_t* __restrict__ dx, int rows,
                                                             int d, int rows_per_trial) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int p = row / rows_per_trial, nc = d >> 3;
  const float r = rstd[row];
  float xh[kMaxChunks][8], gv[kMaxChunks][8];
  float dot = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxChunks; ++k) {
    const int c = lane + 64 * k;
    if (c < nc) {
      float wv[8], dv[8];
      unpack8(*(const uint4*)(x + (size_t)row * d + 8 * c), xh[k]);
      unpack8(*(const uint4*)(w + (size_t)p * d + 8 * c), wv);
      unpack8(*(const uint4*)(dy + (size_t)row * d + 8 * c), dv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xh[k][e] *= r;
        gv[k][e] = dv[e] * wv[e];
        dot += gv[k][e] * xh[k][e];
      }
    }
  }
  const float mdot = wave_sum(dot) / d;
#pragma unroll
  for (int k = 0; k < kMaxChunks; ++k) {
    const int c = lane + 64 * k;
    if (c < nc) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = r * (gv[k][e] - xh[k][e] * mdot);
      if (RES) {
        float rv[8];
        unpack8(*(const uint4*)(dres + (size_t)row * d + 8 * c), rv);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += rv[e];
      }
      *(uint4*)(dx + (size_t)row * d + 8 * c) = pack8(o);
    }
  }
}

// The same backward with the weight gradient's partial sums fused in: workgroup (s, p) takes
// split s of trial p's rows (the slices of rmsnorm_dw_partial_kernel), its 4 waves a row each in
// turn, every lane summing dy * xhat of its columns across the rows; the 4 waves' sums meet in
// LDS and one f32 partial per (trial, split, column) is stored in rmsnorm_dw_partial_kernel's
// layout for rmsnorm_dw_reduce_kernel -- the partial kernel's second read of x and dy (a full
// pass over two activations per norm) goes.  NCH: 8-column chunks per lane (d <= 512 NCH).
template <bool RES, int NCH>
__global__ __launch_bounds__(256) void rmsnorm_bwd_dxdw_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ w, const bf16_t* __restrict__ dy,
    const bf16_t* __restrict__ dres, const float* __restrict__ rstd, bf16_t* __restrict__ dx,
    float* __restrict__ part, int d, int rows_per_trial, int S) {
  extern __shared__ __attribute__((aligned(16))) float red[];   // [4][d]
  const int s = blockIdx.x, p = blockIdx.y, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nc = d >> 3, G = nc;
  const int per = (rows_per_trial + S - 1) / S;
  const int r0 = p * rows_per_trial + s * per;
  const int r1 = min(r0 + per, (p + 1) * rows_per_trial);
  float wv[NCH][8], acc[NCH][8];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = lane + 64 * k;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[k][e] = 0.f;
    if (c < nc) unpack8(*(const uint4*)(w + (size_t)p * d + 8 * c), wv[k]);
  }
  for (int row = r0 + wave; row < r1; row += 4) {
    const float r = rstd[row];
    float xh[NCH][8], gv[NCH][8];
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = lane + 64 * k;
      if (c < nc) {
        float dv[8];
        unpack8(*(const uint4*)(x + (size_t)row * d + 8 * c), xh[k]);
        unpack8(*(const uint4*)(dy + (size_t)row * d + 8 * c), dv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          xh[k][e] *= r;
          acc[k][e] += dv[e] * xh[k][e];
          gv[k][e] = dv[e] * wv[k][e];
          dot += gv[k][e] * xh[k][e];
        }
      }
    }
    const float mdot = wave_sum(dot) / d;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = lane + 64 * k;
      if (c < nc) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = r * (gv[k][e] - xh[k][e] * mdot);
        if (RES) {
          float rv[8];
          unpack8(*(const uint4*)(dres + (size_t)row * d + 8 * c), rv);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] += rv[e];
        }
        *(uint4*)(dx + (size_t)row * d + 8 * c) = pack8(o);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = lane + 64 * k;
    if (c < nc) {
      *(f32x4*)(red + wave * d + 8 * c) = f32x4{acc[k][0], acc[k][1], acc[k][2], acc[k][3]};
      *(f32x4*)(red + wave * d + 8 * c + 4) = f32x4{acc[k][4], acc[k][5], acc[k][6], acc[k][7]};
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < d; i += 256) {
    const float v = (red[i] + red[d + i]) + (red[2 * d + i] + red[3 * d + i]);
    part[(((size_t)p * G + i / 8) * S + s) * 8 + i % 8] = v;
  }
}

// dw[p][col] += sum over a slice of trial p's rows of dy * x * rstd.  grid (d/256, splits, P).
__global__ __launch_bounds__(256) void rmsnorm_bwd_dw_kernel(const bf16_t* __restrict__ x,
                                                             const bf16_t* __restrict__ dy,
                                                             const float* __restrict__ rstd,
                                                             float* __restrict__ dw32, int d,
                                                             int rows_per_trial) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= d) return;
  const int p = blockIdx.z, splits = gridDim.y;
  const int per = (rows_per_trial + splits - 1) / splits;
  const int r0 = p * rows_per_trial + blockIdx.y * per;
  const int r1 = min(r0 + per, (p + 1) * rows_per_trial);
  float acc = 0.f;
  for (int r = r0; r < r1; ++r)
    acc += bf2f(dy[(size_t)r * d + col]) * bf2f(x[(size_t)r * d + col]) * rstd[r];
  atomicAdd(dw32 + (size_t)p * d + col, acc);
}

// ---------------------------------------------------------------------------------- RoPE
// qkv [B' * T][3][H][64] -> Q/K/V [B'][H][T][64]; thread = (row, part, head, 8-pair chunk).
// 4 interleaved RoPE pairs (x[2j], x[2j+1]) rotated by angle j (cs / sn: the 4 angles' tables),
// sign -1: the inverse (transposed) rotation of the backward
__device__ __forceinline__ void rope_pairs8(const float (&x)[8], const float* cs, const float* sn,
                                            float sign, float (&o)[8]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float c = cs[j], s = sign * sn[j];
    o[2 * j] = x[2 * j] * c - x[2 * j + 1] * s;
    o[2 * j + 1] = x[2 * j + 1] * c + x[2 * j] * s;
  }
}

__global__ __launch_bounds__(256) void rope_fwd_kernel(const bf16_t* __restrict__ qkv,
                                                       const float* __restrict__ cosv,
                                                       const float* __restrict__ sinv,
                                                       bf16_t* __restrict__ Q,
                                                       bf16_t* __restrict__ K,
                                                       bf16_t* __restrict__ V, int rows, int T,
                                                       int H, int il) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)rows * 3 * H * 4;
  if (i >= total) return;
  const int chunk = i & 3;
  const int64_t rest = i >> 2;
  const int hh = rest % H, part = (rest / H) % 3;
  const int64_t row = rest / (3 * H);
  const int t = row % T;
  const int64_t b = row / T;
  const bf16_t* src = qkv + ((row * 3 + part) * H + hh) * 64 + 8 * chunk;
  bf16_t* dst = (part == 0 ? Q : part == 1 ? K : V) + ((b * H + hh) * T + t) * 64 + 8 * chunk;
  const uint4 a = *(const uint4*)src, bb = *(const uint4*)(src + 32);
  if (part == 2) {
    *(uint4*)dst = a;
    *(uint4*)(dst + 32) = bb;
    return;
  }
  float x1[8], x2[8], o1[8], o2[8];
  unpack8(a, x1);
  unpack8(bb, x2);
  if (il) {   // interleaved pairs (2j, 2j + 1), angle j: elements 8 chunk .. and 32 + 8 chunk ..
    rope_pairs8(x1, cosv + (size_t)t * 32 + 4 * chunk, sinv + (size_t)t * 32 + 4 * chunk, 1.f, o1);
    rope_pairs8(x2, cosv + (size_t)t * 32 + 16 + 4 * chunk, sinv + (size_t)t * 32 + 16 + 4 * chunk,
                1.f, o2);
  } else {    // rotate-half pairs (j, j + 32)
    const float* cs = cosv + (size_t)t * 32 + 8 * chunk;
    const float* sn = sinv + (size_t)t * 32 + 8 * chunk;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o1[e] = x1[e] * cs[e] - x2[e] * sn[e];
      o2[e] = x2[e] * cs[e] + x1[e] * sn[e];
    }
  }
  *(uint4*)dst = pack8(o1);
  *(uint4*)(dst + 32) = pack8(o2);
}

__global__ __launch_bounds__(256) void rope_bwd_kernel(const bf16_t* __restrict__ dQ,
                                                       const bf16_t* __restrict__ dK,
                                                       const bf16_t* __restrict__ dV,
                                                       const float* __restrict__ cosv,
                                                       const float* __restrict__ sinv,
                                                       bf16_t* __restrict__ dqkv, int rows, int T,
                                                       int H, int il) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)rows * 3 * H * 4;
  if (i >= total) return;
  const int chunk = i & 3;
  const int64_t rest = i >> 2;
  const int hh = rest % H, part = (rest / H) % 3;
  const int64_t row = rest / (3 * H);
  const int t = row % T;
  const int64_t b = row / T;
  const bf16_t* src = (part == 0 ? dQ : part == 1 ? dK : dV) + ((b * H + hh) * T + t) * 64 + 8 * chunk;
  bf16_t* dst = dqkv + ((row * 3 + part) * H + hh) * 64 + 8 * chunk;
  const uint4 a = *(const uint4*)src, bb = *(const uint4*)(src + 32);
  if (part == 2) {
    *(uint4*)dst = a;
    *(uint4*)(dst + 32) = bb;
    return;
  }
  float y1[8], y2[8], o1[8], o2[8];
  unpack8(a, y1);
  unpack8(bb, y2);
  if (il) {   // the transposed rotation: the angle negated
    rope_pairs8(y1, cosv + (size_t)t * 32 + 4 * chunk, sinv + (size_t)t * 32 + 4 * chunk, -1.f, o1);
    rope_pairs8(y2, cosv + (size_t)t * 32 + 16 + 4 * chunk, sinv + (size_t)t * 32 + 16 + 4 * chunk,
                -1.f, o2);
  } else {
    const float* cs = cosv + (size_t)t * 32 + 8 * chunk;
    const float* sn = sinv + (size_t)t * 32 + 8 * chunk;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o1[e] = y1[e] * cs[e] + y2[e] * sn[e];
      o2[e] = y2[e] * cs[e] - y1[e] * sn[e];
    }
  }
  *(uint4*)dst = pack8(o1);
  *(uint4*)(dst + 32) = pack8(o2);
}

// ---------------------------------------------------------------------------------- SwiGLU
// gate / up columns of activation column c: halves [g | u] (il = 0), or interleaved 16-column
// groups [g0..g15 u0..u15 g16..] (il = 1: the layout the gate/up GEMM's SwiGLU epilogue writes,
// csrc/pgemm.hip EPI 1 / 2); c a multiple of 8
__device__ __forceinline__ int64_t gate_col(int c, int F, int il) {
  return il ? 32 * (c >> 4) + (c & 15) : c;
}
__device__ __forceinline__ int64_t up_col(int c, int F, int il) {
  return il ? 32 * (c >> 4) + 16 + (c & 15) : F + c;
}

__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16_t* __restrict__ gu,
                                                         bf16_t* __restrict__ h, int64_t rows,
                                                         int F, int il) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;   // 8-element chunk of h
  const int64_t nch = rows * (F >> 3);
  if (i >= nch) return;
  const int64_t r = i / (F >> 3);
  const int c = (int)(i % (F >> 3)) * 8;
  float gv[8], uv[8], o[8];
  unpack8(*(const uint4*)(gu + r * 2 * F + gate_col(c, F, il)), gv);
  unpack8(*(const uint4*)(gu + r * 2 * F + up_col(c, F, il)), uv);
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = gv[e] / (1.f + __expf(-gv[e])) * uv[e];
  *(uint4*)(h + r * F + c) = pack8(o);
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16_t* __restrict__ gu,
                                                         const bf16_t* __restrict__ dh,
                                                         bf16_t* __restrict__ dgu, int64_t rows,
                                                         int F, int il) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nch = rows * (F >> 3);
  if (i >= nch) return;
  const int64_t r = i / (F >> 3);
  const int c = (int)(i % (F >> 3)) * 8;
  float gv[8], uv[8], dv[8], dg[8], du[8];
  const int64_t cg = gate_col(c, F, il), cu = up_col(c, F, il);
  unpack8(*(const uint4*)(gu + r * 2 * F + cg), gv);
  unpack8(*(const uint4*)(gu + r * 2 * F + cu), uv);
  unpack8(*(const uint4*)(dh + r * F + c), dv);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float sg = 1.f / (1.f + __expf(-gv[e]));
    const float silu = gv[e] * sg;
    du[e] = dv[e] * silu;
    dg[e] = dv[e] * uv[e] * sg * (1.f + gv[e] * (1.f - sg));
  }
  *(uint4*)(dgu + r * 2 * F + cg) = pack8(dg);
  *(uint4*)(dgu + r * 2 * F + cu) = pack8(du);
}

// ---------------------------------------------------------------------------------- loss
// One workgroup per row: loss_sum[p] += logsumexp(z) - z[y];  z <- (softmax(z) - onehot) * scale.
__global__ __launch_bounds__(256) void ce_fwd_bwd_kernel(bf16_t* __restrict__ logits,
                                                         const int32_t* __restrict__ labels,
                                                         float* __restrict__ loss_sum, int V,
                                                         int rows_per_trial, float scale,
                                                         int write_grad) {
  __shared__ float red[8];
  const int64_t row = blockIdx.x;
  bf16_t* z = logits + row * V;
  const int nc = V >> 3;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x; c < nc; c += 256) {
    float v[8];
    unpack8(*(const uint4*)(z + 8 * c), v);
    float mx = v[0];
#pragma unroll
    for (int e = 1; e < 8; ++e) mx = fmaxf(mx, v[e]);
    const float mn = fmaxf(m, mx);
    float acc = s * __expf(m - mn);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += __expf(v[e] - mn);
    m = mn;
    s = acc;
  }
  // combine (m, s) over the block
  // lanes (or whole waves) without any chunk hold m = -inf: they contribute 0, never NaN
  const float wm = wave_max(m);
  float ws = (m == -INFINITY) ? 0.f : s * __expf(m - wm);
  ws = wave_sum(ws);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    red[wave] = wm;
    red[4 + wave] = ws;
  }
  __syncthreads();
  float M = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float S = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w)
    if (red[w] != -INFINITY) S += red[4 + w] * __expf(red[w] - M);
  int y = labels[row];
  if (!MOPT_IN_RANGE(y, V, "ce_fwd_bwd label")) y = -1;  // checked build: no loss, no one-hot
  if (threadIdx.x == 0 && y >= 0) {
    const float zy = bf2f(z[y]);
    atomicAdd(loss_sum + row / rows_per_trial, M + __logf(S) - zy);
  }
  if (!write_grad) return;
  __syncthreads();   // z[y] read above before it is overwritten
  const float inv = 1.f / S;
  for (int c = threadIdx.x; c < nc; c += 256) {
    float v[8];
    unpack8(*(const uint4*)(z + 8 * c), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float p = __expf(v[e] - M) * inv - ((8 * c + e) == y ? 1.f : 0.f);
      v[e] = p * scale;
    }
    *(uint4*)(z + 8 * c) = pack8(v);
  }
}

// Register-resident variant for V <= 256 * 8 * NPT: the row is loaded once into NPT 16-byte
// registers per thread, the softmax statistics and the gradient are computed from them -- one
// read and one write of the logits instead of two reads and a write (the second pass of the
// kernel above re-read a 64 KB row per workgroup with ~128 MB of rows in flight: from HBM).
template <int NPT>
__global__ __launch_bounds__(256) void ce_fwd_bwd_reg_kernel(bf16_t* __restrict__ logits,
                                                             const int32_t* __restrict__ labels,
                                                             float* __restrict__ loss_sum, int V,
                                                             int rows_per_trial, float scale,
                                                             int write_grad) {
  __shared__ float red[8];
  const int64_t row = blockIdx.x;
  bf16_t* z = logits + row * V;
  const int nc = V >> 3;
  const int tid = threadIdx.x;
  uint4 r[NPT];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int c = tid + 256 * k;
    r[k] = c < nc ? *(const uint4*)(z + 8 * c) : make_uint4(0, 0, 0, 0);
  }
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    if (tid + 256 * k < nc) {
      float v[8];
      unpack8(r[k], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) m = fmaxf(m, v[e]);
    }
  }
  const float wm = wave_max(m);
  const int wave = tid >> 6, lane = tid & 63;
  if (lane == 0) red[wave] = wm;
  __syncthreads();
  const float M = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    if (tid + 256 * k < nc) {
      float v[8];
      unpack8(r[k], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += __expf(v[e] - M);
    }
  }
  s = wave_sum(s);
  if (lane == 0) red[4 + wave] = s;
  __syncthreads();
  const float S = red[4] + red[5] + red[6] + red[7];
  int y = labels[row];
  if (!MOPT_IN_RANGE(y, V, "ce_fwd_bwd label")) y = -1;  // checked build: no loss, no one-hot
  if (tid == 0 && y >= 0) atomicAdd(loss_sum + row / rows_per_trial, M + __logf(S) - bf2f(z[y]));
  if (!write_grad) return;
  __syncthreads();   // z[y] read above before it is overwritten
  const float inv = 1.f / S;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int c = tid + 256 * k;
    if (c < nc) {
      float v[8];
      unpack8(r[k], v);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        v[e] = (__expf(v[e] - M) * inv - ((8 * c + e) == y ? 1.f : 0.f)) * scale;
      *(uint4*)(z + 8 * c) = pack8(v);
    }
  }
}

// ---------------------------------------------------------------------------------- embedding
__global__ __launch_bounds__(256) void embed_fwd_kernel(const int32_t* __restrict__ tok,
                                                        const bf16_t* __restrict__ table,
                                                        bf16_t* __restrict__ out, int64_t rows,
                                                        int d, int V, int rows_per_trial) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int per = d >> 3;
  if (i >= rows * per) return;
  const int64_t r = i / per;
  const int c = (int)(i % per) * 8;
  const int64_t p = r / rows_per_trial;
  const int t = tok[r];
  if (!MOPT_IN_RANGE(t, V, "embedding token")) {
    *(uint4*)(out + r * d + c) = make_uint4(0, 0, 0, 0);
    return;
  }
  *(uint4*)(out + r * d + c) = *(const uint4*)(table + (p * V + t) * (int64_t)d + c);
}

__global__ __launch_bounds__(256) void embed_bwd_kernel(const int32_t* __restrict__ tok,
                                                        const bf16_t* __restrict__ dout,
                                                        float* __restrict__ dtable32,
                                                        int64_t rows, int d, int V,
                                                        int rows_per_trial) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int per = d >> 3;
  if (i >= rows * per) return;
  const int64_t r = i / per;
  const int c = (int)(i % per) * 8;
  const int64_t p = r / rows_per_trial;
  float v[8];
  unpack8(*(const uint4*)(dout + r * d + c), v);
  if (!MOPT_IN_RANGE(tok[r], V, "embedding backward token")) return;
  float* dst = dtable32 + (p * V + tok[r]) * (int64_t)d + c;
#pragma unroll
  for (int e = 0; e < 8; ++e) atomicAdd(dst + e, v[e]);
}

// Embedding gradient from the (trial, token) keys sorted stably: one wave per sorted position;
// the wave at the start of each run of equal keys sums the run's dout rows in f32 (in token
// order: deterministic) and writes the bf16 row of the table gradient -- no atomics, no f32
// table.  The caller zeroes the table gradient first (rows no token touched stay zero).
__global__ __launch_bounds__(256) void embed_bwd_sorted_kernel(const int64_t* __restrict__ keys,
                                                               const int64_t* __restrict__ order,
                                                               const bf16_t* __restrict__ dout,
                                                               bf16_t* __restrict__ dtable,
                                                               int64_t rows, int d,
                                                               int64_t table_rows) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= rows) return;
  const int64_t key = keys[w];
  if (w > 0 && keys[w - 1] == key) return;  // not the first of its run
  if (!MOPT_IN_RANGE(key, table_rows, "embedding backward token")) return;
  const int nc = d >> 3;
  float acc[kMaxChunks][8];
#pragma unroll
  for (int k = 0; k < kMaxChunks; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[k][e] = 0.f;
  for (int64_t j = w; j < rows && keys[j] == key; ++j) {
    if (!MOPT_IN_RANGE(order[j], rows, "embedding backward sorted order")) continue;
    const bf16_t* src = dout + order[j] * (int64_t)d;
#pragma unroll
    for (int k = 0; k < kMaxChunks; ++k) {
      const int c = lane + 64 * k;
      if (c < nc) {
        float v[8];
        unpack8(*(const uint4*)(src + 8 * c), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[k][e] += v[e];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < kMaxChunks; ++k) {
    const int c = lane + 64 * k;
    if (c < nc) *(uint4*)(dtable + key * (int64_t)d + 8 * c) = pack8(acc[k]);
  }
}

// The keys of embed_bwd_sorted_kernel without a library sort (round 6; torch.sort was eight
// rocprim / aten launches per step): one 1024-thread workgroup per trial sorts the trial's (token,
// row) pairs as 64-bit words token << 32 | row -- the row in the low half makes the order stable
// -- with a bitonic network in LDS (n = the next power of two >= rows_per_trial, padded with
// all-ones words), then writes keys = trial V + token and order = the global row.  Rows per trial
// <= kEmbedSortMax (n 8-byte words of LDS).
constexpr int kEmbedSortMax = 8192;
__global__ __launch_bounds__(1024) void embed_sort_kernel(const int32_t* __restrict__ tok,
                                                          int64_t* __restrict__ keys,
                                                          int64_t* __restrict__ order, int rpt,
                                                          int n, int V) {
  __shared__ uint64_t s[kEmbedSortMax];
  const int p = blockIdx.x, tid = threadIdx.x;
  const int32_t* t = tok + (int64_t)p * rpt;
  for (int i = tid; i < n; i += 1024)
    s[i] = i < rpt ? ((uint64_t)(uint32_t)t[i] << 32) | (uint32_t)i : ~0ull;
  __syncthreads();
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < n; i += 1024) {
        const int ij = i ^ j;
        if (ij > i) {
          const uint64_t a = s[i], b = s[ij];
          if ((a > b) == ((i & k) == 0)) {
            s[i] = b;
            s[ij] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < rpt; i += 1024) {
    const uint64_t w = s[i];
    keys[(int64_t)p * rpt + i] = (int64_t)p * V + (int64_t)(int32_t)(uint32_t)(w >> 32);
    order[(int64_t)p * rpt + i] = (int64_t)p * rpt + (int64_t)(uint32_t)w;
  }
}

// Zero the table-gradient rows of the previous step's sorted keys (one wave per run of equal
// keys; negative / out-of-range keys -- the initial fill -- are skipped).  With it the table
// gradient is never cleared whole: every row outside the previous step's keys is already zero
// (by induction from the zero-initialised buffer), and the rows of this step's keys are fully
// overwritten by embed_bwd_sorted_kernel -- ~50 MB of row stores instead of a 393 MB fill for
// the 125M LM (8 trials x 32000 x 768).
__global__ __launch_bounds__(256) void embed_zero_rows_kernel(const int64_t* __restrict__ keys,
                                                              bf16_t* __restrict__ dtable,
                                                              int64_t rows, int d,
                                                              int64_t table_rows) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= rows) return;
  const int64_t key = keys[w];
  if ((w > 0 && keys[w - 1] == key) || key < 0 || key >= table_rows) return;
  for (int c = lane; c < (d >> 3); c += 64)
    *(uint4*)(dtable + key * (int64_t)d + 8 * c) = make_uint4(0, 0, 0, 0);
}

// RMSNorm weight gradient straight into a bf16 gradient view, two passes without atomics.
// Pass 1: thread (column group cg of 8, slice s, trial p) sums dy * x * rstd over its slice of
// the trial's rows with 16-byte loads and writes 8 floats to part[(p * G + cg) * S + s]
// (G = d / 8: the S partials of one column group are contiguous).  grid (ceil(G/bx), S, P),
// bx = G rounded up to whole waves (<= 256).
// Pass 2: one wave per (p, cg) reads its S partials coalesced (32 B per lane), reduces them
// across the wave and writes the 8 bf16 gradients.
__global__ __launch_bounds__(256) void rmsnorm_dw_partial_kernel(const bf16_t* __restrict__ x,
                                                                 const bf16_t* __restrict__ dy,
                                                                 const float* __restrict__ rstd,
                                                                 float* __restrict__ part, int d,
                                                                 int rows_per_trial) {
  const int cg = blockIdx.x * blockDim.x + threadIdx.x, G = d / 8;
  if (cg >= G) return;
  const int p = blockIdx.z, s = blockIdx.y, S = gridDim.y;
  const int per = (rows_per_trial + S - 1) / S;
  const int r0 = p * rows_per_trial + s * per;
  const int r1 = min(r0 + per, (p + 1) * rows_per_trial);
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll 4
  for (int r = r0; r < r1; ++r) {
    float xv[8], dv[8];
    unpack8(*(const uint4*)(x + (size_t)r * d + 8 * cg), xv);
    unpack8(*(const uint4*)(dy + (size_t)r * d + 8 * cg), dv);
    const float rs = rstd[r];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += dv[e] * xv[e] * rs;
  }
  float* o = part + (((size_t)p * G + cg) * S + s) * 8;
  *(f32x4*)o = f32x4{acc[0], acc[1], acc[2], acc[3]};
  *(f32x4*)(o + 4) = f32x4{acc[4], acc[5], acc[6], acc[7]};
}

__global__ __launch_bounds__(256) void rmsnorm_dw_reduce_kernel(const float* __restrict__ part,
                                                                bf16_t* __restrict__ dw16,
                                                                int groups, int S) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (w >= groups) return;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  const float* q = part + (size_t)w * S * 8;
  for (int s = lane; s < S; s += 64) {
    const f32x4 a = *(const f32x4*)(q + 8 * s), b = *(const f32x4*)(q + 8 * s + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[e] += a[e];
      acc[4 + e] += b[e];
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += __shfl_xor(acc[e], m, 64);
  if (lane == 0) *(uint4*)(dw16 + (size_t)w * 8) = pack8(acc);
}

// f32 -> bf16 (n multiple of 8).
__global__ __launch_bounds__(256) void cast_bf16_kernel(const float* __restrict__ src,
                                                        bf16_t* __restrict__ dst, int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i >= n) return;
  const f32x4 a = *(const f32x4*)(src + i), b = *(const f32x4*)(src + i + 4);
  const float f[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  *(uint4*)(dst + i) = pack8(f);
}

// ---------------------------------------------------------------------------------- AdamW
// Per-trial sum of squared gradients.  One block walks kSumChunks consecutive chunks (the table
// is segment-major, trial-minor, so a block's chunks almost always belong to one trial) and
// issues one atomic per trial run: ~64x fewer same-address atomics than one per chunk, which
// serialised at the L2 and held this pass at ~0.3 TB/s.
constexpr int kSumChunks = 64;

__global__ __launch_bounds__(256) void grad_sumsq_kernel(const Segment* __restrict__ segs,
                                                         const SegChunk* __restrict__ chunks,
                                                         int n_chunks,
                                                         const bf16_t* __restrict__ g16,
                                                         float* __restrict__ sumsq) {
  // The block's chunk descriptors are staged in LDS first (one dependent descriptor load per
  // chunk kept the loop a latency chain: 0.42 ms for 268 MB, ~0.6 TB/s), then the data loads of
  // four chunks are issued back to back.
  __shared__ float red[4];
  __shared__ int64_t c_off[kSumChunks];
  __shared__ int c_len[kSumChunks], c_trial[kSumChunks];
  const int c0 = blockIdx.x * kSumChunks;
  const int n = min(kSumChunks, n_chunks - c0);
  if ((int)threadIdx.x < n) {
    const SegChunk ch = chunks[c0 + threadIdx.x];
    const Segment sg = segs[ch.seg];
    const int64_t end = min(ch.start + (int64_t)kAdamChunk, (int64_t)(ch.trial + 1) * sg.numel);
    c_off[threadIdx.x] = sg.off + ch.start;
    c_len[threadIdx.x] = (int)(end - ch.start);
    c_trial[threadIdx.x] = ch.trial;
  }
  __syncthreads();
  const int e0 = 8 * threadIdx.x;
  float acc = 0.f;
  int trial = c_trial[0];
  int j = 0;
  while (j < n) {
    // fast path: four chunks of the current trial, four independent 16-byte loads in flight
    if (j + 4 <= n && c_trial[j] == trial && c_trial[j + 1] == trial &&
        c_trial[j + 2] == trial && c_trial[j + 3] == trial) {
      uint4 u[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        u[k] = e0 < c_len[j + k] ? *(const uint4*)(g16 + c_off[j + k] + e0) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float v[8];
        unpack8(u[k], v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc += v[e] * v[e];
      }
      j += 4;
      continue;
    }
    if (c_trial[j] != trial) {        // block-uniform: flush the finished trial's run
      const float tot = block_sum(acc, red);
      if (threadIdx.x == 0) atomicAdd(sumsq + trial, tot);
      acc = 0.f;
      trial = c_trial[j];
    }
    if (e0 < c_len[j]) {
      float v[8];
      unpack8(*(const uint4*)(g16 + c_off[j] + e0), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += v[e] * v[e];
    }
    ++j;
  }
  const float tot = block_sum(acc, red);
  if (threadIdx.x == 0) atomicAdd(sumsq + trial, tot);
}

// 8 consecutive master weights at element o: f32 (p32), or SPLIT, the (hi, lo) halves of
// common.h -- hi is the bf16 working copy p16 itself, lo a 16-bit residual in ``master`` -- so
// the master costs 2 bytes beyond the working copy instead of 4, and the update writes no
// separately rounded copy.
template <bool SPLIT>
__device__ __forceinline__ void load_master8(const void* master, const bf16_t* p16, int64_t o,
                                             float (&w)[8]) {
  f32x4 a, b;
  if constexpr (SPLIT) {
    const uint4 hi = *(const uint4*)(p16 + o);
    const uint4 lo = *(const uint4*)((const uint16_t*)master + o);
    a = join4(make_uint2(hi.x, hi.y), make_uint2(lo.x, lo.y));
    b = join4(make_uint2(hi.z, hi.w), make_uint2(lo.z, lo.w));
  } else {
    a = *(const f32x4*)((const float*)master + o);
    b = *(const f32x4*)((const float*)master + o + 4);
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    w[e] = a[e];
    w[4 + e] = b[e];
  }
}

template <bool SPLIT>
__device__ __forceinline__ void store_master8(void* master, bf16_t* p16, int64_t o,
                                              const float (&w)[8]) {
  const f32x4 a{w[0], w[1], w[2], w[3]}, b{w[4], w[5], w[6], w[7]};
  if constexpr (SPLIT) {
    uint2 ha, la, hb, lb;
    split4(a, ha, la);
    split4(b, hb, lb);
    *(uint4*)(p16 + o) = make_uint4(ha.x, ha.y, hb.x, hb.y);
    *(uint4*)((uint16_t*)master + o) = make_uint4(la.x, la.y, lb.x, lb.y);
  } else {
    *(f32x4*)((float*)master + o) = a;
    *(f32x4*)((float*)master + o + 4) = b;
    *(uint4*)(p16 + o) = pack8(w);
  }
}

// M16: the first moment is kept in bf16 (RNE after each update; the update itself uses the f32
// value).  The second moment stays f32: with b2 = 0.999 its per-step change (0.1 %) is below
// bf16 resolution and would stall.  Bytes per parameter and step: gradient 2, master 4 (SPLIT:
// hi + lo, of which hi is the working copy) or 4 + the 2 of the rewritten bf16 copy, first
// moment 2 x 2 (M16), second moment 2 x 4 -- 22 with M16 + SPLIT, 24 with M16 alone.
template <bool M16, bool SPLIT>
__global__ __launch_bounds__(256) void adamw_multi_kernel(const Segment* __restrict__ segs,
                                                          const SegChunk* __restrict__ chunks,
                                                          const LmHP* __restrict__ hp,
                                                          const float* __restrict__ sumsq,
                                                          void* __restrict__ master,
                                                          bf16_t* __restrict__ p16,
                                                          const bf16_t* __restrict__ g16,
                                                          void* __restrict__ mbuf,
                                                          float* __restrict__ v32) {
  const SegChunk ch = chunks[blockIdx.x];
  const Segment sg = segs[ch.seg];
  const int64_t i = ch.start + 8 * threadIdx.x;
  const int64_t end = min(ch.start + (int64_t)kAdamChunk, (int64_t)(ch.trial + 1) * sg.numel);
  if (i >= end) return;
  const int p = ch.trial;
  const LmHP h = hp[p];
  float clip = 1.f;
  if (h.max_norm > 0.f) {
    const float nrm = sqrtf(sumsq[p]);
    if (nrm > h.max_norm) clip = h.max_norm / (nrm + 1e-6f);
  }
  const float tf = (float)h.t;
  const float bc1 = 1.f - __powf(h.b1, tf), bc2 = 1.f - __powf(h.b2, tf);
  const float step = h.lr / bc1, rbc2 = rsqrtf(bc2);
  const int64_t o = sg.off + i;
  float gv[8], we[8];
  unpack8(*(const uint4*)(g16 + o), gv);
  load_master8<SPLIT>(master, p16, o, we);
  f32x4 m0, m1;
  if constexpr (M16) {
    const uint4 mv = *(const uint4*)((const bf16_t*)mbuf + o);
    m0 = bf4_to_f32(make_uint2(mv.x, mv.y));
    m1 = bf4_to_f32(make_uint2(mv.z, mv.w));
  } else {
    m0 = *(const f32x4*)((const float*)mbuf + o);
    m1 = *(const f32x4*)((const float*)mbuf + o + 4);
  }
  const f32x4 v0 = *(const f32x4*)(v32 + o), v1 = *(const f32x4*)(v32 + o + 4);
  float me[8] = {m0[0], m0[1], m0[2], m0[3], m1[0], m1[1], m1[2], m1[3]};
  float ve[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float gr = gv[e] * clip;
    we[e] *= 1.f - h.lr * h.wd;
    me[e] = h.b1 * me[e] + (1.f - h.b1) * gr;
    ve[e] = h.b2 * ve[e] + (1.f - h.b2) * gr * gr;
    we[e] -= step * me[e] / (sqrtf(ve[e]) * rbc2 + h.eps);
  }
  store_master8<SPLIT>(master, p16, o, we);
  if constexpr (M16) {
    *(uint4*)((bf16_t*)mbuf + o) = pack8(me);
  } else {
    *(f32x4*)((float*)mbuf + o) = f32x4{me[0], me[1], me[2], me[3]};
    *(f32x4*)((float*)mbuf + o + 4) = f32x4{me[4], me[5], me[6], me[7]};
  }
  *(f32x4*)(v32 + o) = f32x4{ve[0], ve[1], ve[2], ve[3]};
  *(f32x4*)(v32 + o + 4) = f32x4{ve[4], ve[5], ve[6], ve[7]};
}

// SGD with momentum (PyTorch convention: m = mu m + (g + wd w); w -= lr m), per-trial lr /
// momentum (LmHP.b1) / wd, optional per-trial grad-norm clipping (north-star kernel K5).
template <bool SPLIT>
__global__ __launch_bounds__(256) void sgd_multi_kernel(const Segment* __restrict__ segs,
                                                        const SegChunk* __restrict__ chunks,
                                                        const LmHP* __restrict__ hp,
                                                        const float* __restrict__ sumsq,
                                                        void* __restrict__ master,
                                                        bf16_t* __restrict__ p16,
                                                        const bf16_t* __restrict__ g16,
                                                        float* __restrict__ m32) {
  const SegChunk ch = chunks[blockIdx.x];
  const Segment sg = segs[ch.seg];
  const int64_t i = ch.start + 8 * threadIdx.x;
  const int64_t end = min(ch.start + (int64_t)kAdamChunk, (int64_t)(ch.trial + 1) * sg.numel);
  if (i >= end) return;
  const LmHP h = hp[ch.trial];
  float clip = 1.f;
  if (h.max_norm > 0.f) {
    const float nrm = sqrtf(sumsq[ch.trial]);
    if (nrm > h.max_norm) clip = h.max_norm / (nrm + 1e-6f);
  }
  const int64_t o = sg.off + i;
  float gv[8], we[8];
  unpack8(*(const uint4*)(g16 + o), gv);
  load_master8<SPLIT>(master, p16, o, we);
  const f32x4 m0 = *(const f32x4*)(m32 + o), m1 = *(const f32x4*)(m32 + o + 4);
  float me[8] = {m0[0], m0[1], m0[2], m0[3], m1[0], m1[1], m1[2], m1[3]};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    me[e] = h.b1 * me[e] + gv[e] * clip + h.wd * we[e];
    we[e] -= h.lr * me[e];
  }
  store_master8<SPLIT>(master, p16, o, we);
  *(f32x4*)(m32 + o) = f32x4{me[0], me[1], me[2], me[3]};
  *(f32x4*)(m32 + o + 4) = f32x4{me[4], me[5], me[6], me[7]};
}

inline dim3 grid1(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

}  // namespace

extern "C" {

int mopt_rmsnorm_fwd(const void* x, const void* w, void* y, void* rstd, int rows, int d,
                     int rows_per_trial, float eps, void* stream) {
  if (d % 8 || d > 64 * 8 * kMaxChunks) return 1;
  hipLaunchKernelGGL(rmsnorm_fwd_kernel<false>, dim3((rows + 3) / 4), dim3(256), 0,
                     (hipStream_t)stream, (const bf16_t*)x, (const bf16_t*)nullptr,
                     (bf16_t*)nullptr, (const bf16_t*)w, (bf16_t*)y, (float*)rstd, rows, d,
                     rows_per_trial, eps);
  return (int)hipGetLastError();
}

// xs = x + res; y = rmsnorm(xs) * w   (the transformer's residual add fused into the next norm)
int mopt_add_rmsnorm_fwd(const void* x, const void* res, void* xs, const void* w, void* y,
                         void* rstd, int rows, int d, int rows_per_trial, float eps,
                         void* stream) {
  if (d % 8 || d > 64 * 8 * kMaxChunks) return 1;
  hipLaunchKernelGGL(rmsnorm_fwd_kernel<true>, dim3((rows + 3) / 4), dim3(256), 0,
                     (hipStream_t)stream, (const bf16_t*)x, (const bf16_t*)res, (bf16_t*)xs,
                     (const bf16_t*)w, (bf16_t*)y, (float*)rstd, rows, d, rows_per_trial, eps);
  return (int)hipGetLastError();
}

// dx = rmsnorm_bwd(dy) (+ dres when dres != null); dw32 += the weight gradient
int mopt_rmsnorm_bwd_res(const void* x, const void* w, const void* dy, const void* dres,
                         const void* rstd, void* dx, void* dw32, int rows, int d,
                         int rows_per_trial, void* stream);

int mopt_rmsnorm_bwd(const void* x, const void* w, const void* dy, const void* rstd, void* dx,
                     void* dw32, int rows, int d, int rows_per_trial, void* stream) {
  return mopt_rmsnorm_bwd_res(x, w, dy, nullptr, rstd, dx, dw32, rows, d, rows_per_trial,
                              stream);
}

int mopt_rmsnorm_bwd_res(const void* x, const void* w, const void* dy, const void* dres,
                         const void* rstd, void* dx, void* dw32, int rows, int d,
                         int rows_per_trial, void* stream) {
  if (d % 8 || d > 64 * 8 * kMaxChunks) return 1;
  hipStream_t st = (hipStream_t)stream;
  if (dres != nullptr)
    hipLaunchKernelGGL(rmsnorm_bwd_dx_kernel<true>, dim3((rows + 3) / 4), dim3(256), 0, st,
                       (const bf16_t*)x, (const bf16_t*)w, (const bf16_t*)dy,
                       (const bf16_t*)dres, (const float*)rstd, (bf16_t*)dx, rows, d,
                       rows_per_trial);
  else
    hipLaunchKernelGGL(rmsnorm_bwd_dx_kernel<false>, dim3((rows + 3) / 4), dim3(256), 0, st,
                       (const bf16_t*)x, (const bf16_t*)w, (const bf16_t*)dy,
                       (const bf16_t*)nullptr, (const float*)rstd, (bf16_t*)dx, rows, d,
                       rows_per_trial);
  if (dw32 == nullptr) return (int)hipGetLastError();  // weight gradient via mopt_rmsnorm_dw16
  const int P = rows / rows_per_trial;
  const int splits = max(1, min(64, rows_per_trial / 64));
  hipLaunchKernelGGL(rmsnorm_bwd_dw_kernel, dim3((d + 255) / 256, splits, P), dim3(256), 0, st,
                     (const bf16_t*)x, (const bf16_t*)dy, (const float*)rstd, (float*)dw32, d,
                     rows_per_trial);
  return (int)hipGetLastError();
}

// il: interleaved pairs (2j, 2j + 1) instead of rotate-half pairs (j, j + 32) -- the layout the
// QKV GEMM's RoPE epilogue writes (csrc/pgemm.hip EPI 3)
int mopt_rope_fwd(const void* qkv, const void* cosv, const void* sinv, void* q, void* k, void* v,
                  int rows, int T, int H, int il, void* stream) {
  const int64_t total = (int64_t)rows * 3 * H * 4;
  hipLaunchKernelGGL(rope_fwd_kernel, grid1(total), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)qkv, (const float*)cosv, (const float*)sinv, (bf16_t*)q,
                     (bf16_t*)k, (bf16_t*)v, rows, T, H, il);
  return (int)hipGetLastError();
}

int mopt_rope_bwd(const void* dq, const void* dk, const void* dv, const void* cosv,
                  const void* sinv, void* dqkv, int rows, int T, int H, int il, void* stream) {
  const int64_t total = (int64_t)rows * 3 * H * 4;
  hipLaunchKernelGGL(rope_bwd_kernel, grid1(total), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)dq, (const bf16_t*)dk, (const bf16_t*)dv, (const float*)cosv,
                     (const float*)sinv, (bf16_t*)dqkv, rows, T, H, il);
  return (int)hipGetLastError();
}

// il: gate / up in interleaved 16-column groups (F a multiple of 16) instead of two halves
int mopt_swiglu_fwd(const void* gu, void* h, int64_t rows, int F, int il, void* stream) {
  if (F % 8 || (il && F % 16)) return 1;
  hipLaunchKernelGGL(swiglu_fwd_kernel, grid1(rows * (F / 8)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)gu, (bf16_t*)h, rows, F, il);
  return (int)hipGetLastError();
}

int mopt_swiglu_bwd(const void* gu, const void* dh, void* dgu, int64_t rows, int F, int il,
                    void* stream) {
  if (F % 8 || (il && F % 16)) return 1;
  hipLaunchKernelGGL(swiglu_bwd_kernel, grid1(rows * (F / 8)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)gu, (const bf16_t*)dh, (bf16_t*)dgu, rows, F, il);
  return (int)hipGetLastError();
}

int mopt_ce_fwd_bwd(void* logits, const void* labels, void* loss_sum, int rows, int V,
                    int rows_per_trial, float scale, int write_grad, void* stream) {
  if (V % 8) return 1;
  if (V <= 256 * 8 * 16)    // the row fits 16 registers of 16 bytes per thread
    hipLaunchKernelGGL(ce_fwd_bwd_reg_kernel<16>, dim3(rows), dim3(256), 0, (hipStream_t)stream,
                       (bf16_t*)logits, (const int32_t*)labels, (float*)loss_sum, V,
                       rows_per_trial, scale, write_grad);
  else
    hipLaunchKernelGGL(ce_fwd_bwd_kernel, dim3(rows), dim3(256), 0, (hipStream_t)stream,
                       (bf16_t*)logits, (const int32_t*)labels, (float*)loss_sum, V,
                       rows_per_trial, scale, write_grad);
  return (int)hipGetLastError();
}

int mopt_embed_fwd(const void* tok, const void* table, void* out, int64_t rows, int d, int V,
                   int rows_per_trial, void* stream) {
  if (d % 8) return 1;
  hipLaunchKernelGGL(embed_fwd_kernel, grid1(rows * (d / 8)), dim3(256), 0, (hipStream_t)stream,
                     (const int32_t*)tok, (const bf16_t*)table, (bf16_t*)out, rows, d, V,
                     rows_per_trial);
  return (int)hipGetLastError();
}

int mopt_embed_bwd(const void* tok, const void* dout, void* dtable32, int64_t rows, int d, int V,
                   int rows_per_trial, void* stream) {
  if (d % 8) return 1;
  hipLaunchKernelGGL(embed_bwd_kernel, grid1(rows * (d / 8)), dim3(256), 0, (hipStream_t)stream,
                     (const int32_t*)tok, (const bf16_t*)dout, (float*)dtable32, rows, d, V,
                     rows_per_trial);
  return (int)hipGetLastError();
}

// keys [rows] = trial * V + token sorted ascending (stably), order [rows] the dout row of each;
// dtable bf16 [P][V][d] zeroed by the caller.
int mopt_embed_bwd_sorted(const void* keys, const void* order, const void* dout, void* dtable,
                          int64_t rows, int d, int64_t table_rows, void* stream) {
  if (d % 8 || d > 64 * 8 * kMaxChunks) return 1;
  hipLaunchKernelGGL(embed_bwd_sorted_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, (const int64_t*)keys, (const int64_t*)order,
                     (const bf16_t*)dout, (bf16_t*)dtable, rows, d, table_rows);
  return (int)hipGetLastError();
}

// The in-tree key sort (embed_sort_kernel): tok [P * rpt] int32 -> keys, order [P * rpt] int64.
int mopt_embed_sort(const void* tok, void* keys, void* order, int P, int rpt, int V,
                    void* stream) {
  int n = 1;
  while (n < rpt) n <<= 1;
  if (P <= 0 || rpt <= 0 || n > kEmbedSortMax) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(embed_sort_kernel, dim3(P), dim3(1024), 0, (hipStream_t)stream,
                     (const int32_t*)tok, (int64_t*)keys, (int64_t*)order, rpt, n, V);
  return (int)hipGetLastError();
}

// Zero the dtable rows named by the previous step's sorted keys (embed_zero_rows_kernel).
int mopt_embed_zero_rows(const void* keys, void* dtable, int64_t rows, int d, int64_t table_rows,
                         void* stream) {
  if (d % 8) return 1;
  hipLaunchKernelGGL(embed_zero_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, (const int64_t*)keys, (bf16_t*)dtable, rows, d,
                     table_rows);
  return (int)hipGetLastError();
}

// dw16 (bf16 [P][d], a gradient view) = the RMSNorm weight gradient; part: f32 scratch of
// mopt_rmsnorm_dw_splits(rows_per_trial) * P * d elements (fully overwritten, no zeroing).
int mopt_rmsnorm_dw_splits(int rows_per_trial) { return max(1, min(256, rows_per_trial / 16)); }

int mopt_rmsnorm_dw16(const void* x, const void* dy, const void* rstd, void* part, void* dw16,
                      int rows, int d, int rows_per_trial, void* stream) {
  if (d % 8 || rows % rows_per_trial) return 1;
  hipStream_t st = (hipStream_t)stream;
  const int P = rows / rows_per_trial, S = mopt_rmsnorm_dw_splits(rows_per_trial), G = d / 8;
  const int bx = min(256, (G + 63) / 64 * 64);
  hipLaunchKernelGGL(rmsnorm_dw_partial_kernel, dim3((G + bx - 1) / bx, S, P), dim3(bx), 0, st,
                     (const bf16_t*)x, (const bf16_t*)dy, (const float*)rstd, (float*)part, d,
                     rows_per_trial);
  hipLaunchKernelGGL(rmsnorm_dw_reduce_kernel, dim3((P * G + 3) / 4), dim3(256), 0, st,
                     (const float*)part, (bf16_t*)dw16, P * G, S);
  return (int)hipGetLastError();
}

// dx = rmsnorm_bwd(dy) (+ dres when non-null) and the bf16 weight gradient dw16 [P][d] of the same
// pass (rmsnorm_bwd_dxdw_kernel + rmsnorm_dw_reduce_kernel; part: mopt_rmsnorm_dw_splits(rpt) *
// P * d f32, fully overwritten)
int mopt_rmsnorm_bwd_dw16(const void* x, const void* w, const void* dy, const void* dres,
                          const void* rstd, void* dx, void* part, void* dw16, int rows, int d,
                          int rows_per_trial, void* stream) {
  if (d % 8 || d > 64 * 8 * kMaxChunks || rows % rows_per_trial) return 1;
  hipStream_t st = (hipStream_t)stream;
  const int P = rows / rows_per_trial, S = mopt_rmsnorm_dw_splits(rows_per_trial), G = d / 8;
  const int nch = (G + 63) / 64;
  const size_t lds = (size_t)4 * d * sizeof(float);
#define L(RES, N)                                                                               \
  hipLaunchKernelGGL((rmsnorm_bwd_dxdw_kernel<RES, N>), dim3(S, P), dim3(256), lds, st,         \
                     (const bf16_t*)x, (const bf16_t*)w, (const bf16_t*)dy, (const bf16_t*)dres, \
                     (const float*)rstd, (bf16_t*)dx, (float*)part, d, rows_per_trial, S)
  const bool res = dres != nullptr;
  switch (nch) {
    case 1: if (res) L(true, 1); else L(false, 1); break;
    case 2: if (res) L(true, 2); else L(false, 2); break;
    case 3: if (res) L(true, 3); else L(false, 3); break;
    default: if (res) L(true, 4); else L(false, 4); break;
  }
#undef L
  hipLaunchKernelGGL(rmsnorm_dw_reduce_kernel, dim3((P * G + 3) / 4), dim3(256), 0, st,
                     (const float*)part, (bf16_t*)dw16, P * G, S);
  return (int)hipGetLastError();
}

int mopt_cast_bf16(const void* src, void* dst, int64_t n, void* stream) {
  if (n % 8) return 1;
  hipLaunchKernelGGL(cast_bf16_kernel, grid1(n / 8), dim3(256), 0, (hipStream_t)stream,
                     (const float*)src, (bf16_t*)dst, n);
  return (int)hipGetLastError();
}

// m16: the first moment buffer is bf16 (else f32)
// master: f32 master weights, or (split) the 16-bit low halves whose high halves are p16
int mopt_adamw_multi(const void* segs, const void* chunks, int n_chunks, const void* hp,
                     void* sumsq, void* master, void* p16, const void* g16, void* m, void* v32,
                     int P, int clip, int m16, int split, void* stream) {
  if (n_chunks <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (clip) {
    (void)hipMemsetAsync(sumsq, 0, sizeof(float) * P, st);
    hipLaunchKernelGGL(grad_sumsq_kernel, dim3((n_chunks + kSumChunks - 1) / kSumChunks),
                       dim3(256), 0, st, (const Segment*)segs, (const SegChunk*)chunks, n_chunks,
                       (const bf16_t*)g16, (float*)sumsq);
  }
  auto kern = m16 ? (split ? adamw_multi_kernel<true, true> : adamw_multi_kernel<true, false>)
                  : (split ? adamw_multi_kernel<false, true> : adamw_multi_kernel<false, false>);
  hipLaunchKernelGGL(kern, dim3(n_chunks), dim3(256), 0, st, (const Segment*)segs,
                     (const SegChunk*)chunks, (const LmHP*)hp, (const float*)sumsq, master,
                     (bf16_t*)p16, (const bf16_t*)g16, m, (float*)v32);
  return (int)hipGetLastError();
}

int mopt_sgd_multi(const void* segs, const void* chunks, int n_chunks, const void* hp,
                   void* sumsq, void* master, void* p16, const void* g16, void* m32, int P,
                   int clip, int split, void* stream) {
  if (n_chunks <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (clip) {
    (void)hipMemsetAsync(sumsq, 0, sizeof(float) * P, st);
    hipLaunchKernelGGL(grad_sumsq_kernel, dim3((n_chunks + kSumChunks - 1) / kSumChunks),
                       dim3(256), 0, st, (const Segment*)segs, (const SegChunk*)chunks, n_chunks,
                       (const bf16_t*)g16, (float*)sumsq);
  }
  hipLaunchKernelGGL((split ? sgd_multi_kernel<true> : sgd_multi_kernel<false>), dim3(n_chunks),
                     dim3(256), 0, st, (const Segment*)segs, (const SegChunk*)chunks,
                     (const LmHP*)hp, (const float*)sumsq, master, (bf16_t*)p16,
                     (const bf16_t*)g16, (float*)m32);
  return (int)hipGetLastError();
}

}  // extern "C"

// device-side index checks of the checked build (common.h)
MOPT_VIOLATIONS_READER(lm_ops)
