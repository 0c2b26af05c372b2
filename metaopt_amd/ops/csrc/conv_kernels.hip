// Fused BatchNorm(+residual)(+ReLU) for the population ResNet (north-star kernel K8; the
// convolutions themselves are implicit GEMMs in pgemm.hip, K3).  Activations are NHWC bf16 with
// a leading population dimension folded into N: x[(p * B + n)][h][w][c]; C is a multiple of 8 so
// every lane moves 16 bytes.
//
//   bn_reduce   per (trial, channel) sums over the trial's N*H*W rows (statistics / backward)
//   bn_finalize mean / rstd per (trial, channel), running-statistics update (momentum, unbiased)
//   bn_apply    y = relu?(gamma (x - mean) rstd + beta + residual?)
//   bn_bwd_*    dz = dy * relu'(y); sums of dz and dz * xhat; dx, dgamma, dbeta, dresidual
//
// relu mode of the backward: 0 none, 1 relu'(y) read off the stored output y, 2 relu'(.)
// recomputed from x (x sc + sh > 0, the forward's own arithmetic) -- for a BatchNorm without a
// residual, which then never reads y: one tensor less through both backward passes.
#include "common.h"

using namespace mopt;

namespace {

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

// Every kernel below runs on a grid (row chunks, P): blockIdx.y is the trial, thread = (row group
// rg, 8-channel chunk ch), so a thread's per-channel constants (statistics, gamma, beta) are loaded
// once into registers and its rows are strided by the 256 / (C / 8) row groups of the block --
// no 64-bit division per element, and UNROLL independent 16-byte loads in flight per thread
// (round 2's one-vector-per-thread versions ran at ~1.5 TB/s: 37 % of a ResNet-20 step).
#ifndef MOPT_BN_UNROLL
#define MOPT_BN_UNROLL 4
#endif
constexpr int UNROLL = MOPT_BN_UNROLL;

// Per (trial, channel) reductions over the trial's M rows: a wave's lanes with the same ch are
// summed by xor-shuffles over the lane bits above log2(C/8), then the 4 waves through LDS, then
// one atomic per (trial, channel) and block.  C / 8 a power of two <= 64.
//   BWD = false: sums[p][0][c] += x,  sums[p][1][c] += x^2                 (batch statistics)
//   BWD = true:  dz = dy * relu'(y); sums[p][0][c] += dz, sums[p][1][c] += dz * xhat
template <bool BWD>
__global__ __launch_bounds__(256) void bn_reduce_kernel(const bf16_t* __restrict__ x,
                                                        const bf16_t* __restrict__ y,
                                                        const bf16_t* __restrict__ dy,
                                                        const float* __restrict__ stat,
                                                        const bf16_t* __restrict__ gamma,
                                                        const bf16_t* __restrict__ beta,
                                                        float* __restrict__ sums, int64_t M,
                                                        int C, int rows_per_block, int relu) {
  __shared__ float red[4][2][64];
  const int cc = C >> 3, p = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ch = tid & (cc - 1), rg = tid / cc, ng = 256 / cc;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(r0 + rows_per_block, M);
  const int64_t base = (int64_t)p * M * C + 8 * ch;
  float mean[8], rstd[8], sc[8], sh[8];
  if (BWD) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      mean[e] = stat[(2 * p) * C + 8 * ch + e];
      rstd[e] = stat[(2 * p + 1) * C + 8 * ch + e];
    }
    if (relu == 2) {
      float g[8], b[8];
      unpack8(*(const uint4*)(gamma + (int64_t)p * C + 8 * ch), g);
      unpack8(*(const uint4*)(beta + (int64_t)p * C + 8 * ch), b);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sc[e] = g[e] * rstd[e];
        sh[e] = b[e] - mean[e] * sc[e];
      }
    }
  }
  float a[8], b[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = b[e] = 0.f;
  for (int64_t r = r0 + rg; r < r1; r += UNROLL * ng) {
    uint4 xr[UNROLL], dr[UNROLL], yr[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {          // all loads first: UNROLL rows in flight
      const int64_t ru = r + u * ng;
      const int64_t o = base + (ru < r1 ? ru : r) * C;
      xr[u] = *(const uint4*)(x + o);
      if (BWD) {
        dr[u] = *(const uint4*)(dy + o);
        if (relu == 1) yr[u] = *(const uint4*)(y + o);
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (r + u * ng >= r1) break;
      float xv[8];
      unpack8(xr[u], xv);
      if (!BWD) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          a[e] += xv[e];
          b[e] += xv[e] * xv[e];
        }
      } else {
        float dv[8], yv[8];
        unpack8(dr[u], dv);
        if (relu == 1) unpack8(yr[u], yv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool off = relu == 1 ? yv[e] <= 0.f
                                     : (relu == 2 && xv[e] * sc[e] + sh[e] + 0.f <= 0.f);
          const float dz = off ? 0.f : dv[e];
          a[e] += dz;
          b[e] += dz * (xv[e] - mean[e]) * rstd[e];
        }
      }
    }
  }
  for (int off = 32; off >= cc; off >>= 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      a[e] += __shfl_xor(a[e], off, 64);
      b[e] += __shfl_xor(b[e], off, 64);
    }
  }
  if (lane < cc) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[wave][0][8 * lane + e] = a[e];
      red[wave][1][8 * lane + e] = b[e];
    }
  }
  __syncthreads();
  if (tid < 2 * C) {
    const int k = tid / C, c = tid % C;
    const float v = red[0][k][c] + red[1][k][c] + red[2][k][c] + red[3][k][c];
    atomicAdd(sums + (2 * p + k) * C + c, v);
  }
}

// one thread per (trial, channel): mean / rstd (train: batch stats, eval: running stats)
__global__ void bn_finalize_kernel(const float* __restrict__ sums, float* __restrict__ stat,
                                   float* __restrict__ running, int P, int C, int64_t M,
                                   float eps, float momentum, int train) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * C) return;
  const int p = i / C, c = i % C;
  float* rm = running + (int64_t)p * 2 * C;  // [P][2][C]: running mean, running var
  float mean, var;
  if (train) {
    mean = sums[(2 * p) * C + c] / (float)M;
    var = fmaxf(sums[(2 * p + 1) * C + c] / (float)M - mean * mean, 0.f);
    rm[c] = (1.f - momentum) * rm[c] + momentum * mean;
    rm[C + c] = (1.f - momentum) * rm[C + c] + momentum * var * (float)M / (float)max(M - 1, (int64_t)1);
  } else {
    mean = rm[c];
    var = rm[C + c];
  }
  stat[(2 * p) * C + c] = mean;
  stat[(2 * p + 1) * C + c] = rsqrtf(var + eps);
}

// y = relu?(x * sc + sh + residual?), sc = gamma rstd, sh = beta - mean sc (per trial, channel);
// gamma/beta bf16 [P][C]; stat [P][2][C].  res_c > 0: the residual is the option-A shortcut of
// the full-resolution block input (x[2i][2j][c < res_c], zero above).
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16_t* __restrict__ x,
                                                       const float* __restrict__ stat,
                                                       const bf16_t* __restrict__ gamma,
                                                       const bf16_t* __restrict__ beta,
                                                       const bf16_t* __restrict__ res,
                                                       bf16_t* __restrict__ y, int64_t M, int C,
                                                       int rows_per_block, int relu, int res_c,
                                                       int res_ohl) {
  const int cc = C >> 3, p = blockIdx.y;
  const int tid = threadIdx.x, ch = tid & (cc - 1), rg = tid / cc, ng = 256 / cc;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(r0 + rows_per_block, M);
  float sc[8], sh[8];
  {
    float g[8], b[8];
    unpack8(*(const uint4*)(gamma + (int64_t)p * C + 8 * ch), g);
    unpack8(*(const uint4*)(beta + (int64_t)p * C + 8 * ch), b);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float mean = stat[(2 * p) * C + 8 * ch + e], rstd = stat[(2 * p + 1) * C + 8 * ch + e];
      sc[e] = g[e] * rstd;
      sh[e] = b[e] - mean * sc[e];
    }
  }
  const bool sub2 = res != nullptr && res_c > 0;
  const bool res_here = !sub2 || 8 * ch < res_c;     // option A: channels >= res_c add zero
  const int hin = 2 << res_ohl;
  for (int64_t r = r0 + rg; r < r1; r += UNROLL * ng) {
    uint4 xr[UNROLL], rr[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t ru = r + u * ng;
      const int64_t row = (int64_t)p * M + (ru < r1 ? ru : r);
      xr[u] = *(const uint4*)(x + row * C + 8 * ch);
      if (res != nullptr && res_here) {
        if (!sub2) {
          rr[u] = *(const uint4*)(res + row * C + 8 * ch);
        } else {
          const int64_t img = row >> (2 * res_ohl);
          const int pix = (int)(row & ((1 << (2 * res_ohl)) - 1));
          const int i2 = 2 * (pix >> res_ohl), j2 = 2 * (pix & ((1 << res_ohl) - 1));
          rr[u] = *(const uint4*)(res + ((img * hin + i2) * hin + j2) * res_c + 8 * ch);
        }
      } else {
        rr[u] = make_uint4(0u, 0u, 0u, 0u);
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t ru = r + u * ng;
      if (ru >= r1) break;
      float v[8], rv[8];
      unpack8(xr[u], v);
      unpack8(rr[u], rv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        // (explicit fma: conv_direct.hip's bnres_chunk forms the same block output in its
        //  staging and must round identically)
        const float o = fmaf(v[e], sc[e], sh[e]) + rv[e];
        v[e] = relu ? fmaxf(o, 0.f) : o;
      }
      *(uint4*)(y + ((int64_t)p * M + ru) * C + 8 * ch) = pack8(v);
    }
  }
}

// dz = dy * relu'(y); dx = gamma rstd (dz - sum(dz)/M - xhat sum(dz xhat)/M) = k1 dz + k2 x + k3
// per (trial, channel) constants; dres = dz.  Block (0, 0) also writes (sum dz xhat, sum dz)
// straight into the bf16 dgamma / dbeta gradients when given.
// RELU (the relu mode) is a template parameter: with one kernel for all three modes the y stream's
// registers and the shift constants were allocated for every mode (130 VGPRs, 3 waves per SIMD)
template <int RELU>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16_t* __restrict__ x,
                                                           const bf16_t* __restrict__ y,
                                                           const bf16_t* __restrict__ dy,
                                                           const float* __restrict__ stat,
                                                           const float* __restrict__ sums,
                                                           const bf16_t* __restrict__ gamma,
                                                           const bf16_t* __restrict__ beta,
                                                           bf16_t* __restrict__ dx,
                                                           bf16_t* __restrict__ dres,
                                                           bf16_t* __restrict__ dgamma,
                                                           bf16_t* __restrict__ dbeta, int64_t M,
                                                           int C, int P, int rows_per_block,
                                                           int relu_rt) {
  const int relu = RELU >= 0 ? RELU : relu_rt;   // (-1: the runtime mode, MOPT_BN_APPLY_RT A/B)
  const int cc = C >> 3, p = blockIdx.y;
  const int tid = threadIdx.x, ch = tid & (cc - 1), rg = tid / cc, ng = 256 / cc;
  if (blockIdx.x == 0 && blockIdx.y == 0 && dgamma != nullptr) {
    for (int k = tid; k < P * C; k += 256) {
      const int pk = k / C, c = k % C;
      dgamma[k] = f2bf(sums[(2 * pk + 1) * C + c]);
      dbeta[k] = f2bf(sums[(2 * pk) * C + c]);
    }
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(r0 + rows_per_block, M);
  float k1[8], k2[8], k3[8], sh[8];
  {
    float g[8], b[8];
    unpack8(*(const uint4*)(gamma + (int64_t)p * C + 8 * ch), g);
    if (relu == 2) unpack8(*(const uint4*)(beta + (int64_t)p * C + 8 * ch), b);
    const float invM = 1.f / (float)M;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = 8 * ch + e;
      const float mean = stat[(2 * p) * C + c], rstd = stat[(2 * p + 1) * C + c];
      const float A = sums[(2 * p) * C + c] * invM, B = sums[(2 * p + 1) * C + c] * invM;
      k1[e] = g[e] * rstd;                 // = the forward's scale sc
      k2[e] = -k1[e] * rstd * B;
      k3[e] = -k1[e] * A - k2[e] * mean;
      sh[e] = relu == 2 ? b[e] - mean * k1[e] : 0.f;
    }
  }
  const int64_t base = (int64_t)p * M * C + 8 * ch;
  for (int64_t r = r0 + rg; r < r1; r += UNROLL * ng) {
    uint4 xr[UNROLL], yr[UNROLL], dr[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t ru = r + u * ng;
      const int64_t o = base + (ru < r1 ? ru : r) * C;
      xr[u] = *(const uint4*)(x + o);
      dr[u] = *(const uint4*)(dy + o);
      if (relu == 1) yr[u] = *(const uint4*)(y + o);
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t ru = r + u * ng;
      if (ru >= r1) break;
      float xv[8], yv[8], dv[8], o[8];
      unpack8(xr[u], xv);
      unpack8(dr[u], dv);
      if (relu == 1) unpack8(yr[u], yv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool off = relu == 1 ? yv[e] <= 0.f
                                   : (relu == 2 && xv[e] * k1[e] + sh[e] + 0.f <= 0.f);
        const float dz = off ? 0.f : dv[e];
        o[e] = k1[e] * dz + k2[e] * xv[e] + k3[e];
        dv[e] = dz;
      }
      const int64_t off = base + ru * C;
      *(uint4*)(dx + off) = pack8(o);
      if (dres) *(uint4*)(dres + off) = pack8(dv);
    }
  }
}

// rows per block (per trial): ~MOPT_BN_BLOCKS blocks over the population, a multiple of the row
// groups times the unroll (ResNet-20 at 1024 / 2048 / 4096 / 8192 blocks: 5.56 / 5.49 / 5.46 /
// 5.46 ms per step, profiles/r5/conv_blocks)
#ifndef MOPT_BN_BLOCKS
#define MOPT_BN_BLOCKS 4096
#endif
inline int reduce_rows(int P, int64_t M, int C) {
  const int ng = UNROLL * (256 / (C / 8));
  int64_t rpb = ((int64_t)P * M + MOPT_BN_BLOCKS - 1) / MOPT_BN_BLOCKS;
  rpb = (rpb + ng - 1) / ng * ng;
  return (int)(rpb > ng ? rpb : ng);
}

inline bool bn_shape_ok(int C) { return C >= 8 && C <= 512 && C % 8 == 0 && ((C / 8) & (C / 8 - 1)) == 0; }

}  // namespace

extern "C" {

// x [P][M][C] -> y; stat [P][2][C] (mean, rstd) out; running [P][2][C] in/out; sums scratch
// (or, sums_ready, the batch sums of x and x^2 already accumulated by the convolution).
// res_c > 0: res is the block input at twice the resolution with res_c channels and the
// residual is its option-A shortcut (stride-2 subsample, zero channels >= res_c); the output
// side is 1 << res_ohl.
int mopt_bn_fwd(const void* x, const void* gamma, const void* beta, const void* res, void* y,
                void* stat, void* running, void* sums, int P, int64_t M, int C, float eps,
                float momentum, int train, int relu, int sums_ready, int res_c, int res_ohl,
                void* stream) {
  if (!bn_shape_ok(C)) return 1;
  hipStream_t st = (hipStream_t)stream;
  if (train && !sums_ready) {  // else the producing convolution's epilogue summed x, x^2
    (void)hipMemsetAsync(sums, 0, sizeof(float) * 2 * P * C, st);
    const int rpb = reduce_rows(P, M, C);
    hipLaunchKernelGGL(bn_reduce_kernel<false>, dim3((unsigned)((M + rpb - 1) / rpb), P),
                       dim3(256), 0, st, (const bf16_t*)x, nullptr, nullptr, nullptr, nullptr,
                       nullptr, (float*)sums, M, C, rpb, 0);
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((P * C + 255) / 256), dim3(256), 0, st,
                     (const float*)sums, (float*)stat, (float*)running, P, C, M, eps, momentum,
                     train);
  if (y == nullptr) return (int)hipGetLastError();  // statistics only: the consumer applies
  const int rpa = reduce_rows(P, M, C);
  hipLaunchKernelGGL(bn_apply_kernel, dim3((unsigned)((M + rpa - 1) / rpa), P), dim3(256), 0, st,
                     (const bf16_t*)x, (const float*)stat, (const bf16_t*)gamma,
                     (const bf16_t*)beta, (const bf16_t*)res, (bf16_t*)y, M, C, rpa, relu, res_c,
                     res_ohl);
  return (int)hipGetLastError();
}

// sums [P][2][C] out: (sum dz, sum dz * xhat) = (dbeta, dgamma) in f32 (zeroed here unless
// sums_zeroed = 1; sums_zeroed = 2: already accumulated by the producing data gradient's
// epilogue, mopt_dconv_dgrad_bnsums -- no reduction pass); dgamma / dbeta (bf16 [P][C], may be
// null): the gradients written directly.
// relu: 0 none, 1 mask from y, 2 mask recomputed from x with gamma / beta (y may be null)
int mopt_bn_bwd(const void* x, const void* y, const void* dy, const void* stat, const void* gamma,
                const void* beta, void* dx, void* dres, void* sums, void* dgamma, void* dbeta,
                int P, int64_t M, int C, int relu, int sums_zeroed, void* stream) {
  if (relu < 0 || relu > 2 || (relu == 1 && y == nullptr) || (relu == 2 && beta == nullptr))
    return (int)hipErrorInvalidValue;
  if (!bn_shape_ok(C)) return 1;
  hipStream_t st = (hipStream_t)stream;
  if (!sums_zeroed) (void)hipMemsetAsync(sums, 0, sizeof(float) * 2 * P * C, st);
  const int rpb = reduce_rows(P, M, C);
  if (sums_zeroed != 2)
    hipLaunchKernelGGL(bn_reduce_kernel<true>, dim3((unsigned)((M + rpb - 1) / rpb), P),
                       dim3(256), 0, st, (const bf16_t*)x, (const bf16_t*)y, (const bf16_t*)dy,
                       (const float*)stat, (const bf16_t*)gamma, (const bf16_t*)beta,
                       (float*)sums, M, C, rpb, relu);
#ifndef MOPT_BN_APPLY_RT
#define MOPT_BN_APPLY_RT 0
#endif
  auto apply = MOPT_BN_APPLY_RT ? bn_bwd_apply_kernel<-1>
               : relu == 0      ? bn_bwd_apply_kernel<0>
               : relu == 1      ? bn_bwd_apply_kernel<1>
                                : bn_bwd_apply_kernel<2>;
  hipLaunchKernelGGL(apply, dim3((unsigned)((M + rpb - 1) / rpb), P), dim3(256), 0,
                     st, (const bf16_t*)x, (const bf16_t*)y, (const bf16_t*)dy, (const float*)stat,
                     (const float*)sums, (const bf16_t*)gamma, (const bf16_t*)beta, (bf16_t*)dx,
                     (bf16_t*)dres,
                     (bf16_t*)dgamma, (bf16_t*)dbeta, M, C, P, rpb, relu);
  return (int)hipGetLastError();
}

}  // extern "C"
