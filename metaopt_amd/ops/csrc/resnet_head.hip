// Classifier head of the population ResNet (BASELINE config 3; SURVEY §2.3 assigns K1/K4 to it):
// global average pool -> linear C -> NP (NP = 16 padded logits, the first ncls real) -> softmax
// cross-entropy, forward AND backward in one pass over the features:
//
//   head_kernel   grid (B / IMG, P), 256 threads, IMG = 16 images of one trial per workgroup:
//                 pooled features [IMG][C] (f32 sums of the bf16 NHWC activations), logits from
//                 the trial's W [C][NP] / b [NP] (staged in LDS as f32), per-image loss /
//                 correct, dlogits = (softmax - onehot) * scale, and (training) the input
//                 gradient dh[i][pixel][c] = (dlogits W^T)[i][c] / HW written straight to HBM,
//                 plus this workgroup's partial dW = feat^T dlogits and db = colsum(dlogits)
//   head_reduce   grid P: sums the partials of a trial in a fixed order (deterministic, no
//                 atomics) and writes the bf16 dW / db into the flat gradient buffer, the loss
//                 sum and #correct into the statistics
//
// Replaces the aten mean / hipBLASLt baddbmm / cross_entropy chain (about a dozen framework
// kernels per step, profiles/r3/resnet20_bn_into_conv_kernel_stats.csv).  Activations are
// x[(p * B + b)][pixel][c] bf16 (C a multiple of 8, <= 64), 16-byte accesses throughout.
#include "common.h"

using namespace mopt;

namespace {

constexpr int IMG = 16;   // images per workgroup
constexpr int NP = 16;    // padded logits
constexpr int CMAX = 64;  // channels

__device__ __forceinline__ void unpack8h(const uint4& u, float (&f)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[2 * e] = bf2f(w[e] & 0xFFFF);
    f[2 * e + 1] = bf2f(w[e] >> 16);
  }
}

// reductions over the 16 lanes of an image (lanes n = 0..15 of one 16-lane group)
__device__ __forceinline__ float max16(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float sum16(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// partial record per (trial, image block): dW [C][NP], db [NP], loss, correct
__host__ __device__ constexpr int rec_floats(int C) { return C * NP + NP + 2; }

// BN: x is the last block's pre-BatchNorm conv output and the features are formed on the fly,
// h = relu(BN(x) + res) rounded to bf16 exactly as bn_apply_kernel / the conv staging round it;
// the backward writes dz = dh relu'(h) (the BatchNorm's input gradient before its apply pass and
// the block's shortcut gradient) and adds the BatchNorm's reductions (sum dz, sum dz xhat) into
// bsums [P][2][C] -- the block output is never written.  dz is constant over an image's pixels
// up to the mask, so those sums are g * count and g * rstd * sum(x - mean) over the pixels the
// mask keeps, gathered while pooling (the mask bits wait in LDS for the dz stores).
struct HeadBN {
  const bf16_t* res;
  float* stat;           // [P][2][C] mean, rstd (written here when xsums is given)
  const bf16_t* gamma;
  const bf16_t* beta;
  float* bsums;          // [P][2][C], accumulated
  // finalize in the head (bn_finalize_kernel's arithmetic): the forward batch sums of x, the
  // running statistics the trial's first workgroup updates; xsums == nullptr: stat is given
  const float* xsums;
  float* running;
  float Mf, Mm1f, eps, momentum;
};

// pixels per iteration of a thread's BatchNorm pooling loop (loads in flight: 2 x HEAD_PX)
#ifndef MOPT_HEAD_PX
#define MOPT_HEAD_PX 8
#endif
constexpr int HEAD_PX = MOPT_HEAD_PX;
static_assert(HEAD_PX == 4 || HEAD_PX == 8, "mask words hold 4 pixels");

template <bool BN>
__global__ __launch_bounds__(256) void head_kernel(const bf16_t* __restrict__ x,
                                                   const bf16_t* __restrict__ W,
                                                   const bf16_t* __restrict__ bias,
                                                   const int64_t* __restrict__ labels, int B,
                                                   int HW, int C, int ncls, float scale,
                                                   int train, float* __restrict__ part,
                                                   bf16_t* __restrict__ dx, HeadBN bn) {
  __shared__ float Ws[CMAX][NP + 1];
  // BN: one mask word per 4 pixels of a thread (host: HW / nph <= 32, HW % (HEAD_PX nph) == 0)
  __shared__ uint32_t mbits[BN ? 8 * 256 : 1];
  __shared__ float bred[BN ? 2 : 1][CMAX];
  __shared__ float bs[NP];
  __shared__ float feat[IMG][CMAX + 1];
  __shared__ float dl[IMG][NP + 1];
  __shared__ float fsum[IMG][2][CMAX];   // the two pixel phases of the pooling sums
  __shared__ float lrec[IMG][2];
  const int p = blockIdx.y, blk = blockIdx.x, nblk = gridDim.x;
  const int tid = threadIdx.x;
  const int cc = C >> 3;                 // 16-byte chunks per pixel (<= 8)
  // ---- stage the trial's W [C][NP] and b as f32 ----
  const bf16_t* Wp = W + (int64_t)p * C * NP;
  for (int e = tid; e < C * NP; e += 256) Ws[e / NP][e % NP] = bf2f(Wp[e]);
  if (tid < NP) bs[tid] = bf2f(bias[(int64_t)p * NP + tid]);

  // ---- pooled features: thread = (image i, pixel phase ph, channel chunk ch) ----
  const int i = tid >> 4, sub = tid & 15;
  const int ch = sub % cc, ph = sub / cc, nph = 16 / cc;   // C = 64: 8 chunks, 2 phases
  const int64_t row = (int64_t)p * B + (int64_t)blk * IMG + i;
  const bf16_t* xi = x + row * HW * C;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float cnt[8], sxm[8], rs[8];   // BN: pixels the mask keeps, sum of (x - mean) over them, rstd
  if constexpr (BN) {
    float sc[8], sh[8], mu[8];
    {
      float gm[8], bt[8];
      unpack8h(*(const uint4*)(bn.gamma + (int64_t)p * C + 8 * ch), gm);
      unpack8h(*(const uint4*)(bn.beta + (int64_t)p * C + 8 * ch), bt);
      const bool fin_w = bn.xsums != nullptr && blk == 0 && i == 0 && ph == 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = 8 * ch + e;
        if (bn.xsums != nullptr) {
          mu[e] = bn.xsums[(2 * p) * C + c] / bn.Mf;
          const float var = fmaxf(bn.xsums[(2 * p + 1) * C + c] / bn.Mf - mu[e] * mu[e], 0.f);
          rs[e] = rsqrtf(var + bn.eps);
          if (fin_w) {
            float* rm = bn.running + (int64_t)p * 2 * C;
            rm[c] = (1.f - bn.momentum) * rm[c] + bn.momentum * mu[e];
            rm[C + c] = (1.f - bn.momentum) * rm[C + c] + bn.momentum * var * bn.Mf / bn.Mm1f;
            bn.stat[(2 * p) * C + c] = mu[e];
            bn.stat[(2 * p + 1) * C + c] = rs[e];
          }
        } else {
          mu[e] = bn.stat[(2 * p) * C + c];
          rs[e] = bn.stat[(2 * p + 1) * C + c];
        }
        sc[e] = gm[e] * rs[e];
        sh[e] = bt[e] - mu[e] * sc[e];
        cnt[e] = 0.f;
        sxm[e] = 0.f;
      }
    }
    for (int e = tid; e < 2 * CMAX; e += 256) bred[e / CMAX][e % CMAX] = 0.f;
    const bf16_t* ri = bn.res + row * HW * C;
    int j = 0;
    for (int px = ph; px < HW; px += HEAD_PX * nph) {
      uint4 u[HEAD_PX], r[HEAD_PX];
#pragma unroll
      for (int k = 0; k < HEAD_PX; ++k) {
        u[k] = *(const uint4*)(xi + (int64_t)(px + k * nph) * C + 8 * ch);
        r[k] = *(const uint4*)(ri + (int64_t)(px + k * nph) * C + 8 * ch);
      }
#pragma unroll
      for (int w = 0; w < HEAD_PX / 4; ++w, ++j) {
        uint32_t mw = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float f[8], rv[8];
          unpack8h(u[4 * w + k], f);
          unpack8h(r[4 * w + k], rv);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float hb = bf2f(f2bf(fmaxf(fmaf(f[e], sc[e], sh[e]) + rv[e], 0.f)));
            acc[e] += hb;
            if (hb > 0.f) {
              mw |= 1u << (8 * k + e);
              cnt[e] += 1.f;
              sxm[e] += f[e] - mu[e];
            }
          }
        }
        mbits[j * 256 + tid] = mw;
      }
    }
  } else if (ph < nph) {
    int px = ph;
    for (; px + 3 * nph < HW; px += 4 * nph) {        // four 16-byte loads in flight
      uint4 u[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) u[k] = *(const uint4*)(xi + (int64_t)(px + k * nph) * C + 8 * ch);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float f[8];
        unpack8h(u[k], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += f[e];
      }
    }
    for (; px < HW; px += nph) {
      float f[8];
      unpack8h(*(const uint4*)(xi + (int64_t)px * C + 8 * ch), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += f[e];
    }
  }
  // phases combined in a fixed order (two phases at C = 64; up to 16 at C = 8)
  if (ph < 2) {
#pragma unroll
    for (int e = 0; e < 8; ++e) fsum[i][ph][8 * ch + e] = acc[e];
  }
  __syncthreads();
  if (nph > 2) {   // small C: fold the extra phases into phase 0, in order
    for (int q = 2; q < nph; ++q) {
      if (ph == q) {
#pragma unroll
        for (int e = 0; e < 8; ++e) fsum[i][0][8 * ch + e] += acc[e];
      }
      __syncthreads();
    }
  }
  const float inv_hw = 1.f / (float)HW;
  for (int e = sub; e < C; e += 16)
    feat[i][e] = (fsum[i][0][e] + (nph > 1 ? fsum[i][1][e] : 0.f)) * inv_hw;
  __syncthreads();

  // ---- logits, softmax cross-entropy: thread = (image i, logit n) ----
  const int n = sub;
  float z = bs[n];
  for (int c = 0; c < C; ++c) z += feat[i][c] * Ws[c][n];
  const bool valid = n < ncls;
  const float zm = valid ? z : -INFINITY;
  const float m = max16(zm);
  const float ex = valid ? __expf(z - m) : 0.f;
  const float s = sum16(ex);
  const int y = (int)labels[row];
  const bool y_ok = MOPT_IN_RANGE(y, ncls, "resnet head label");
  const float zy = sum16(n == y ? z : 0.f);
  // argmax with the lowest index among equal maxima (torch.argmax)
  int am = (valid && zm == m) ? n : NP;
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) am = min(am, __shfl_xor(am, o, 64));
  if (n == 0) {
    lrec[i][0] = y_ok ? m + __logf(s) - zy : 0.f;
    lrec[i][1] = (am == y) ? 1.f : 0.f;
  }
  dl[i][n] = (valid && y_ok) ? (ex / s - (n == y ? 1.f : 0.f)) * scale : 0.f;
  __syncthreads();

  float* rec = part + ((int64_t)p * nblk + blk) * rec_floats(C);
  if (tid == 0) {   // fixed summation order over the block's images
    float l = 0.f, k = 0.f;
    for (int j = 0; j < IMG; ++j) {
      l += lrec[j][0];
      k += lrec[j][1];
    }
    rec[C * NP + NP] = l;
    rec[C * NP + NP + 1] = k;
  }
  if (!train) return;

  // ---- partial dW [C][NP] = feat^T dl, db = colsum dl (this block's images) ----
  for (int e = tid; e < C * NP; e += 256) {
    const int c = e / NP, nn = e % NP;
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < IMG; ++j) a += feat[j][c] * dl[j][nn];
    rec[e] = a;
  }
  if (tid < NP) {
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < IMG; ++j) a += dl[j][tid];
    rec[C * NP + tid] = a;
  }

  // ---- dx[i][pixel][c] = (dl W^T)[i][c] / HW for every pixel of the image ----
  if (ph < nph) {
    float g[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = 8 * ch + e;
      float a = 0.f;
#pragma unroll
      for (int nn = 0; nn < NP; ++nn) a += dl[i][nn] * Ws[c][nn];
      g[e] = a * inv_hw;
    }
    const uint4 v = make_uint4(pack2bf(g[0], g[1]), pack2bf(g[2], g[3]), pack2bf(g[4], g[5]),
                               pack2bf(g[6], g[7]));
    bf16_t* di = dx + row * HW * C + 8 * ch;
    if constexpr (BN) {
      // dz = the stored (bf16) gradient where the mask keeps the pixel; the BatchNorm sums
      float gb[8];
      unpack8h(v, gb);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        atomicAdd(&bred[0][8 * ch + e], gb[e] * cnt[e]);
        atomicAdd(&bred[1][8 * ch + e], gb[e] * rs[e] * sxm[e]);
      }
      const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
      int j = 0;
      for (int px = ph; px < HW; px += 4 * nph, ++j) {
        const uint32_t mw = mbits[j * 256 + tid];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t m = mw >> (8 * k);
          uint32_t o[4];
#pragma unroll
          for (int q = 0; q < 4; ++q)
            o[q] = (vw[q] & ((m >> (2 * q)) & 1u ? 0xFFFFu : 0u)) |
                   (vw[q] & ((m >> (2 * q + 1)) & 1u ? 0xFFFF0000u : 0u));
          *(uint4*)(di + (int64_t)(px + k * nph) * C) = make_uint4(o[0], o[1], o[2], o[3]);
        }
      }
    } else {
      for (int px = ph; px < HW; px += nph) *(uint4*)(di + (int64_t)px * C) = v;
    }
  }
  if constexpr (BN) {
    __syncthreads();
    for (int e = tid; e < 2 * C; e += 256)
      atomicAdd(bn.bsums + (int64_t)p * 2 * C + e, bred[e / C][e % C]);
  }
}

// one workgroup per trial: fixed-order sums of the partial records -> bf16 dW / db (straight
// into the flat gradient buffer), loss sum and #correct
__global__ __launch_bounds__(256) void head_reduce_kernel(const float* __restrict__ part,
                                                          int nblk, int C, int train,
                                                          bf16_t* __restrict__ dW,
                                                          bf16_t* __restrict__ db,
                                                          float* __restrict__ loss,
                                                          float* __restrict__ correct) {
  const int p = blockIdx.x, tid = threadIdx.x;
  const int R = rec_floats(C);
  const float* base = part + (int64_t)p * nblk * R;
  const int lo = train ? 0 : C * NP + NP;
  for (int e = lo + tid; e < R; e += 256) {
    float a = 0.f;
    for (int k = 0; k < nblk; ++k) a += base[(int64_t)k * R + e];
    if (e < C * NP) dW[(int64_t)p * C * NP + e] = f2bf(a);
    else if (e < C * NP + NP) db[(int64_t)p * NP + e - C * NP] = f2bf(a);
    else if (e == C * NP + NP) loss[p] = a;
    else correct[p] = a;
  }
}

}  // namespace

extern "C" {

// x [P*B][HW][C] bf16, W [P][C][16] bf16, b [P][16] bf16, labels [P*B] int64.  train: also
// dx [P*B][HW][C] bf16, dW / db (bf16, overwritten).  part: f32 scratch of
// P * (B / 16) * (16 C + 18) floats.  loss / correct: f32 [P].
int mopt_resnet_head(const void* x, const void* W, const void* b, const void* labels, int P,
                     int B, int HW, int C, int ncls, float scale, int train, void* part, void* dx,
                     void* dW, void* db, void* loss, void* correct, void* stream) {
  if (P <= 0 || B <= 0 || B % IMG || C % 8 || C < 8 || C > CMAX || ncls < 1 || ncls > NP ||
      HW < 1 || (train && (dx == nullptr || dW == nullptr || db == nullptr)))
    return (int)hipErrorInvalidValue;
  const hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(head_kernel<false>, dim3(B / IMG, P), dim3(256), 0, st, (const bf16_t*)x,
                     (const bf16_t*)W, (const bf16_t*)b, (const int64_t*)labels, B, HW, C, ncls,
                     scale, train, (float*)part, (bf16_t*)dx, HeadBN{});
  hipLaunchKernelGGL(head_reduce_kernel, dim3(P), dim3(256), 0, st, (const float*)part, B / IMG,
                     C, train, (bf16_t*)dW, (bf16_t*)db, (float*)loss, (float*)correct);
  return (int)hipGetLastError();
}

// Training head over the last block's output relu(BN(x) + res) formed on the fly (x, res
// [P*B][HW][C] bf16; stat [P][2][C] mean / rstd; gamma / beta bf16 [P][C]): dz (the BatchNorm's
// masked input gradient, [P*B][HW][C] bf16) instead of dh, and (sum dz, sum dz xhat) added into
// bsums [P][2][C] (zeroed by the caller).  hipErrorNotSupported (801) for shapes it does not take.
int mopt_resnet_head_bn(const void* x, const void* res, void* stat, const void* gamma,
                        const void* beta, const void* W, const void* b, const void* labels, int P,
                        int B, int HW, int C, int ncls, float scale, void* part, void* dz,
                        void* dW, void* db, void* loss, void* correct, void* bsums,
                        const void* xsums, void* running, int64_t M, float eps, float momentum,
                        void* stream) {
  if (P <= 0 || B <= 0 || B % IMG || C % 8 || C < 8 || C > CMAX || ncls < 1 || ncls > NP ||
      HW < 1 || !x || !res || !stat || !gamma || !beta || !dz || !dW || !db || !bsums ||
      (xsums && !running))
    return (int)hipErrorInvalidValue;
  const int cc = C / 8, nph = 16 / cc;
  if (16 % cc || HW % (HEAD_PX * nph) || HW / (4 * nph) > 8) return (int)hipErrorNotSupported;
  const hipStream_t st = (hipStream_t)stream;
  const HeadBN bn{(const bf16_t*)res, (float*)stat, (const bf16_t*)gamma, (const bf16_t*)beta,
                  (float*)bsums, (const float*)xsums, (float*)running, (float)M,
                  (float)(M > 1 ? M - 1 : 1), eps, momentum};
  hipLaunchKernelGGL(head_kernel<true>, dim3(B / IMG, P), dim3(256), 0, st, (const bf16_t*)x,
                     (const bf16_t*)W, (const bf16_t*)b, (const int64_t*)labels, B, HW, C, ncls,
                     scale, 1, (float*)part, (bf16_t*)dz, bn);
  hipLaunchKernelGGL(head_reduce_kernel, dim3(P), dim3(256), 0, st, (const float*)part, B / IMG,
                     C, 1, (bf16_t*)dW, (bf16_t*)db, (float*)loss, (float*)correct);
  return (int)hipGetLastError();
}

int mopt_resnet_head_part_floats(int P, int B, int C) { return P * (B / IMG) * rec_floats(C); }

}  // extern "C"

MOPT_VIOLATIONS_READER(resnet_head)
