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
  const int chunks = (int)min((int64_t)1024, (n / 4 + 255) / 256);
  hipLaunchKernelGGL(hyper_dot_kernel, dim3(chunks, P), dim3(256), 0, (hipStream_t)stream,
                     (const float*)a, (const float*)b0, (const float*)b1, (float*)out, n);
  return (int)hipGetLastError();
}

}  // extern "C"
