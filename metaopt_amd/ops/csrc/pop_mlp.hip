// Population-batched MLP training kernels for MI355X (gfx950 / CDNA4).
//
// A "population" is P independent trials (hyper-parameter configurations) trained side by side.
// Every trial owns its own weights, optimizer state, hyper-parameters and RNG stream; the widths
// are ragged (per-trial), so every launch walks a work list of (trial-layer, tile) items built on
// the host (metaopt_amd/ops/population.py) instead of a dense [P, ...] grid.  Dims are padded to
// multiples of 64 with zero weights, which is exact: a zero-padded unit never receives gradient.
//
// Kernels (north-star inventory K1/K2/K4/K5/K6/K7):
//   mlp_fwd_kernel     Y = dropout(relu(X W^T + b))            K1 + K7, bf16 MFMA, f32 accumulate
//   mlp_fwd_ce_kernel  logits = X W^T + b; fused softmax-CE      K1 + K4 (loss, #correct, dLogits)
//   mlp_bwd_opt_kernel one pass over W per step that computes    K2 + K5/K6
//                        dX = dZ W      (-> masked dZ of the layer below),
//                        dW = dZ^T X, db = colsum(dZ)
//                      and applies the per-trial SGD-momentum / AdamW update in the epilogue, so
//                      dW never touches HBM.  W is read once (f32 master) for both dX and the update.
//   mlp_bwd0_fwd_kernel the first layer's backward + update of step t fused with its forward of
//                      step t + 1 (one pass over W0 instead of two; bit-identical results)
//
// Memory-bound by design: per parameter and step the population moves 2 B (forward) + 18 B (fused
// backward + SGD; 14 B with the bf16 momentum buffer of kSGD16) through HBM; the MFMA work
// (6 * B FLOP per parameter) is a small fraction of the chip's bf16 rate at B = 128.  See
// profiles/ for measured bandwidth.
#include "common.h"

using namespace mopt;

extern "C" {

// Work lists are [n][2] int32 (trial-layer, tile), position 8 i + x = the i-th item of XCD x
// (workgroups are dealt to the XCDs round-robin), built and cost-balanced on the host
// (metaopt_amd/ops/population.py _xcd_schedule); (-1, *) entries are padding.
//
// One (trial, layer) of the population; 64 bytes, mirrored by metaopt_amd/ops/population.py.
struct MlpTL {
  int32_t K;       // padded input features (multiple of 64)
  int32_t N;       // padded output features (multiple of 64)
  int32_t trial;   // population slot (index into the hyper-parameter table)
  int32_t n_real;  // real outputs (classes of the CE layer, the member's width otherwise)
  int64_t w_off;   // W [N][K] (k-strip-major, see w_row_stride): offset into the parameters
  int64_t b_off;   // bias [N]: offset into the f32 master / optimizer buffers
  int64_t x_off;   // layer input  [rows][K] bf16: offset into the x buffer of the launch
  int64_t y_off;   // layer output [rows][N] bf16: offset into act (forward) / grad (backward)
  int64_t gx_off;  // dZ of the layer below [rows][K] bf16 in grad (backward), -1 if none
  int32_t rows;    // rows this trial uses in the launch (its batch size; <= the launch's rows):
                   // row blocks at or past it are skipped, the loss is normalised by it
  int32_t k_real;  // real inputs: W[:, k] is zero for k >= k_real (padding to K)
};

// Dead padding (round 6): K and N are padded to multiples of 64, but W[n][k] (and its optimizer
// state) is zero forever for n >= n_real or k >= k_real -- its gradient is X[:, k]^T dZ[:, n] with
// a zero column on either side, and zero stays zero under SGD / AdamW.  The kernels skip the HBM
// traffic of those elements at 8-element granularity (live extents rounded up to 8: whole 16-byte
// lanes, and 8-row groups = whole wave-instructions of the state layout): no load, no store.  A
// skipped load leaves its register stale (never a select on a load: hipcc turns that into a
// branch and a vmcnt(0) per element), so every value derived from a dead element is either
// discarded (the skipped stores), multiplied by an exact zero, or zeroed explicitly where it
// reaches memory (the W^T image of dX, the forward's dead output columns).  12 % of the headline's
// state bytes are such padding (loguniform(64, 1024) widths padded to 64).
#ifndef MOPT_DEAD_SKIP
#define MOPT_DEAD_SKIP 1   // 0: a build that moves the padding like live data (A/B baseline)
#endif
__device__ __forceinline__ int live8(int n) { return MOPT_DEAD_SKIP ? (n + 7) & ~7 : 1 << 30; }

// One (member, layer) to initialise; 48 bytes, mirrored by metaopt_amd/ops/population.py.
struct InitDesc {
  int64_t w_off, b_off;   // W [N][K] and bias [N] offsets (elements)
  int32_t K, N;           // padded dims
  int32_t k_real, n_real; // real dims (outside them: zeros)
  uint32_t seed;          // member seed
  int32_t layer;
  float bound;            // U(-bound, bound), bound = 1/sqrt(k_real) computed on the host
  int32_t pad;
};

// Per-trial hyper-parameters; 32 bytes.  SGD: b1 = momentum.  AdamW: b1, b2, eps, t = step count.
struct TrialHP {
  float lr, b1, wd, drop, b2, eps;
  uint32_t seed, t;
};

}  // extern "C"

namespace {

constexpr int BM = 128;  // rows (batch) per workgroup
constexpr int BN = 64;   // output features per forward tile / per backward chunk
constexpr int BK = 64;   // reduction step of the forward, width of a backward k-strip
// LDS tiles: bf16 rows padded to 72 elements (144 B), f32 dW staging rows padded to 68.  (The
// row-XOR swizzle of common.h, conflict-free by scripts/lds_banks.py, was measured slower in
// round 3: its address math spilled the backward -- profiles/round3.md "MLP kernels: A/B".)
constexpr int TS = kLdsStride;
#define TOFF(r, c) ((r) * TS + (c))
// Forward tiles: rows of 80 elements (160 B = 10 16-byte slots, 2 mod 4), so the 16 rows of a
// fragment read (ds_read_b128) hit 16 distinct slots -- conflict-free where 72 costs 4 extra
// cycles per read (scripts/lds_banks.py "pad80"); the backward keeps 72 (its transposed reads
// and dZ copy-out conflict more at 80).
constexpr int TSF = 80;
#define TOFFF(r, c) ((r) * TSF + (c))
#define FOFF(r, c) ((r) * (BN + 4) + (c))

// Weight layout in HBM: k-strip-major [K/64][N][64] -- W[n][k] at (k / 64) N 64 + n 64 + k % 64,
// so the backward's k-strip is one contiguous N x 128-B block and every 64 x 64 tile the forward
// or the backward touches is 8 KB contiguous (a micro-benchmark of the backward's three-array
// read-modify-write by 64 x 64 tiles measured 5.4 TB/s contiguous vs 4.65 TB/s with 128-B rows
// K * 2 bytes apart: scripts/dev/tile_layout_bench.*).  The bias and the optimizer state share
// the layout; metaopt_amd/ops/population.py views the weights row-major through it.
__device__ __forceinline__ int w_row_stride(int) { return BK; }
__device__ __forceinline__ int w_kstep(int N) { return N; }
// stored index e -> (n, k)
__device__ __forceinline__ void w_coords(int64_t e, int N, int, int& n, int& k) {
  const int64_t strip = e / ((int64_t)N * BK), r = e - strip * (int64_t)N * BK;
  n = (int)(r / BK);
  k = (int)(strip * BK + (r % BK));
}

// kStoreStats: one row block per trial -- store the trial's loss / #correct instead of
// accumulating atomically into zeroed counters (saves the per-step zero-fill launch).
// kCountStep: advance the trial's step counter hp.t (the hidden layers of the same step read
// hp.t + 1; the backward, launched after, reads the new value) -- saves the per-step increment
// launch.
// kNarrow (loss layer, <= 16 classes): the layer's N is padded to one 64-wide tile but only its
// first 16 rows of W (and columns of dZ) can be non-zero -- the kernels skip the other 48 rows'
// weight / optimizer traffic and MFMAs (the 10-class head moved 4x its real bytes per step).
enum FwdFlags { kRelu = 1, kDropout = 2, kWriteGrad = 4, kStoreStats = 8, kCountStep = 16,
                kNarrowCE = 32 };
enum BwdFlags { kHasDx = 1, kInDropout = 2, kUpdateBias = 4, kNarrow = 8 };
constexpr int kNarrowRows = 16;
// kSGD16: SGD with the momentum buffer stored as bf16 (RNE after every update; the update uses
// the rounded value) -- 4 bytes per parameter and step less HBM traffic than kSGD.
enum Opt { kSGD = 0, kAdamW = 1, kSGD16 = 2 };

// ----------------------------------------------------------------------------------------------
// Forward GEMM core: acc[i][j] = X[row0 + 32*wave + 16i .., :] . W[n0 + 16j .., :]^T over all K.
// Register-staged pipelining (T14), NSET (2) K-steps deep: the register sets rotate over an
// unrolled loop of NSET K-steps (no register is copied; the counted vmcnt wait at each step
// leaves the other sets' loads in flight).  With one step of look-ahead a K = 1024 strip was a
// chain of 16 exposed HBM round trips (~2 TB/s); two steps reach ~3 TB/s.  Three sets (3 or 4
// workgroups per CU) measured no faster (profiles/r4/kbench_fwd_v*.log): the forward is bound by
// its LDS traffic (6 B of fragment reads per weight byte at 128 rows), not by look-ahead.  Loads
// past the last K-step re-read the last tile (clamped address) instead of branching, so no
// control flow sits around a load.
// ----------------------------------------------------------------------------------------------
// (the two register sets are plain scalars behind a macro: held in a struct passed by reference
//  they were demoted to scratch; 32-bit element offsets keep both sets within the 128 VGPRs of
//  4 waves per SIMD -- 64-bit ones needed 132.  The pipelined loop below measured 658 -> 650 us
//  per 256-member step, profiles/round4.md.)
#define MOPT_FWD_LOAD(x0, x1, x2, x3, w0, w1, k)        \
  do {                                                  \
    const uint32_t kk_ = (uint32_t)(k), kw_ = kk_ * (uint32_t)WKS; \
    x0 = *(const uint4*)(X + (uint32_t)(g0 + kk_));     \
    x1 = *(const uint4*)(X + (uint32_t)(g1 + kk_));     \
    x2 = *(const uint4*)(X + (uint32_t)(g2 + kk_));     \
    x3 = *(const uint4*)(X + (uint32_t)(g3 + kk_));     \
    if (WROWS >= 32 || w_live) w0 = *(const uint4*)(W + (uint32_t)(gw0 + kw_)); \
    if (TN >= 64 && WROWS >= 64) w1 = *(const uint4*)(W + (uint32_t)(gw1 + kw_)); \
    if (TN >= 128) {                                    \
      w1##b = *(const uint4*)(W + (uint32_t)(gw2 + kw_)); \
      w1##c = *(const uint4*)(W + (uint32_t)(gw3 + kw_)); \
    }                                                   \
  } while (0)
#define MOPT_FWD_STORE(x0, x1, x2, x3, w0, w1) \
  do {                                         \
    *(uint4*)as0 = x0;                         \
    *(uint4*)as1 = x1;                         \
    *(uint4*)as2 = x2;                         \
    *(uint4*)as3 = x3;                         \
    *(uint4*)bs0 = w0;                         \
    if (TN >= 64) *(uint4*)bs1 = w1;           \
    if (TN >= 128) {                           \
      *(uint4*)bs2 = w1##b;                    \
      *(uint4*)bs3 = w1##c;                    \
    }                                          \
  } while (0)

// TN: output features per tile (64, or 32 for twice the workgroups: the hidden layers' launches
// hold ~1.5 workgroups per slot of the chip at 64, a tail of half-empty CUs)
// WROWS: rows of the W tile that can be non-zero (TN, or kNarrowRows for a narrow loss layer:
// only those B fragments are read and multiplied)
template <int TN, int WROWS = TN>
__device__ __forceinline__ void fwd_step(const bf16_t* As, const bf16_t* Bs, int wave, int li,
                                         int g, f32x4 (&acc)[2][TN / 16]) {
  constexpr int NJ = (WROWS < TN ? WROWS : TN) / 16;
#pragma unroll
  for (int ks = 0; ks < BK / 32; ++ks) {
    bf16x8 a[2], b[NJ];
#pragma unroll
    for (int i = 0; i < 2; ++i) a[i] = lds_frag(As + TOFFF(wave * 32 + i * 16 + li, ks * 32 + g * 8));
#pragma unroll
    for (int j = 0; j < NJ; ++j) b[j] = lds_frag(Bs + TOFFF(j * 16 + li, ks * 32 + g * 8));
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
  }
}

// W: the tile's first row (w_off + n0 * w_row_stride(K)); N: rows of the layer's weight matrix
// nlive / klive: the tile's live W rows (from its first) and K's live extent, multiples of 8
// (live8): dead W rows / k-chunks are not loaded (stale registers -- the dead k meet exact-zero X
// columns, the dead rows' outputs are zeroed by the caller's epilogue)
template <int TN, int NSET = 2, int WROWS = TN>
__device__ __forceinline__ void fwd_gemm(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                         int K, int N, bf16_t* As, bf16_t* Bs,
                                         f32x4 (&acc)[2][TN / 16], int nlive, int klive) {
  static_assert(WROWS == TN || WROWS == kNarrowRows, "narrow tiles keep 16 W rows");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TN / 16; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int c0 = tid, c1 = tid + 256, c2 = tid + 512, c3 = tid + 768;
  const int g0 = (c0 >> 3) * K + (c0 & 7) * 8, g1 = (c1 >> 3) * K + (c1 & 7) * 8;
  const int g2 = (c2 >> 3) * K + (c2 & 7) * 8, g3 = (c3 >> 3) * K + (c3 & 7) * 8;
  // W rows are WRS apart; a K-step of kk columns moves kk * WKS elements (w_row_stride / w_kstep)
  const int WRS = w_row_stride(K), WKS = w_kstep(N);
  // dead W rows (>= nlive, 8-row groups): their loads re-read the tile's first row (always
  // live) -- an L2 hit instead of HBM traffic, with no branch around the pipelined loads (a
  // predicated load here became a branch + vmcnt(0) and spilled); the caller's epilogue zeroes
  // those output columns
  const int gw0 = ((c0 >> 3) < nlive ? (c0 >> 3) * WRS : 0) + (c0 & 7) * 8;
  const int gw1 = ((c1 >> 3) < nlive ? (c1 >> 3) * WRS : 0) + (c1 & 7) * 8;
  const int gw2 = (c2 >> 3) * WRS + (c2 & 7) * 8, gw3 = (c3 >> 3) * WRS + (c3 & 7) * 8;
  bf16_t* as0 = As + TOFFF(c0 >> 3, (c0 & 7) * 8);
  bf16_t* as1 = As + TOFFF(c1 >> 3, (c1 & 7) * 8);
  bf16_t* as2 = As + TOFFF(c2 >> 3, (c2 & 7) * 8);
  bf16_t* as3 = As + TOFFF(c3 >> 3, (c3 & 7) * 8);
  bf16_t* bs0 = Bs + TOFFF(c0 >> 3, (c0 & 7) * 8);
  bf16_t* bs1 = Bs + TOFFF(c1 >> 3, (c1 & 7) * 8);
  bf16_t* bs2 = Bs + TOFFF(c2 >> 3, (c2 & 7) * 8);
  bf16_t* bs3 = Bs + TOFFF(c3 >> 3, (c3 & 7) * 8);
  const int klast = K - BK;
  // narrow: thread t stages W row t / 8 -- rows >= WROWS stay zero (never loaded)
  const bool w_live = (c0 >> 3) < WROWS;
  (void)klive;   // dead k-chunks meet exact-zero X columns: loaded as they are
  uint4 p0, p1, p2, p3, pw0{}, pw1{}, pw1b{}, pw1c{};  // K-steps 0, 3, 6, ...
  uint4 q0, q1, q2, q3, qw0{}, qw1{}, qw1b{}, qw1c{};  // K-steps 1, 4, 7, ...
  uint4 r0, r1, r2, r3, rw0{}, rw1{}, rw1b{}, rw1c{};  // K-steps 2, 5, 8, ...
  MOPT_FWD_LOAD(p0, p1, p2, p3, pw0, pw1, 0);
  MOPT_FWD_LOAD(q0, q1, q2, q3, qw0, qw1, min(BK, klast));
  if (NSET == 3) MOPT_FWD_LOAD(r0, r1, r2, r3, rw0, rw1, min(2 * BK, klast));
  // K-step from set S: its tile to LDS, then S fetches the tile NSET steps ahead
#define MOPT_FWD_KSTEP(S, KNEXT)                                         \
  MOPT_FWD_STORE(S##0, S##1, S##2, S##3, S##w0, S##w1);                  \
  __syncthreads();                                                       \
  MOPT_FWD_LOAD(S##0, S##1, S##2, S##3, S##w0, S##w1, min(KNEXT, klast)); \
  fwd_step<TN, WROWS>(As, Bs, wave, li, g, acc);                         \
  __syncthreads();
  if (NSET == 3) {
    int k0 = 0;
    for (; k0 + 3 * BK <= K; k0 += 3 * BK) {
      MOPT_FWD_KSTEP(p, k0 + 3 * BK)
      MOPT_FWD_KSTEP(q, k0 + 4 * BK)
      MOPT_FWD_KSTEP(r, k0 + 5 * BK)
    }
    if (k0 < K) {
      MOPT_FWD_KSTEP(p, k0 + 3 * BK)
    }
    if (k0 + BK < K) {
      MOPT_FWD_KSTEP(q, k0 + 4 * BK)
    }
  } else {
    // whole pairs of K-steps, then the odd last one: no exit between the two steps, so the
    // loop body is one block -- with a mid-body exit hipcc sank the p refill past the exit
    // branch (it is dead on that path) into the next iteration, one step before its use
    // instead of two, and the waits at the q store then drained every load in flight
    int k0 = 0;
    for (; k0 + 2 * BK <= K; k0 += 2 * BK) {
      MOPT_FWD_KSTEP(p, k0 + 2 * BK)
      MOPT_FWD_KSTEP(q, k0 + 3 * BK)
    }
    if (k0 < K) {
      MOPT_FWD_KSTEP(p, k0 + 2 * BK)
    }
  }
#undef MOPT_FWD_KSTEP
}
#undef MOPT_FWD_LOAD
#undef MOPT_FWD_STORE

// (Measured and rejected, round 4: X fragments loaded straight from global memory into the
// A operands with only W staged through LDS -- 40 instead of 72 KB of LDS traffic per K-step --
// ran fwd0 at 58.7 vs 48.5 us: each lane's 16-byte row pieces coalesce into 64-byte segments;
// profiles/round4.md.)
// (Measured and rejected: an LDS-free variant loading every MFMA fragment -- 16 bytes of one
// row of X or W per lane -- straight from global memory ran the forward 2.5x slower than the
// LDS-staged tiles above; profiles/README.md.)
template <int TN, int NSET = 2, int WROWS = TN>
__device__ __forceinline__ void fwd_core(const bf16_t* X, const bf16_t* W, int K, int N,
                                         bf16_t* As, bf16_t* Bs, f32x4 (&acc)[2][TN / 16],
                                         int nlive, int klive) {
  fwd_gemm<TN, NSET, WROWS>(X, W, K, N, As, Bs, acc, nlive, klive);
}

// Y[rows, n0:n0+TN] = dropout(relu(X W^T + b)) for one (trial-layer, n-tile, 128-row block).
// NSET register sets of look-ahead, WAVES waves per SIMD (workgroups per CU)
template <int TN, int NSET, int WAVES>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WAVES))) void mlp_fwd_kernel(const MlpTL* __restrict__ tls,
                                                      const int2* __restrict__ work, int n_work,
                                                      const bf16_t* __restrict__ xb,
                                                      const bf16_t* __restrict__ plo,
                                                      const bf16_t* __restrict__ p16,
                                                      bf16_t* __restrict__ act,
                                                      const TrialHP* __restrict__ hp,
                                                      uint32_t step, int layer, int flags) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[(BM + TN) * TSF];
  bf16_t* As = smem;
  bf16_t* Bs = smem + BM * TSF;
  const int2 wi = work[blockIdx.x];   // XCD-balanced order built on the host (_xcd_schedule)
  if (wi.x < 0) return;                // padding: a no-op workgroup
  const MlpTL tl = tls[wi.x];
  const int K = tl.K, N = tl.N, n0 = wi.y * TN, row0 = blockIdx.y * BM;
  if (row0 >= tl.rows) return;           // a smaller batch than the launch's: uniform exit
  const bf16_t* X = xb + tl.x_off + (size_t)row0 * K;
  const bf16_t* W = p16 + tl.w_off + (size_t)n0 * w_row_stride(K);

  f32x4 acc[2][TN / 16];
  const int nlive = live8(tl.n_real) - n0;      // live output columns of this tile (may be <= 0)
  fwd_core<TN, NSET>(X, W, K, N, As, Bs, acc, nlive, live8(tl.k_real));

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, g = lane >> 4;
  const bf16_t* bias_hi = p16 + tl.b_off + n0;
  const bf16_t* bias_lo = plo + tl.b_off + n0;
  const TrialHP h = hp[tl.trial];
  const bool drop = (flags & kDropout) && h.drop > 0.f;
  const float inv_keep = drop ? 1.f / (1.f - h.drop) : 1.f;
  // The dropout stream is keyed by the trial's own step count (h.t), so a trial draws the same
  // masks whichever slot it occupies and whenever it joined the population.
  const uint32_t key = rng_key(h.seed, (uint32_t)layer, h.t + step);
  bf16_t* Cs = smem;  // reuse As (the last K-step ended with a barrier)
#pragma unroll
  for (int j = 0; j < TN / 16; ++j) {
    const int col = j * 16 + li;
    const float bj = join_hilo(bias_hi[col], bias_lo[col]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wave * 32 + i * 16 + g * 4 + r;
        float v = col < nlive ? acc[i][j][r] + bj : 0.f;   // dead columns: exact zeros
        if (flags & kRelu) v = fmaxf(v, 0.f);
        if (drop) {
          const uint32_t idx = (uint32_t)((row0 + row) * N + n0 + col);
          v = rng_uniform(key, idx) >= h.drop ? v * inv_keep : 0.f;
        }
        Cs[TOFFF(row, col)] = f2bf(v);
      }
  }
  __syncthreads();
  bf16_t* Y = act + tl.y_off + (size_t)row0 * N + n0;
  constexpr int CPR = TN / 8;   // 16-byte chunks per row
#pragma unroll
  for (int i = 0; i < TN / 16; ++i) {
    const int c = tid + 256 * i, r = c / CPR, ch = c % CPR;
    *(uint4*)(Y + (size_t)r * N + ch * 8) = *(const uint4*)(Cs + TOFFF(r, ch * 8));
  }
}

// (Round 5: a W-direct forward -- 128-column tiles, each wave loading its W B-fragments straight
// from HBM into registers, only X staged through LDS: 1 + 4 instead of 3 + 6 LDS bytes per
// weight byte -- trained bit for bit like this kernel but ran the headline 781.8 vs 789.6
// trials/s on one stream and 824 vs 827 on four (800 workgroups against 768 slots: a near-empty
// second wave); removed, profiles/round5.md.)

// Output layer: logits = X W^T + b (N padded to 64 >= classes), fused softmax cross-entropy.
// Writes dLogits = (softmax - onehot) * inv_b as bf16 (training) and accumulates the per-trial
// loss sum and #correct (atomic, one add per wave).  NARROW (<= 16 classes): W rows 16..63 are
// neither read nor multiplied, and only the first 16 dLogits columns are written (the narrow
// backward reads no others).
template <bool NARROW>
__global__ __launch_bounds__(256) void mlp_fwd_ce_kernel(const MlpTL* __restrict__ tls,
                                                         const int2* __restrict__ work, int n_work,
                                                         const bf16_t* __restrict__ xb,
                                                         const bf16_t* __restrict__ plo,
                                                         const bf16_t* __restrict__ p16,
                                                         const int32_t* __restrict__ labels,
                                                         bf16_t* __restrict__ grad,
                                                         float* __restrict__ loss_out,
                                                         float* __restrict__ correct_out,
                                                         TrialHP* __restrict__ hp, float inv_b,
                                                         int flags) {
  constexpr int CS = BN + 1;  // f32 logits row stride
  constexpr int kSmemBytes = BM * CS * 4 > (BM + BN) * TSF * 2 ? BM * CS * 4 : (BM + BN) * TSF * 2;
  __shared__ __attribute__((aligned(16))) char smem_raw[kSmemBytes];
  bf16_t* As = (bf16_t*)smem_raw;
  bf16_t* Bs = As + BM * TSF;
  float* Ls = (float*)smem_raw;

  const int2 wi = work[blockIdx.x];   // XCD-balanced order built on the host (_xcd_schedule)
  if (wi.x < 0) return;                // padding: a no-op workgroup
  const MlpTL tl = tls[wi.x];
  const int K = tl.K, N = tl.N, row0 = blockIdx.y * BM, C = tl.n_real;
  if (row0 >= tl.rows) return;           // a smaller batch than the launch's: uniform exit
  // inv_b <= 0: the mean over the trial's own batch (per-trial batch sizes)
  const float ib = inv_b > 0.f ? inv_b : 1.f / (float)tl.rows;
  const bf16_t* X = xb + tl.x_off + (size_t)row0 * K;
  const bf16_t* W = p16 + tl.w_off;

  f32x4 acc[2][4];
  // only the C real classes' logits are used below: the dead rows' stale sums are never read
  fwd_core<64, 2, NARROW ? kNarrowRows : 64>(X, W, K, N, As, Bs, acc, live8(C),
                                             live8(tl.k_real));

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, g = lane >> 4;
  const bf16_t* bias_hi = p16 + tl.b_off;
  const bf16_t* bias_lo = plo + tl.b_off;
  constexpr int NJ = NARROW ? kNarrowRows / 16 : 4;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = j * 16 + li;
    const float bj = join_hilo(bias_hi[col], bias_lo[col]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) Ls[(wave * 32 + i * 16 + g * 4 + r) * CS + col] = acc[i][j][r] + bj;
  }
  __syncthreads();

  float loss = 0.f, corr = 0.f;
  if (tid < BM) {
    const float* z = Ls + tid * CS;
    int y = labels[row0 + tid];
    const bool y_ok = MOPT_IN_RANGE(y, C, "mlp cross-entropy label");
    if (!y_ok) y = -1;                // checked build: no loss, no one-hot
    float m = -INFINITY;
    int am = 0;
    for (int c = 0; c < C; ++c)
      if (z[c] > m) { m = z[c]; am = c; }
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += __expf(z[c] - m);
    const float lse = m + __logf(s);
    loss = y_ok ? lse - z[y] : 0.f;
    corr = (am == y) ? 1.f : 0.f;
    if (flags & kWriteGrad) {
      const float rs = 1.f / s;
      bf16_t* dz = grad + tl.y_off + (size_t)(row0 + tid) * N;
#pragma unroll
      for (int ch = 0; ch < (NARROW ? kNarrowRows : BN) / 8; ++ch) {
        uint32_t w4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c0 = ch * 8 + 2 * e, c1 = c0 + 1;
          const float g0 = c0 < C ? (__expf(z[c0] - m) * rs - (c0 == y ? 1.f : 0.f)) * ib : 0.f;
          const float g1 = c1 < C ? (__expf(z[c1] - m) * rs - (c1 == y ? 1.f : 0.f)) * ib : 0.f;
          w4[e] = pack2bf(g0, g1);
        }
        *(uint4*)(dz + ch * 8) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
      }
    }
  }
  loss = wave_sum(loss);
  corr = wave_sum(corr);
  if ((flags & kCountStep) && blockIdx.y == 0 && tid == 0) hp[tl.trial].t += 1u;
  if (flags & kStoreStats) {
    __shared__ float red[2][2];
    if (lane == 0 && wave < 2) {
      red[wave][0] = loss;
      red[wave][1] = corr;
    }
    __syncthreads();
    if (tid == 0) {
      loss_out[tl.trial] = red[0][0] + red[1][0];
      correct_out[tl.trial] = red[0][1] + red[1][1];
    }
  } else if (lane == 0 && wave < 2) {
    atomicAdd(loss_out + tl.trial, loss);
    atomicAdd(correct_out + tl.trial, corr);
  }
}

// Backward tiles (X strip, dZ chunk, W^T image): unpadded 128-byte rows, 16-byte chunk c of row r
// stored at c ^ swz128(r) (common.h).  Conflict-free for every per-chunk LDS access of the backward -- the dZ
// A fragments (ds_read_b128), the three transposed ds_read_b64_tr_b16 reads and the staging
// stores (scripts/lds_banks.py, searched over all XOR maps of the row bits) -- where the rows
// padded to 72 elements cost 2 extra cycles per transposed read and 4 per fragment read
// (1.66 conflict cycles per LDS instruction measured, profiles/r4/pmc_mlp_r4aa.txt).
#define BOFF(r, c) soff((r), (c))   // common.h swz128 (BK = 64-element rows)

// The per-parameter optimizer update of four consecutive parameters, shared by every kernel that
// updates weights (mlp_bwd_opt_kernel, mlp_bwd0_fwd_kernel).  Explicit fmaf: the two kernels
// must round identically, and hipcc's fp-contraction of the written-out expressions differed
// between them (1-ulp momentum differences with weight decay, round 5).
template <int OPT>
__device__ __forceinline__ void opt_update4(f32x4& wv, f32x4& mv, f32x4& vv, const f32x4& gv,
                                            const TrialHP& h, float c1, float c2) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float gr = gv[r];
    if (OPT == kSGD || OPT == kSGD16) {
      const float gg = fmaf(h.wd, wv[r], gr);
      float mn = fmaf(h.b1, mv[r], gg);
      if (OPT == kSGD16) mn = bf2f(f2bf(mn));   // the stored (rounded) momentum drives W
      mv[r] = mn;
      wv[r] = fmaf(-h.lr, mn, wv[r]);
    } else {
      wv[r] = wv[r] * (1.f - h.lr * h.wd);
      mv[r] = fmaf(h.b1, mv[r], (1.f - h.b1) * gr);
      vv[r] = fmaf(h.b2, vv[r], ((1.f - h.b2) * gr) * gr);
      wv[r] = wv[r] - (c1 * mv[r]) / fmaf(sqrtf(vv[r]), c2, h.eps);
    }
  }
}

// the bias update (no weight decay), shared the same way
template <int OPT>
__device__ __forceinline__ void bias_update(float& bw, float& mb, float& vb, float gb,
                                            const TrialHP& h, float c1, float c2) {
  if (OPT == kSGD || OPT == kSGD16) {
    mb = fmaf(h.b1, mb, gb);
    if (OPT == kSGD16) mb = bf2f(f2bf(mb));
    bw = fmaf(-h.lr, mb, bw);
  } else {
    mb = fmaf(h.b1, mb, (1.f - h.b1) * gb);
    vb = fmaf(h.b2, vb, ((1.f - h.b2) * gb) * gb);
    bw = bw - (c1 * mb) / fmaf(sqrtf(vb), c2, h.eps);
  }
}

// ----------------------------------------------------------------------------------------------
// Fused backward + optimizer for one (trial-layer, 64-wide k-strip of W).  The workgroup holds the
// X strip X[:, k0:k0+64] in LDS for the whole pass and walks W[:, k0:k0+64] in 64-row chunks:
//   dX[:, strip] += dZ[:, chunk] . W[chunk, strip]        (A: dZ row reads, B: W^T by tr-reads)
//   dW^T[strip, chunk] = X[:, strip]^T . dZ[:, chunk]     (A: X tr-reads held in VGPRs, B: dZ tr)
//   W, M (, V) <- optimizer(W, M, dW)                       (dW^T C-layout = 4 consecutive k/lane)
// One LDS image per operand serves both row reads and ds_read_b64_tr_b16 transposed reads.
// ----------------------------------------------------------------------------------------------
//
// Batches of R = rows / 128 row blocks (per-trial batch sizes): MODE 0 is the one-block kernel
// above; MODE 2 computes only dX of row block 1 + blockIdx.y (W hi and dZ read, no update) and is
// launched first; MODE 1 then does the fused pass -- dX of row block 0, dW summed over all R
// blocks (the X strip and dZ chunk of blocks 1.. restaged through the same LDS tiles), the
// update, the bias over all rows.  Trials with fewer rows than the launch skip the extra blocks.
//
// LDS: the f32 dW staging tile aliases the dZ chunk tile (one more barrier per chunk), 47 KB per
// workgroup instead of 64.5 KB, so three workgroups fit a CU's 160 KB; the variant without the
// prefetch register set (<= 168 VGPRs) then runs 3 waves per SIMD.  The prefetch variant needs
// more VGPRs and stays at 2.  Optimizer state moves 16 bytes per lane (2 rows x 8 k per thread;
// -1.7 % step time against 8-byte accesses, profiles/round3.md).
constexpr int bwd_waves(int opt, bool pf, int mode) {
  // AdamW and the multi-row-block pass spill at 168 VGPRs: they keep 2 waves per SIMD
  return (!pf && opt != kAdamW && mode != 1) ? 3 : 2;
}
template <int OPT, bool PF, int MODE, bool NARROW = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(
    bwd_waves(OPT, PF, MODE), bwd_waves(OPT, PF, MODE)))) void mlp_bwd_opt_kernel(const MlpTL* __restrict__ tls,
                                                          const int2* __restrict__ work, int n_work,
                                                          const bf16_t* __restrict__ xb,
                                                          bf16_t* __restrict__ grad,
                                                          bf16_t* __restrict__ plo,
                                                          bf16_t* __restrict__ p16,
                                                          float* __restrict__ m32,
                                                          float* __restrict__ v32,
                                                          const TrialHP* __restrict__ hp, int flags) {
  constexpr int DS = BN + 4;  // f32 row stride bound of the dW staging tile (FOFF)
  // the dZ tile's region also holds the f32 dW staging tile (aliased, one more barrier per chunk)
  constexpr int ZE = (BM * BK > 2 * BN * DS) ? BM * BK : 2 * BN * DS;
  __shared__ __attribute__((aligned(16)))
      bf16_t smem[BM * BK + ZE + BN * BK + 2 * 4 * BN];
  bf16_t* Xs = smem;
  bf16_t* Zs = smem + BM * BK;
  bf16_t* Ws = smem + BM * BK + ZE;
  float* red = (float*)(smem + BM * BK + ZE + BN * BK);  // [4][64] bias partial sums
  // [64 n][DS] dW of the current chunk
  float* Dw = (float*)Zs;

  const int2 wi = work[blockIdx.x];   // XCD-balanced order built on the host (_xcd_schedule)
  if (wi.x < 0) return;                // padding: a no-op workgroup
  const MlpTL tl = tls[wi.x];
  const int K = tl.K, N = tl.N, k0 = wi.y * BK;
  const int R = MODE == 0 ? 1 : (int)(tl.rows / BM);       // the trial's row blocks
  const int rbx = MODE == 2 ? 1 + (int)blockIdx.y : 0;      // this launch's row block
  if (MODE == 2 && rbx >= R) return;                         // uniform per workgroup
  const bf16_t* X = xb + tl.x_off + (size_t)rbx * BM * K;
  const bf16_t* dZ = grad + tl.y_off + (size_t)rbx * BM * N;
  bf16_t* WLO = plo + tl.w_off;                      // master = (hi, lo) pairs, see common.h
  float* M32 = m32 + tl.w_off;                       // kSGD / kAdamW
  bf16_t* M16 = (bf16_t*)m32 + tl.w_off;             // kSGD16
  float* V32 = v32 + tl.w_off;  // AdamW only
  bf16_t* W16 = p16 + tl.w_off;
  const TrialHP h = hp[tl.trial];
  const bool has_dx = flags & kHasDx;
  const bool do_bias = (flags & kUpdateBias) && wi.y == 0 && MODE != 2;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4, q = li >> 2, pp = li & 3;
  const int wk = wave >> 1, wn = wave & 1;
  // NARROW (the loss layer, N = 64 of which <= 16 rows live): thread t owns W rows t / 8 and
  // t / 8 + 32 -- only threads < 128 (rows < 16) move weights / optimizer state, and only the
  // first 16 dZ columns (8-column chunks 0, 1) are read; the rest stay zero in registers
  const bool st_live = !NARROW || tid < 8 * kNarrowRows;
  const bool z_live = !NARROW || (tid & 7) < kNarrowRows / 8;
  // dead padding (see live8): this thread's state rows nc + tid / 8 (+ 32) are live below nl
  // (whole 128-byte rows of the strip: wave-uniform; dead k-chunks are moved like live ones --
  // skipping them made the row's stores partial lines, which the memory side fills by a read,
  // measured slower: profiles/round6.md)
  const int nl = live8(tl.n_real);
  const int rlo = tid >> 3;
  constexpr bool k_ok = true;

  // Optimizer constants (uniform per workgroup).
  float c1 = 1.f, c2 = 1.f;
  if (OPT == kAdamW) {
    const float t = (float)h.t;
    c1 = h.lr / (1.f - __powf(h.b1, t));           // lr / bias_correction1
    c2 = 1.f / sqrtf(1.f - __powf(h.b2, t));        // 1 / sqrt(bias_correction2)
  }

  // Stage X[:, k0:k0+64] (128 x 64 bf16).
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i, r = c >> 3, ch = c & 7;
    *(uint4*)(Xs + BOFF(r, ch * 8)) = *(const uint4*)(X + (size_t)r * K + k0 + ch * 8);
  }
  __syncthreads();

  f32x4 dx[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) dx[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Chunk operands (dZ rows, W hi/lo, momentum) live in named registers, never in arrays
  // captured by a lambda (see fwd_gemm).  PF (prefetch): the operands of chunk c+1 are loaded
  // into a second register set right after chunk c's operands reached LDS / f32 registers, so
  // every workgroup keeps two chunks of HBM traffic in flight across its MFMA + update phase
  // (without it the loads of a chunk are exposed at the top of the chunk and only the second
  // workgroup per CU hides them).
  const int zo0 = (tid >> 3) * N + (tid & 7) * 8, zo1 = ((tid + 256) >> 3) * N + (tid & 7) * 8;
  const int zo2 = ((tid + 512) >> 3) * N + (tid & 7) * 8, zo3 = ((tid + 768) >> 3) * N + (tid & 7) * 8;
  bf16_t* zs0 = Zs + BOFF(tid >> 3, (tid & 7) * 8);     // rows +32 i keep the swizzle
  const int WRS = w_row_stride(K);
  // Optimizer-state layout: thread -> rows 32 i + tid / 8 (i < 2), 8 consecutive k at 8 (tid % 8):
  // every W / M (/ V) access is 16 bytes per lane and a wave-instruction moves 8 rows x 128 B
  // (1 KB) -- half the memory instructions of the 8-byte layout below.
  const size_t wo = (size_t)k0 * w_kstep(N) + (size_t)(tid >> 3) * WRS + 8 * (tid & 7);
  uint4 cz0{}, cz1{}, cz2{}, cz3{}, nz0{}, nz1{}, nz2{}, nz3{};
  f32x4 cm0{}, cm1{}, cm2{}, cm3{}, cv0{}, cv1{}, cv2{}, cv3{};   // rows i = 0,1: (lo4, hi4)
  f32x4 nm0{}, nm1{}, nm2{}, nm3{}, nv0{}, nv1{}, nv2{}, nv3{};
  uint4 cwh0{}, cwh1{}, cwl0{}, cwl1{}, nwh0{}, nwh1{}, nwl0{}, nwl1{};  // master hi, lo halves
  uint4 ch0{}, ch1{}, nh0{}, nh1{};                                    // kSGD16 momentum
#define MOPT_BWD_LOAD(NC, P)                                                                     \
  {                                                                                              \
    const bf16_t* zc_ = dZ + (NC);                                                               \
    if (z_live) {                                                                                \
    P##z0 = *(const uint4*)(zc_ + zo0);                                                          \
    P##z1 = *(const uint4*)(zc_ + zo1);                                                          \
    P##z2 = *(const uint4*)(zc_ + zo2);                                                          \
    P##z3 = *(const uint4*)(zc_ + zo3);                                                          \
    }                                                                                            \
    const size_t ob = (size_t)(NC) * WRS + wo;                                                   \
    if (NARROW) {                                                                                \
    if (st_live) {                                                                               \
    P##wh0 = *(const uint4*)(W16 + ob);                                                          \
    if (MODE != 2) {                                                                             \
    P##wl0 = *(const uint4*)(WLO + ob);                                                          \
    if (OPT == kSGD16) {                                                                         \
      P##h0 = *(const uint4*)(M16 + ob);                                                         \
    } else {                                                                                     \
      P##m0 = *(const f32x4*)(M32 + ob);                                                         \
      P##m1 = *(const f32x4*)(M32 + ob + 4);                                                     \
    }                                                                                            \
    if (OPT == kAdamW) {                                                                         \
      P##v0 = *(const f32x4*)(V32 + ob);                                                         \
      P##v1 = *(const f32x4*)(V32 + ob + 4);                                                     \
    }                                                                                            \
    }                                                                                            \
    }                                                                                            \
    } else {                                                                                     \
    /* dead rows / k-chunks re-read the chunk's first row at the strip's first k (both always  \
       live): L2 hits instead of HBM traffic, no branch around the loads */                     \
    const size_t od_ = (size_t)(NC) * WRS + (size_t)k0 * w_kstep(N);                             \
    const size_t o0_ = k_ok && (NC) + rlo < nl ? ob : od_;                                       \
    const size_t o1_ = k_ok && (NC) + rlo + 32 < nl ? ob + 32 * WRS : od_;                       \
    P##wh0 = *(const uint4*)(W16 + o0_);                                                         \
    P##wh1 = *(const uint4*)(W16 + o1_);                                                         \
    if (MODE != 2) {                                                                             \
    P##wl0 = *(const uint4*)(WLO + o0_);                                                         \
    P##wl1 = *(const uint4*)(WLO + o1_);                                                         \
    if (OPT == kSGD16) {                                                                         \
      P##h0 = *(const uint4*)(M16 + o0_);                                                        \
      P##h1 = *(const uint4*)(M16 + o1_);                                                        \
    } else {                                                                                     \
      P##m0 = *(const f32x4*)(M32 + o0_);                                                        \
      P##m1 = *(const f32x4*)(M32 + o0_ + 4);                                                    \
      P##m2 = *(const f32x4*)(M32 + o1_);                                                        \
      P##m3 = *(const f32x4*)(M32 + o1_ + 4);                                                    \
    }                                                                                            \
    if (OPT == kAdamW) {                                                                         \
      P##v0 = *(const f32x4*)(V32 + o0_);                                                        \
      P##v1 = *(const f32x4*)(V32 + o0_ + 4);                                                    \
      P##v2 = *(const f32x4*)(V32 + o1_);                                                        \
      P##v3 = *(const f32x4*)(V32 + o1_ + 4);                                                    \
    }                                                                                            \
    }                                                                                            \
    }                                                                                            \
  }
#define MOPT_BWD_ADVANCE()                                                                       \
  {                                                                                              \
    cz0 = nz0; cz1 = nz1; cz2 = nz2; cz3 = nz3;                                                  \
    cwh0 = nwh0; cwh1 = nwh1; cwl0 = nwl0; cwl1 = nwl1;                                          \
    if (OPT == kSGD16) { ch0 = nh0; ch1 = nh1; }                                                 \
    else { cm0 = nm0; cm1 = nm1; cm2 = nm2; cm3 = nm3; }                                         \
    if (OPT == kAdamW) { cv0 = nv0; cv1 = nv1; cv2 = nv2; cv3 = nv3; }                           \
  }
  MOPT_BWD_LOAD(0, c)
  for (int nc = 0; nc < N; nc += BN) {
    // ---- this chunk's operands -> LDS (dZ row-major; W^T image as bf16 for the dX MFMAs) ----
    *(uint4*)(zs0) = cz0;
    *(uint4*)(zs0 + 32 * BK) = cz1;
    *(uint4*)(zs0 + 64 * BK) = cz2;
    *(uint4*)(zs0 + 96 * BK) = cz3;
    // per thread: 2 rows x 8 k = 4 groups of 4 (row 0 k 0-3, row 0 k 4-7, row 1 k 0-3, 4-7)
    if (OPT == kSGD16) {
      cm0 = bf4_to_f32(make_uint2(ch0.x, ch0.y)); cm1 = bf4_to_f32(make_uint2(ch0.z, ch0.w));
      cm2 = bf4_to_f32(make_uint2(ch1.x, ch1.y)); cm3 = bf4_to_f32(make_uint2(ch1.z, ch1.w));
    }
    const f32x4 w[4] = {join4(make_uint2(cwh0.x, cwh0.y), make_uint2(cwl0.x, cwl0.y)),
                        join4(make_uint2(cwh0.z, cwh0.w), make_uint2(cwl0.z, cwl0.w)),
                        join4(make_uint2(cwh1.x, cwh1.y), make_uint2(cwl1.x, cwl1.y)),
                        join4(make_uint2(cwh1.z, cwh1.w), make_uint2(cwl1.z, cwl1.w))};
    const f32x4 m[4] = {cm0, cm1, cm2, cm3};
    f32x4 v[4];
    if (OPT == kAdamW) {
      v[0] = cv0; v[1] = cv1; v[2] = cv2; v[3] = cv3;
    }
    // this chunk's live state rows (dead ones: stale registers, zeroed in the W^T image)
    const bool lv[2] = {NARROW ? st_live : k_ok && nc + rlo < nl,
                        NARROW ? false : k_ok && nc + rlo + 32 < nl};
    const uint4 wh[2] = {cwh0, cwh1};
    const bool more = nc + BN < N;
    if (PF && more) MOPT_BWD_LOAD(nc + BN, n)
    if (has_dx) {   // the bf16 working copy (hi) is the dX operand, as in the forward
#pragma unroll
      for (int i = 0; i < 2; ++i)
        *(uint4*)(Ws + BOFF(32 * i + (tid >> 3), 8 * (tid & 7))) =
            lv[i] ? wh[i] : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();

    // ---- dX[:, strip] += dZ[:, chunk] . W[chunk, strip] ----
    if (has_dx) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 a[2], b[4];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = lds_frag(Zs + BOFF(32 * wave + 16 * i + li, 32 * s + 8 * g));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const s16x4 lo = lds_tr4(Ws + BOFF(32 * s + 8 * g + q, 16 * j + 4 * pp));
          const s16x4 hi = lds_tr4(Ws + BOFF(32 * s + 8 * g + 4 + q, 16 * j + 4 * pp));
          b[j] = cat_frag(lo, hi);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) dx[i][j] = mfma16(a[i], b[j], dx[i][j]);
      }
    }

    // ---- dW^T[strip, chunk] = X^T dZ, summed over the trial's row blocks ----
    f32x4 dw[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < 2; ++u) dw[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
#define MOPT_BWD_DW()                                                                            \
  _Pragma("unroll") for (int s = 0; s < 4; ++s) {                                                \
    bf16x8 xa[2], bz[2];                                                                         \
    _Pragma("unroll") for (int t = 0; t < 2; ++t) {                                              \
      const int c0 = 32 * wk + 16 * t + 4 * pp;                                                  \
      const s16x4 lo = lds_tr4(Xs + BOFF(32 * s + 8 * g + q, c0));                               \
      const s16x4 hi = lds_tr4(Xs + BOFF(32 * s + 8 * g + 4 + q, c0));                           \
      xa[t] = cat_frag(lo, hi);                                                                  \
    }                                                                                            \
    _Pragma("unroll") for (int u = 0; u < 2; ++u) {                                              \
      const int c0 = 32 * wn + 16 * u + 4 * pp;                                                  \
      const s16x4 lo = lds_tr4(Zs + BOFF(32 * s + 8 * g + q, c0));                               \
      const s16x4 hi = lds_tr4(Zs + BOFF(32 * s + 8 * g + 4 + q, c0));                           \
      bz[u] = cat_frag(lo, hi);                                                                  \
    }                                                                                            \
    _Pragma("unroll") for (int t = 0; t < 2; ++t)                                                \
      _Pragma("unroll") for (int u = 0; u < 2; ++u) dw[t][u] = mfma16(xa[t], bz[u], dw[t][u]);  \
  }
    // bias partial sums of this thread's (row quarter, column), over every row block
    const int bcol = tid & 63, bpart = tid >> 6;
    float bsum = 0.f;
    if (MODE != 2) {
      MOPT_BWD_DW()
      if (do_bias)
        for (int r = bpart * 32; r < bpart * 32 + 32; ++r) bsum += bf2f(Zs[BOFF(r, bcol)]);
      if (MODE == 1) {
        for (int rb = 1; rb < R; ++rb) {      // R is uniform per workgroup
          __syncthreads();                    // every wave is done with the previous block
          const bf16_t* Xr = X + (size_t)rb * BM * K + k0;
          const bf16_t* Zr = dZ + (size_t)rb * BM * N + nc;
          // (NARROW: the CE kernel wrote dZ columns < kNarrowRows only -- the dead columns are
          // zero-filled here, never read: the narrow backward touches no other dZ bytes)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int c = tid + 256 * i, r = c >> 3, ch = c & 7;
            *(uint4*)(Xs + BOFF(r, ch * 8)) = *(const uint4*)(Xr + (size_t)r * K + ch * 8);
            *(uint4*)(Zs + BOFF(r, ch * 8)) =
                z_live ? *(const uint4*)(Zr + (size_t)r * N + ch * 8) : make_uint4(0, 0, 0, 0);
          }
          __syncthreads();
          MOPT_BWD_DW()
          if (do_bias)
            for (int r = bpart * 32; r < bpart * 32 + 32; ++r) bsum += bf2f(Zs[BOFF(r, bcol)]);
        }
        if (R > 1) {                          // row block 0's X strip back (next chunk, dX mask)
          __syncthreads();
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int c = tid + 256 * i, r = c >> 3, ch = c & 7;
            *(uint4*)(Xs + BOFF(r, ch * 8)) = *(const uint4*)(X + (size_t)r * K + k0 + ch * 8);
          }
        }
      }
    }
#undef MOPT_BWD_DW

    // ---- optimizer epilogue: dW^T C-fragments (register r of dw[t][u] = dW[n][k + r]) are
    //      restaged through LDS into the row-contiguous layout of W/M (/V) ----
    if (MODE != 2) {
    __syncthreads();   // every wave is done reading Zs (dX, dW, bias): Dw aliases it
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < 2; ++u)
        *(f32x4*)(Dw + FOFF(32 * wn + 16 * u + li, 32 * wk + 16 * t + 4 * g)) = dw[t][u];
    __syncthreads();
    uint2 ph{}, pl{}, pm{};   // the row's first group, stored with the second
#pragma unroll
    for (int i = 0; i < (NARROW ? 2 : 4); ++i) {
      if (NARROW && !st_live) break;   // rows >= 16 of a narrow loss layer: zero, untouched
      if (!lv[i >> 1]) continue;       // dead padding: nothing loaded, nothing stored
      // group i: row 32 (i / 2) + tid / 8, k 8 (tid % 8) + 4 (i % 2) .. + 3
      const int gr = 32 * (i >> 1) + (tid >> 3), gk = 8 * (tid & 7) + 4 * (i & 1);
      const f32x4 gv = *(const f32x4*)(Dw + FOFF(gr, gk));
      const size_t o = (size_t)nc * WRS + wo + (size_t)(32 * (i >> 1)) * WRS + 4 * (i & 1);
      f32x4 wv = w[i], mv = m[i], vv;
      if (OPT == kAdamW) vv = v[i];
      opt_update4<OPT>(wv, mv, vv, gv, h, c1, c2);
      uint2 nh, nl;
      split4(wv, nh, nl);
      // the two groups of a row (k 0-3, 4-7) leave as one 16-byte store per array
      if ((i & 1) == 0) {
        ph = nh;
        pl = nl;
        pm = f32_to_bf4(mv);
      } else {
        *(uint4*)(W16 + o - 4) = make_uint4(ph.x, ph.y, nh.x, nh.y);
        *(uint4*)(WLO + o - 4) = make_uint4(pl.x, pl.y, nl.x, nl.y);
        if (OPT == kSGD16) {
          const uint2 mb = f32_to_bf4(mv);
          *(uint4*)(M16 + o - 4) = make_uint4(pm.x, pm.y, mb.x, mb.y);
        }
      }
      if (OPT != kSGD16) *(f32x4*)(M32 + o) = mv;
      if (OPT == kAdamW) *(f32x4*)(V32 + o) = vv;
    }

    // ---- bias: db[n] = sum_b dZ[b][n]; only the k-strip-0 workgroup owns the bias ----
    if (do_bias) {
      red[bpart * 64 + bcol] = bsum;
      __syncthreads();
      if (tid < (NARROW ? kNarrowRows : 64)) {
        const float gb = red[tid] + red[64 + tid] + red[128 + tid] + red[192 + tid];
        bf16_t* bph = p16 + tl.b_off + nc + tid;
        bf16_t* bpl = plo + tl.b_off + nc + tid;
        float* bm = m32 + tl.b_off + nc + tid;
        bf16_t* bm16 = (bf16_t*)m32 + tl.b_off + nc + tid;
        float bw = join_hilo(*bph, *bpl), mb = OPT == kSGD16 ? bf2f(*bm16) : *bm;
        float* bv = v32 + tl.b_off + nc + tid;
        float vb = OPT == kAdamW ? *bv : 0.f;
        bias_update<OPT>(bw, mb, vb, gb, h, c1, c2);
        if (OPT == kAdamW) *bv = vb;
        const uint32_t ub = __float_as_uint(bw), hb = split_hi(ub) & 0xFFFFu;
        *bph = (bf16_t)hb;
        *bpl = (bf16_t)split_lo(ub, hb);
        if (OPT == kSGD16) *bm16 = f2bf(mb);
        else *bm = mb;
      }
    }
    }  // MODE != 2
    __syncthreads();
    if (more) {
      if (PF) MOPT_BWD_ADVANCE()
      else MOPT_BWD_LOAD(nc + BN, c)
    }
  }
#undef MOPT_BWD_LOAD
#undef MOPT_BWD_ADVANCE

  if (!has_dx) return;
  // ---- dZ of the layer below: dX * relu'(.) * dropout mask, both read off X (X > 0) ----
  const float inv_keep = ((flags & kInDropout) && h.drop > 0.f) ? 1.f / (1.f - h.drop) : 1.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 32 * wave + 16 * i + 4 * g + r, col = 16 * j + li;
        const float xv = bf2f(Xs[BOFF(row, col)]);
        Zs[BOFF(row, col)] = f2bf(xv > 0.f ? dx[i][j][r] * inv_keep : 0.f);
      }
  __syncthreads();
  bf16_t* GX = grad + tl.gx_off + (size_t)rbx * BM * K + k0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i, r = c >> 3, ch = c & 7;
    *(uint4*)(GX + (size_t)r * K + ch * 8) = *(const uint4*)(Zs + BOFF(r, ch * 8));
  }
}

// ----------------------------------------------------------------------------------------------
// First layer, fused across two steps: the backward + optimizer of step t AND the forward of
// step t + 1 (round 5).  The first layer has no dX, and its input (the shared minibatch) of the
// next step is known while step t runs, so one pass over W0 can update it and immediately
// multiply the NEW weights with the next batch -- the separate forward of layer 0 (a second read
// of the largest weight matrix, ~10 % of the step) disappears.  A workgroup owns one 64-row
// output chunk n0 of W0 for ALL of K (the other kernels own a k-strip for all of N), so it holds
// the complete dot products of the next step's outputs Y'[:, n0:n0+64]:
//   dZ[:, chunk] staged once; the chunk's bias gradient / update;
//   for each 64-wide k-strip s:  dW^T = X[:, s]^T dZ[:, chunk]          (as mlp_bwd_opt_kernel)
//                                W, M <- update(W, M, dW)   in the MFMA C layout (4 consecutive
//                                          k of one row per lane: no LDS restaging)
//                                acc += X'[:, s] W_new[chunk, s]^T     (as mlp_fwd_kernel: same
//                                          fragments, same K order -> bit-identical outputs)
//   Y' = dropout(relu(acc + b_new)) with the t + 1 dropout key.
// Every result equals the unfused step pair bit for bit (tests/test_kernels_gpu.py).  Batches of
// one 128-row block only (MODE 0); the caller keeps the unfused launches otherwise.
// ----------------------------------------------------------------------------------------------
// PF: the next strip's state in a second register set (SGD, SGD16; AdamW's f32 moments do not
// fit twice); two waves per SIMD
template <int OPT, bool PF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void mlp_bwd0_fwd_kernel(
    const MlpTL* __restrict__ tls, const int2* __restrict__ work, int n_work,
    const bf16_t* __restrict__ xb, const bf16_t* __restrict__ xn, const bf16_t* __restrict__ grad,
    bf16_t* __restrict__ act, bf16_t* __restrict__ plo, bf16_t* __restrict__ p16,
    float* __restrict__ m32, float* __restrict__ v32, const TrialHP* __restrict__ hp, int flags) {
  constexpr int DS = BN + 4;   // f32 row stride of the dW staging tile (FOFF)
  __shared__ __attribute__((aligned(16)))
      bf16_t smem[2 * BM * TS + BN * TSF + 2 * BN * DS + 2 * 4 * BN + 2 * BN];
  bf16_t* Zs = smem;                  // dZ[:, chunk]      [128][TS]  (the whole pass)
  bf16_t* Xs = smem + BM * TS;        // X[:, strip]       [128][TS]  (then the output tile)
  bf16_t* Ws = smem + 2 * BM * TS;    // W_new[chunk, strip] hi [64][TSF]
  float* Dw = (float*)(smem + 2 * BM * TS + BN * TSF);     // dW[chunk, strip] f32 [64][DS]
  float* red = Dw + BN * DS;                               // [4][64] bias partial sums
  float* bnew = red + 4 * BN;                              // [64] updated bias (f32)

  const int2 wi = work[blockIdx.x];
  if (wi.x < 0) return;
  const MlpTL tl = tls[wi.x];
  const int K = tl.K, N = tl.N, n0 = wi.y * BN;
  const bf16_t* X = xb + tl.x_off;
  const bf16_t* Xn = xn + tl.x_off;
  const bf16_t* dZ = grad + tl.y_off;
  bf16_t* WLO = plo + tl.w_off;
  float* M32 = m32 + tl.w_off;
  bf16_t* M16 = (bf16_t*)m32 + tl.w_off;
  float* V32 = v32 + tl.w_off;
  bf16_t* W16 = p16 + tl.w_off;
  const TrialHP h = hp[tl.trial];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4, q = li >> 2, pp = li & 3;
  const int wk = wave >> 1, wn = wave & 1;
  float c1 = 1.f, c2 = 1.f;
  if (OPT == kAdamW) {
    const float t = (float)h.t;
    c1 = h.lr / (1.f - __powf(h.b1, t));
    c2 = 1.f / sqrtf(1.f - __powf(h.b2, t));
  }

  // dZ[:, n0:n0+64] -> LDS once; X[:, strip 0] into registers
  const int xo0 = (tid >> 3) * K + (tid & 7) * 8;       // + 32 K i: rows tid / 8 + 32 i
  uint4 xr0, xr1, xr2, xr3;
  xr0 = *(const uint4*)(X + xo0);
  xr1 = *(const uint4*)(X + xo0 + 32 * K);
  xr2 = *(const uint4*)(X + xo0 + 64 * K);
  xr3 = *(const uint4*)(X + xo0 + 96 * K);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i, r = c >> 3, ch = c & 7;
    *(uint4*)(Zs + TOFF(r, ch * 8)) = *(const uint4*)(dZ + (size_t)r * N + n0 + ch * 8);
  }
  __syncthreads();

  // ---- bias of the chunk: db[n] = sum_b dZ[b][n] (mlp_bwd_opt_kernel's order) and its update ----
  const bool do_bias = flags & kUpdateBias;
  if (do_bias) {
    const int bcol = tid & 63, bpart = tid >> 6;
    float bsum = 0.f;
    for (int r = bpart * 32; r < bpart * 32 + 32; ++r) bsum += bf2f(Zs[TOFF(r, bcol)]);
    red[bpart * 64 + bcol] = bsum;
  }
  __syncthreads();
  if (tid < 64) {
    bf16_t* bph = p16 + tl.b_off + n0 + tid;
    bf16_t* bpl = plo + tl.b_off + n0 + tid;
    float bw = join_hilo(*bph, *bpl);
    if (do_bias) {
      const float gb = red[tid] + red[64 + tid] + red[128 + tid] + red[192 + tid];
      float* bm = m32 + tl.b_off + n0 + tid;
      bf16_t* bm16 = (bf16_t*)m32 + tl.b_off + n0 + tid;
      float mb = OPT == kSGD16 ? bf2f(*bm16) : *bm;
      float* bv = v32 + tl.b_off + n0 + tid;
      float vb = OPT == kAdamW ? *bv : 0.f;
      bias_update<OPT>(bw, mb, vb, gb, h, c1, c2);
      if (OPT == kAdamW) *bv = vb;
      const uint32_t ub = __float_as_uint(bw), hb = split_hi(ub) & 0xFFFFu;
      *bph = (bf16_t)hb;
      *bpl = (bf16_t)split_lo(ub, hb);
      if (OPT == kSGD16) *bm16 = f2bf(mb);
      else *bm = mb;
    }
    bnew[tid] = bw;   // join_hilo of the stored pair is bw exactly
  }

  // the next batch's A fragments (rows 32 wave + 16 i + li, k 32 ks + 8 g) straight from global
  // memory (the shared minibatch: L2-resident), 4 per strip
  const int ao = (32 * wave + li) * K + 8 * g;              // + 16 K i + 32 ks
  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  // Weight / optimizer state in mlp_bwd_opt_kernel's thread layout: rows tid / 8 + 32 i (i < 2),
  // 8 consecutive k at 8 (tid % 8) -- 16 bytes per lane, a wave-instruction moves 8 whole
  // 128-byte rows.  (The MFMA C layout -- 4 k of one row per lane, 16 rows x 32 bytes per
  // instruction, no LDS restaging -- ran the pass ~45 % slower.)  The current strip's set (c*)
  // and, PF, the next strip's (n*), loaded while this strip is multiplied and updated.
  const int so = (tid >> 3) * BK + 8 * (tid & 7);           // + 32 BK: the second row
  // dead padding (live8): this thread's rows n0 + tid / 8 (+ 32) below nl, its k-chunk of strip
  // S at S BK + 8 (tid % 8) below kl -- dead state is neither loaded nor stored
  const int nl = live8(tl.n_real);
  const bool rl0 = n0 + (tid >> 3) < nl, rl1 = n0 + (tid >> 3) + 32 < nl;
  uint4 cwh0{}, cwh1{}, cwl0{}, cwl1{}, cmh0{}, cmh1{}, nwh0{}, nwh1{}, nwl0{}, nwl1{}, nmh0{},
      nmh1{};
  f32x4 cm[4]{}, cv[4]{}, nm[4]{}, nv[4]{};
#define MOPT_B0F_LOAD(P, S)                                                                      \
  {                                                                                              \
    const size_t o_ = (size_t)(S) * BK * N + (size_t)n0 * BK + so;                               \
    /* dead rows / k-chunks re-read the chunk's first row at the strip's first k (live): L2   \
       hits instead of HBM traffic, no branch around the loads */                              \
    constexpr bool kl_ = true;   /* dead k-chunks: moved like live ones (whole lines) */         \
    const size_t od_ = (size_t)(S) * BK * N + (size_t)n0 * BK;                                   \
    const size_t o0_ = rl0 && kl_ ? o_ : od_, o1_ = rl1 && kl_ ? o_ + 32 * BK : od_;             \
    P##wh0 = *(const uint4*)(W16 + o0_);                                                         \
    P##wh1 = *(const uint4*)(W16 + o1_);                                                         \
    P##wl0 = *(const uint4*)(WLO + o0_);                                                         \
    P##wl1 = *(const uint4*)(WLO + o1_);                                                         \
    if (OPT == kSGD16) {                                                                         \
      P##mh0 = *(const uint4*)(M16 + o0_);                                                       \
      P##mh1 = *(const uint4*)(M16 + o1_);                                                       \
    } else {                                                                                     \
      _Pragma("unroll") for (int i = 0; i < 4; ++i)                                              \
        P##m[i] = *(const f32x4*)(M32 + ((i >> 1) ? o1_ : o0_) + 4 * (i & 1));                   \
    }                                                                                            \
    if (OPT == kAdamW) {                                                                         \
      _Pragma("unroll") for (int i = 0; i < 4; ++i)                                              \
        P##v[i] = *(const f32x4*)(V32 + ((i >> 1) ? o1_ : o0_) + 4 * (i & 1));                   \
    }                                                                                            \
  }
  MOPT_B0F_LOAD(c, 0)
  for (int s = 0; s < nk; ++s) {
    const int k0 = s * BK;
    const size_t sb = (size_t)k0 * N + (size_t)n0 * BK + so;   // strip s, this thread's rows
    const int sn = s + 1 < nk ? s + 1 : s;   // the next strip (the last re-reads its own: every
                                             // load unconditional, the counted waits exact)
    // X[:, strip s] -> LDS; the next strip's X and state into registers
    *(uint4*)(Xs + TOFF(tid >> 3, (tid & 7) * 8)) = xr0;
    *(uint4*)(Xs + TOFF(32 + (tid >> 3), (tid & 7) * 8)) = xr1;
    *(uint4*)(Xs + TOFF(64 + (tid >> 3), (tid & 7) * 8)) = xr2;
    *(uint4*)(Xs + TOFF(96 + (tid >> 3), (tid & 7) * 8)) = xr3;
    {
      const int kn = sn * BK;
      xr0 = *(const uint4*)(X + xo0 + kn);
      xr1 = *(const uint4*)(X + xo0 + 32 * K + kn);
      xr2 = *(const uint4*)(X + xo0 + 64 * K + kn);
      xr3 = *(const uint4*)(X + xo0 + 96 * K + kn);
    }
    if (PF) MOPT_B0F_LOAD(n, sn)
    uint4 an[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        an[i][ks] = *(const uint4*)(Xn + ao + 16 * K * i + k0 + 32 * ks);
    __syncthreads();   // Xs visible; the previous strip's readers of Dw / Ws are done

    // ---- dW^T[strip, chunk] = X^T dZ (mlp_bwd_opt_kernel's fragments and order) -> Dw ----
    {
      f32x4 dw[2][2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u) dw[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        bf16x8 xa[2], bz[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int c0 = 32 * wk + 16 * t + 4 * pp;
          xa[t] = cat_frag(lds_tr4(Xs + TOFF(32 * s4 + 8 * g + q, c0)),
                           lds_tr4(Xs + TOFF(32 * s4 + 8 * g + 4 + q, c0)));
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int c0 = 32 * wn + 16 * u + 4 * pp;
          bz[u] = cat_frag(lds_tr4(Zs + TOFF(32 * s4 + 8 * g + q, c0)),
                           lds_tr4(Zs + TOFF(32 * s4 + 8 * g + 4 + q, c0)));
        }
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int u = 0; u < 2; ++u) dw[t][u] = mfma16(xa[t], bz[u], dw[t][u]);
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u)
          *(f32x4*)(Dw + FOFF(32 * wn + 16 * u + li, 32 * wk + 16 * t + 4 * g)) = dw[t][u];
    }
    __syncthreads();   // Dw visible

    // ---- optimizer (mlp_bwd_opt_kernel's epilogue): group i = row 32 (i / 2) + tid / 8,
    //      k 8 (tid % 8) + 4 (i % 2) .. + 3 ----
    {
      const f32x4 w[4] = {join4(make_uint2(cwh0.x, cwh0.y), make_uint2(cwl0.x, cwl0.y)),
                          join4(make_uint2(cwh0.z, cwh0.w), make_uint2(cwl0.z, cwl0.w)),
                          join4(make_uint2(cwh1.x, cwh1.y), make_uint2(cwl1.x, cwl1.y)),
                          join4(make_uint2(cwh1.z, cwh1.w), make_uint2(cwl1.z, cwl1.w))};
      f32x4 m[4];
      if (OPT == kSGD16) {
        m[0] = bf4_to_f32(make_uint2(cmh0.x, cmh0.y)); m[1] = bf4_to_f32(make_uint2(cmh0.z, cmh0.w));
        m[2] = bf4_to_f32(make_uint2(cmh1.x, cmh1.y)); m[3] = bf4_to_f32(make_uint2(cmh1.z, cmh1.w));
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) m[i] = cm[i];
      }
      uint2 ph{}, pl{}, pm{};
      constexpr bool kls = true;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int gr = 32 * (i >> 1) + (tid >> 3), gk = 8 * (tid & 7) + 4 * (i & 1);
        if (!((i >> 1) ? rl1 : rl0) || !kls) {   // dead padding: W_new's image row stays zero
          if (i & 1) *(uint4*)(Ws + TOFFF(gr, gk - 4)) = make_uint4(0, 0, 0, 0);
          continue;
        }
        const f32x4 gv = *(const f32x4*)(Dw + FOFF(gr, gk));
        const size_t o = sb + (size_t)(32 * (i >> 1)) * BK + 4 * (i & 1);
        f32x4 wv = w[i], mv = m[i], vv;
        if (OPT == kAdamW) vv = cv[i];
        opt_update4<OPT>(wv, mv, vv, gv, h, c1, c2);
        uint2 nh, nl;
        split4(wv, nh, nl);
        if ((i & 1) == 0) {
          ph = nh;
          pl = nl;
          pm = f32_to_bf4(mv);
        } else {
          const uint4 hi16 = make_uint4(ph.x, ph.y, nh.x, nh.y);
          *(uint4*)(W16 + o - 4) = hi16;
          *(uint4*)(WLO + o - 4) = make_uint4(pl.x, pl.y, nl.x, nl.y);
          if (OPT == kSGD16) {
            const uint2 mb = f32_to_bf4(mv);
            *(uint4*)(M16 + o - 4) = make_uint4(pm.x, pm.y, mb.x, mb.y);
          }
          *(uint4*)(Ws + TOFFF(gr, gk - 4)) = hi16;
        }
        if (OPT != kSGD16) *(f32x4*)(M32 + o) = mv;
        if (OPT == kAdamW) *(f32x4*)(V32 + o) = vv;
      }
    }
    __syncthreads();   // W_new of the strip complete in LDS

    // ---- the next step's forward: acc += X'[:, strip] . W_new[chunk, strip]^T ----
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = lds_frag(Ws + TOFFF(j * 16 + li, ks * 32 + g * 8));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = mfma16(__builtin_bit_cast(bf16x8, an[i][ks]), b[j], acc[i][j]);
    }
    if (PF) {
      cwh0 = nwh0; cwh1 = nwh1; cwl0 = nwl0; cwl1 = nwl1;
      if (OPT == kSGD16) { cmh0 = nmh0; cmh1 = nmh1; }
      else {
#pragma unroll
        for (int i = 0; i < 4; ++i) cm[i] = nm[i];
      }
      if (OPT == kAdamW) {
#pragma unroll
        for (int i = 0; i < 4; ++i) cv[i] = nv[i];
      }
    } else if (s + 1 < nk) {
      MOPT_B0F_LOAD(c, s + 1)
    }
  }
  __syncthreads();   // every wave is done with Xs (the output tile) and Ws
#undef MOPT_B0F_LOAD

  // ---- Y'[:, chunk] = dropout(relu(acc + b_new)), keyed by step t + 1 (mlp_fwd_kernel's epilogue) ----
  const bool drop = (flags & kInDropout) && h.drop > 0.f;   // kInDropout: the forward's dropout
  const float inv_keep = drop ? 1.f / (1.f - h.drop) : 1.f;
  const uint32_t key = rng_key(h.seed, 0u, h.t + 1u);
  bf16_t* Cs = Xs;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = j * 16 + li;
    const float bj = bnew[col];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wave * 32 + i * 16 + g * 4 + r;
        float v = fmaxf(acc[i][j][r] + bj, 0.f);
        if (drop) {
          const uint32_t idx = (uint32_t)(row * N + n0 + col);
          v = rng_uniform(key, idx) >= h.drop ? v * inv_keep : 0.f;
        }
        Cs[TOFF(row, col)] = f2bf(v);
      }
  }
  __syncthreads();
  bf16_t* Y = act + tl.y_off + n0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i, r = c >> 3, ch = c & 7;
    *(uint4*)(Y + (size_t)r * N + ch * 8) = *(const uint4*)(Cs + TOFF(r, ch * 8));
  }
}

// Member initialisation (torch.nn.Linear-style U(-1/sqrt(fan_in), +)) for every new member of a
// sync in ONE launch: weights and bias from the counter-based RNG (so the PyTorch reference draws
// the same values), zero padding, the bf16 copy, and zeroed optimizer state.  Replaces ~10 small
// framework launches per member.
__global__ __launch_bounds__(256) void mlp_init_kernel(const InitDesc* __restrict__ descs,
                                                       bf16_t* __restrict__ plo,
                                                       bf16_t* __restrict__ p16,
                                                       float* __restrict__ m32,
                                                       float* __restrict__ v32, int flags) {
  const InitDesc d = descs[blockIdx.y];
  const uint32_t wkey = rng_key(d.seed, 0x1000u + (uint32_t)d.layer, 0u);
  const uint32_t bkey = rng_key(d.seed, 0x2000u + (uint32_t)d.layer, 0u);
  const int64_t nw = (int64_t)d.N * d.K;
  const int64_t total = nw + d.N;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    int64_t o;
    if (e < nw) {   // e walks the stored layout; the RNG counter is the row-major index n K + k
      int n, k;
      w_coords(e, d.N, d.K, n, k);
      if (n < d.n_real && k < d.k_real)
        v = (2.f * rng_uniform(wkey, (uint32_t)((int64_t)n * d.K + k)) - 1.f) * d.bound;
      o = d.w_off + e;
    } else {
      const int n = (int)(e - nw);
      if (n < d.n_real) v = (2.f * rng_uniform(bkey, (uint32_t)n) - 1.f) * d.bound;
      o = d.b_off + n;
    }
    const uint32_t u = __float_as_uint(v), h = split_hi(u) & 0xFFFFu;
    p16[o] = (bf16_t)h;
    plo[o] = (bf16_t)split_lo(u, h);
    if (flags & 2) ((bf16_t*)m32)[o] = 0;   // bf16 momentum (kSGD16)
    else m32[o] = 0.f;
    if (flags & 1) v32[o] = 0.f;
  }
}


template <int OPT, bool PF, int MODE>
static void launch_bwd(int n_work, int grid_y, hipStream_t stream, const void* tls,
                       const void* work, const void* xb, void* grad, void* plo, void* p16,
                       void* m32, void* v32, const void* hp, int flags) {
  if (flags & kNarrow)
    hipLaunchKernelGGL((mlp_bwd_opt_kernel<OPT, PF, MODE, true>), dim3(n_work, grid_y), dim3(256),
                       0, stream, (const MlpTL*)tls, (const int2*)work, n_work, (const bf16_t*)xb,
                       (bf16_t*)grad, (bf16_t*)plo, (bf16_t*)p16, (float*)m32, (float*)v32,
                       (const TrialHP*)hp, flags);
  else
    hipLaunchKernelGGL((mlp_bwd_opt_kernel<OPT, PF, MODE, false>), dim3(n_work, grid_y), dim3(256),
                       0, stream, (const MlpTL*)tls, (const int2*)work, n_work, (const bf16_t*)xb,
                       (bf16_t*)grad, (bf16_t*)plo, (bf16_t*)p16, (float*)m32, (float*)v32,
                       (const TrialHP*)hp, flags);
}

// one layer's backward: 128-row batches -> the fused MODE 0 kernel (prefetch per the switch);
// R > 1 row blocks -> MODE 2 (dX of blocks 1..R-1, before W changes) then the fused MODE 1
template <int OPT>
static void launch_bwd_rows(int n_work, int n_rowblocks, hipStream_t stream, const void* tls,
                            const void* work, const void* xb, void* grad, void* plo, void* p16,
                            void* m32, void* v32, const void* hp, int flags) {
  if (n_rowblocks <= 1) {
    // AdamW's second register set (M and V in f32) does not fit next to the MFMA operands: the
    // prefetch variant spills (256 VGPRs + scratch), so AdamW always runs the plain one
    if (OPT != kAdamW)
      launch_bwd<OPT, true, 0>(n_work, 1, stream, tls, work, xb, grad, plo, p16, m32, v32, hp,
                               flags);
    else
      launch_bwd<OPT, false, 0>(n_work, 1, stream, tls, work, xb, grad, plo, p16, m32, v32, hp,
                                flags);
    return;
  }
  if (flags & kHasDx)
    launch_bwd<OPT, false, 2>(n_work, n_rowblocks - 1, stream, tls, work, xb, grad, plo, p16,
                              m32, v32, hp, flags);
  launch_bwd<OPT, false, 1>(n_work, 1, stream, tls, work, xb, grad, plo, p16, m32, v32, hp, flags);
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// C ABI (loaded with ctypes by metaopt_amd/ops/_lib.py).  Every launcher returns a hipError_t.
// ------------------------------------------------------------------------------------------------
extern "C" {

int mopt_abi_version() { return 15; }

// weight layout: 1 = k-strip-major [K/64][N][64] (the only layout)
int mopt_mlp_w_layout() { return 1; }

// 1 when this library is the bounds-checked variant (-DMOPT_BOUNDS_CHECK)
int mopt_checked_build() { return MOPT_CHECKED_BUILD; }

// flags: 1 = zero the AdamW second moment, 2 = the momentum buffer is bf16
int mopt_mlp_init(const void* descs, int n_desc, void* plo, void* p16, void* m32, void* v32,
                  int flags, void* stream) {
  if (n_desc <= 0) return 0;
  hipLaunchKernelGGL(mlp_init_kernel, dim3(64, n_desc), dim3(256), 0, (hipStream_t)stream,
                     (const InitDesc*)descs, (bf16_t*)plo, (bf16_t*)p16, (float*)m32, (float*)v32,
                     flags);
  return (int)hipGetLastError();
}

// tile_n: output features per work item (64: the work list was built for it; 32 and 128 were
// measured slower or neutral in round 3, profiles/round3.md "Forward tile width")
int mopt_mlp_fwd(const void* tls, const void* work, int n_work, int n_rowblocks, const void* xb,
                 const void* plo, const void* p16, void* act, const void* hp, unsigned step,
                 int layer, int flags, int tile_n, void* stream) {
  if (n_work <= 0) return 0;
  if (tile_n != 64) return (int)hipErrorInvalidValue;
  // (three register sets at 3 waves / SIMD, with the same whole-group loop: step 654-656 vs
  //  651-654 us, bench 784-787 vs 790-791 trials/s -- profiles/round4.md)
  hipLaunchKernelGGL((mlp_fwd_kernel<64, 2, 4>), dim3(n_work, n_rowblocks), dim3(256), 0,
                     (hipStream_t)stream, (const MlpTL*)tls, (const int2*)work, n_work,
                     (const bf16_t*)xb, (const bf16_t*)plo, (const bf16_t*)p16, (bf16_t*)act,
                     (const TrialHP*)hp, step, layer, flags);
  return (int)hipGetLastError();
}

int mopt_mlp_fwd_ce(const void* tls, const void* work, int n_work, int n_rowblocks, const void* xb,
                    const void* plo, const void* p16, const void* labels, void* grad, void* loss,
                    void* correct, void* hp, float inv_b, int flags, void* stream) {
  if (n_work <= 0) return 0;
  if ((flags & kStoreStats) && n_rowblocks != 1) return (int)hipErrorInvalidValue;
  if (flags & kNarrowCE)
    hipLaunchKernelGGL(mlp_fwd_ce_kernel<true>, dim3(n_work, n_rowblocks), dim3(256), 0,
                       (hipStream_t)stream, (const MlpTL*)tls, (const int2*)work, n_work,
                       (const bf16_t*)xb, (const bf16_t*)plo, (const bf16_t*)p16,
                       (const int32_t*)labels, (bf16_t*)grad, (float*)loss, (float*)correct,
                       (TrialHP*)hp, inv_b, flags);
  else
    hipLaunchKernelGGL(mlp_fwd_ce_kernel<false>, dim3(n_work, n_rowblocks), dim3(256), 0,
                       (hipStream_t)stream, (const MlpTL*)tls, (const int2*)work, n_work,
                       (const bf16_t*)xb, (const bf16_t*)plo, (const bf16_t*)p16,
                       (const int32_t*)labels, (bf16_t*)grad, (float*)loss, (float*)correct,
                       (TrialHP*)hp, inv_b, flags);
  return (int)hipGetLastError();
}


int mopt_mlp_bwd(const void* tls, const void* work, int n_work, const void* xb, void* grad,
                 void* plo, void* p16, void* m32, void* v32, const void* hp, int opt, int flags,
                 int n_rowblocks, void* stream) {
  if (n_work <= 0) return 0;
  if (n_rowblocks < 1 || n_rowblocks > 64) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (opt == kAdamW)
    launch_bwd_rows<kAdamW>(n_work, n_rowblocks, st, tls, work, xb, grad, plo, p16, m32, v32, hp,
                            flags);
  else if (opt == kSGD16)
    launch_bwd_rows<kSGD16>(n_work, n_rowblocks, st, tls, work, xb, grad, plo, p16, m32, v32, hp,
                            flags);
  else
    launch_bwd_rows<kSGD>(n_work, n_rowblocks, st, tls, work, xb, grad, plo, p16, m32, v32, hp,
                          flags);
  return (int)hipGetLastError();
}

// One whole train step of a group of trials (forward of every layer, fused loss, fused backward
// + optimizer of every layer, top-down) in ONE host call: the per-step host cost of the sweep is
// one C call instead of 2L bound-method calls.  The argument block is built once per work-table
// refresh (metaopt_amd/ops/population.py, _MlpStep mirrors it); x / y change every step.
struct MlpStep {
  const void* tls;
  const void* fwd[8];
  const void* bwd[8];
  int32_t n_fwd[8];
  int32_t n_bwd[8];
  int32_t L, rb, drop, opt;
  void *plo, *p16, *m32, *v32, *act, *grad, *hp, *loss, *correct;
  float inv_b;      // <= 0: each trial's mean over its own rows (MlpTL::rows)
  int32_t n_stats;  // entries of loss / correct (the population's capacity)
  int32_t fwd_tn;   // hidden-layer forward tile width of the work lists (64)
  int32_t narrow;   // 1: the loss layer has <= 16 classes (kNarrowCE / kNarrow launches)
  const void* bwd0f;  // work list of the fused first layer (mlp_bwd0_fwd_kernel): (tl, n-chunk)
  int32_t n_bwd0f;
  int32_t fuse0;      // 1: consecutive steps of mopt_mlp_steps run the fused first layer
};

namespace {

int mlp_bwd0_fwd(const MlpStep* s, const void* x, const void* x_next, void* stream) {
  if (s->n_bwd0f <= 0) return 0;
  const int flags = kUpdateBias | (s->drop ? kInDropout : 0);
  const dim3 grid(s->n_bwd0f), block(256);
#define MOPT_B0F(O, W)                                                                           \
  hipLaunchKernelGGL((mlp_bwd0_fwd_kernel<O, W>), grid, block, 0, (hipStream_t)stream,          \
                     (const MlpTL*)s->tls, (const int2*)s->bwd0f, s->n_bwd0f, (const bf16_t*)x,  \
                     (const bf16_t*)x_next, (const bf16_t*)s->grad, (bf16_t*)s->act,            \
                     (bf16_t*)s->plo, (bf16_t*)s->p16, (float*)s->m32, (float*)s->v32,          \
                     (const TrialHP*)s->hp, flags)
  if (s->opt == kAdamW) MOPT_B0F(kAdamW, false);
  else if (s->opt == kSGD16) MOPT_B0F(kSGD16, true);
  else MOPT_B0F(kSGD, true);
#undef MOPT_B0F
  return (int)hipGetLastError();
}

// one train step; fwd0_done: layer 0's forward of this step already ran (fused into the previous
// step's first-layer backward); x_next != nullptr: fuse this step's first-layer backward with the
// next step's first-layer forward (batch x_next)
int mlp_step(const MlpStep* s, const void* x, const void* y, bool fwd0_done, const void* x_next,
             void* stream) {
  if (s == nullptr || s->L < 1 || s->L > 8 || s->rb < 1) return (int)hipErrorInvalidValue;
  const int L = s->L;
  int err;
  if (s->rb > 1) {   // several row blocks add into the statistics (one stream per population)
    if (s->n_stats < 1) return (int)hipErrorInvalidValue;
    err = (int)hipMemsetAsync(s->loss, 0, sizeof(float) * s->n_stats, (hipStream_t)stream);
    if (!err) err = (int)hipMemsetAsync(s->correct, 0, sizeof(float) * s->n_stats, (hipStream_t)stream);
    if (err) return err;
  }
  for (int l = fwd0_done ? 1 : 0; l < L - 1; ++l) {
    err = mopt_mlp_fwd(s->tls, s->fwd[l], s->n_fwd[l], s->rb, l == 0 ? x : s->act, s->plo,
                       s->p16, s->act, s->hp, 1u, l, kRelu | (s->drop ? kDropout : 0), s->fwd_tn,
                       stream);
    if (err) return err;
  }
  const int ce = kWriteGrad | kCountStep | (s->rb == 1 ? kStoreStats : 0) |
                 (s->narrow ? kNarrowCE : 0);
  err = mopt_mlp_fwd_ce(s->tls, s->fwd[L - 1], s->n_fwd[L - 1], s->rb, L == 1 ? x : s->act,
                        s->plo, s->p16, y, s->grad, s->loss, s->correct, s->hp, s->inv_b, ce,
                        stream);
  if (err) return err;
  for (int l = L - 1; l >= 0; --l) {
    if (l == 0 && x_next != nullptr) return mlp_bwd0_fwd(s, x, x_next, stream);
    int flags = kUpdateBias | ((l == L - 1 && s->narrow) ? kNarrow : 0);
    if (l > 0) flags |= kHasDx | (s->drop ? kInDropout : 0);
    err = mopt_mlp_bwd(s->tls, s->bwd[l], s->n_bwd[l], l == 0 ? x : s->act, s->grad, s->plo,
                       s->p16, s->m32, s->v32, s->hp, s->opt, flags, s->rb, stream);
    if (err) return err;
  }
  return 0;
}

}  // namespace

int mopt_mlp_step(const MlpStep* s, const void* x, const void* y, void* stream) {
  return mlp_step(s, x, y, false, nullptr, stream);
}

// the fused first layer of one step alone (its backward + update with batch x, the next step's
// forward with batch x_next): scripts/kernel_bench.py times it
int mopt_mlp_bwd0_fwd(const MlpStep* s, const void* x, const void* x_next, void* stream) {
  if (s == nullptr || s->rb != 1 || s->L < 2) return (int)hipErrorInvalidValue;
  return mlp_bwd0_fwd(s, x, x_next, stream);
}

// ``n`` consecutive train steps of a group in ONE host call (step i reads batch xs[i] / ys[i]):
// the sweep queues a whole sync interval with it, so the per-step host cost is the launches alone.
int mopt_mlp_steps(const MlpStep* s, const void* const* xs, const void* const* ys, int n,
                   void* stream) {
  if (n < 0 || (n > 0 && (xs == nullptr || ys == nullptr))) return (int)hipErrorInvalidValue;
  // the fused first layer needs one 128-row block per trial and a hidden layer in front of the
  // loss layer; the last step of the call keeps the unfused backward (no next batch)
  const bool fuse = s != nullptr && s->fuse0 && s->rb == 1 && s->L >= 2 && s->n_bwd0f > 0;
  for (int i = 0; i < n; ++i) {
    const void* xn = (fuse && i + 1 < n) ? xs[i + 1] : nullptr;
    const int err = mlp_step(s, xs[i], ys[i], fuse && i > 0, xn, stream);
    if (err) return err;
  }
  return 0;
}

// Steps i0 .. i0 + count - 1 of an n-step interval (xs / ys hold all n batches): the sweep queues
// its trial groups' intervals round-robin in short runs of steps, so every group's stream has
// work from the interval's first microsecond to its last (one group's whole interval queued
// before the next group's left the first group running alone at the start and the last one at
// the end).  The fused first layer spans the runs: step i fuses with batch xs[i + 1] whenever
// i + 1 < n, exactly as one mopt_mlp_steps call over the n steps.
int mopt_mlp_steps_range(const MlpStep* s, const void* const* xs, const void* const* ys, int i0,
                         int n, int count, void* stream) {
  if (i0 < 0 || count < 0 || i0 + count > n || (count > 0 && (xs == nullptr || ys == nullptr)))
    return (int)hipErrorInvalidValue;
  const bool fuse = s != nullptr && s->fuse0 && s->rb == 1 && s->L >= 2 && s->n_bwd0f > 0;
  for (int i = i0; i < i0 + count; ++i) {
    const void* xn = (fuse && i + 1 < n) ? xs[i + 1] : nullptr;
    const int err = mlp_step(s, xs[i], ys[i], fuse && i > 0, xn, stream);
    if (err) return err;
  }
  return 0;
}

}  // extern "C"

// device-side index checks of the checked build (common.h)
MOPT_VIOLATIONS_READER(pop_mlp)
