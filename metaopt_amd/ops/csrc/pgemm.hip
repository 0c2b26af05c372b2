// Population-batched bf16 GEMM on MFMA (gfx950): C[p] = op(A[p]) . op(B[p]) for p < P.
//
// The trial population is the batch dimension.  Each operand is read in the layout it is stored
// in, so the three GEMMs of a linear layer never materialise a transpose:
//     forward   Y  = X . W        A = X [M][K]   B = W [K][N]          (NN)
//     input     dX = dY . W^T     A = dY [M][N]  B = W stored [K][N]   (NT: B is [n][k])
//     weight    dW = X^T . dY     A = X stored [M][K]  B = dY [M][N]   (TN: A is [k][m])
// (this also sidesteps the transposed-operand batched GEMM of the installed library stack that
// returns wrong results for some shapes -- scripts/check_bmm.py).
//
// Structure: 256 threads = 4 waves arranged WM x (4/WM); each wave owns FM x FN fragments of
// v_mfma_f32_16x16x32_bf16 (a 16*FM x 16*FN sub-tile), so the block tile is BM x BN with
// BM = WM*16*FM, BN = (4/WM)*16*FN; BK = 64.  Operand tiles are staged global -> registers ->
// LDS (double-buffered LDS, one barrier per K tile, the next tile's global loads in flight
// while the current one is multiplied).  The LDS image keeps the stored orientation:
//   * k-contiguous operands ([m][k] / [n][k]) as [row][64 + 8 pad] -> fragments by ds_read_b128;
//   * row-contiguous operands ([k][m] / [k][n]) as [k][rows + 8 pad] -> fragments by the
//     transposing ds_read_b64_tr_b16 (two per fragment).
// Split-K (for the weight gradient's long reduction over tokens / pixels) writes f32 partial
// tiles that a second pass sums and rounds to bf16.  Blocks are remapped XCD-aware so the tiles
// sharing an A row panel run on one XCD (one L2).
//
// Large dense shapes (the LM's projections and their gradients: M, N multiples of 128/256) use a
// second kernel, pgemm_big_kernel (below): 8 waves, 256-wide tiles, operands filled straight
// from global memory into swizzled LDS images, persistent over the tiles.
#include "common.h"

using namespace mopt;

namespace {

constexpr int BK = 64;
constexpr int LSK = BK + 8;  // row stride of k-contiguous LDS images (144 B)

// Operand sources.  Each operand is a stored matrix S[outer][inner] (inner contiguous) read in
// 16-byte chunks S[o][i .. i+7]; at() returns the chunk's address, or nullptr outside the matrix
// (the chunk is zero-filled).  Besides dense row-major storage, three gathers make a 3x3
// convolution (pad 1, stride 1 or 2, NHWC, power-of-two spatial dims and channels) an implicit
// GEMM -- no im2col / col2im matrix ever reaches HBM:
//   kIm2col  S[pixel (b, oh, ow)][tap * C + c]  = x[b][oh*s + kh - 1][ow*s + kw - 1][c]
//   kDgrad   S[pixel (b, h, w)][tap * Co + co]  = dY[b][(h + 1 - kh)/s][(w + 1 - kw)/s][co]
//            (zero unless the division is exact: the stride-2 transposed convolution)
//   kWdgrad  S[ci][tap * Co + co]               = W[tap * Ci + ci][co]
//   kDenseF32 dense f32 storage, rounded to bf16 (RNE) as it is staged (the fp32 tensors of the
//            forward-over-reverse hypergradient step need no separate cast kernels)
enum SrcKind { kDense = 0, kIm2col = 1, kDgrad = 2, kWdgrad = 3, kDenseF32 = 4 };

struct Src {
  const bf16_t* ptr;  // trial 0
  int64_t batch;      // elements between trials
  int ld;             // dense row stride
  int n_outer, n_inner;
  int hl2, wl2;       // log2 of the pixel grid enumerated by 'outer' (gathers)
  int sh_l2, sw_l2;   // log2 of the gathered tensor's spatial dims
  int cl2;            // log2 of the gathered tensor's channels
  int stride;
  int cin;            // kWdgrad: input channels of W
};

template <int KIND>
__device__ __forceinline__ const bf16_t* src_at(const Src& s, const bf16_t* base, int o, int i) {
  if (o >= s.n_outer || i >= s.n_inner) return nullptr;
  if (KIND == kDense) return base + (int64_t)o * s.ld + i;
  const int C = 1 << s.cl2;
  const int tap = i >> s.cl2, c = i & (C - 1);
  const int kh = tap / 3, kw = tap - 3 * kh;
  if (KIND == kWdgrad) return base + ((int64_t)(tap * s.cin + o) << s.cl2) + c;
  const int px = o & ((1 << s.wl2) - 1);
  const int py = (o >> s.wl2) & ((1 << s.hl2) - 1);
  const int b = o >> (s.hl2 + s.wl2);
  int iy, ix;
  if (KIND == kIm2col) {
    iy = py * s.stride + kh - 1;
    ix = px * s.stride + kw - 1;
  } else {  // kDgrad
    const int ny = py + 1 - kh, nx = px + 1 - kw;
    if (s.stride == 2 && ((ny | nx) & 1)) return nullptr;
    iy = s.stride == 2 ? ny >> 1 : ny;
    ix = s.stride == 2 ? nx >> 1 : nx;
  }
  if (iy < 0 || ix < 0 || iy >= (1 << s.sh_l2) || ix >= (1 << s.sw_l2)) return nullptr;
  return base + ((((int64_t)b << s.sh_l2 | iy) << s.sw_l2 | ix) << s.cl2) + c;
}

template <int ROWS, bool KCONTIG, int KIND>
struct Img {
  static constexpr int LS = KCONTIG ? LSK : ROWS + 8;
  static constexpr int ELEMS = KCONTIG ? ROWS * LSK : BK * (ROWS + 8);
  static constexpr int CHUNKS = ROWS * BK / 8;  // 16-byte chunks per tile
  static constexpr int NC = (CHUNKS + 255) / 256;
  static constexpr int RCH = ROWS / 8;          // chunks per k-row of a row-contiguous tile

  // global -> registers: chunk c of the tile starting at (row0, k0); zero outside the matrix and
  // past k_end (the split-K slice)
  __device__ __forceinline__ static void load(uint4 (&r)[NC], const Src& s,
                                              const bf16_t* __restrict__ base, int row0, int k0,
                                              int k_end) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = threadIdx.x + 256 * i;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (c < CHUNKS) {
        int gr, gk;
        if (KCONTIG) {
          gr = row0 + (c >> 3);
          gk = k0 + 8 * (c & 7);
        } else {
          gk = k0 + c / RCH;
          gr = row0 + 8 * (c % RCH);
        }
        if constexpr (KIND == kDenseF32) {
          const int o = KCONTIG ? gr : gk, in = KCONTIG ? gk : gr;
          if (gk < k_end && o < s.n_outer && in < s.n_inner) {
            const float* f = (const float*)base + (int64_t)o * s.ld + in;
            const float4 x0 = *(const float4*)f, x1 = *(const float4*)(f + 4);
            v = make_uint4(pack2bf(x0.x, x0.y), pack2bf(x0.z, x0.w), pack2bf(x1.x, x1.y),
                           pack2bf(x1.z, x1.w));
          }
        } else {
          const bf16_t* src = gk < k_end ? src_at<KIND == kDenseF32 ? kDense : KIND>(
                                               s, base, KCONTIG ? gr : gk, KCONTIG ? gk : gr)
                                         : nullptr;
          if (src != nullptr) v = *(const uint4*)src;
        }
      }
      r[i] = v;
    }
  }

  __device__ __forceinline__ static void store(const uint4 (&r)[NC], bf16_t* img) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = threadIdx.x + 256 * i;
      if (c < CHUNKS) {
        const int off = KCONTIG ? (c >> 3) * LSK + 8 * (c & 7) : (c / RCH) * LS + 8 * (c % RCH);
        *(uint4*)(img + off) = r[i];
      }
    }
  }

  // fragment of rows row16 .. row16+15 (lane li -> row row16 + li), k = 32 s + 8 g .. + 7
  __device__ __forceinline__ static bf16x8 frag(const bf16_t* img, int row16, int s, int li, int g,
                                                int q, int pp) {
    if (KCONTIG) return lds_frag(img + (row16 + li) * LSK + 32 * s + 8 * g);
    const s16x4 lo = lds_tr4(img + (32 * s + 8 * g + q) * LS + row16 + 4 * pp);
    const s16x4 hi = lds_tr4(img + (32 * s + 8 * g + 4 + q) * LS + row16 + 4 * pp);
    return cat_frag(lo, hi);
  }
};

struct GemmArgs {
  Src a, b;
  bf16_t* C;
  float* C32;      // f32 output instead of C (register-staged kernel only), else nullptr
  const float* R32;  // f32 output only: C32 = product + R32 (same layout as C32; may BE C32 --
                     // accumulate in place), nullptr: C32 = product
  float* part;     // split-K partials [splits][P][M][N] (nullptr when splits == 1)
  int64_t sC;
  // two-level batch of the register-staged kernel: batch index p = po * nin + pi, operand X at
  // X + po * X.batch + pi * x_in (nin <= 1: one level, the *_in strides unused)
  int nin;
  int64_t a_in, b_in, c_in;
  int P, M, N, K, ldc;
  int tiles_m, tiles_n, splits, k_per_split, nwg;
  // SwiGLU epilogue of the big-tile kernel (EPI 1, see pgemm_big_kernel): the activation
  // h [P][M][N / 2] written next to C
  bf16_t* H;
  int64_t sX;
  int ldx;
  // RoPE epilogue (EPI 3): cos / sin tables [T][32] f32, sequence length, heads
  const float* cosT;
  const float* sinT;
  int T, nH;
};

__device__ __forceinline__ int64_t boff(int p, int nin, int64_t so, int64_t si) {
  if (nin <= 1) return (int64_t)p * so;
  const int po = p / nin;
  return (int64_t)po * so + (int64_t)(p - po * nin) * si;
}

template <int KA, int KB, bool TA, bool TB, int WM, int FM, int FN>
__global__ __launch_bounds__(256) void pgemm_kernel(const GemmArgs g) {
  constexpr int WN = 4 / WM;
  constexpr int BM = WM * 16 * FM, BN = WN * 16 * FN;
  using IA = Img<BM, !TA, KA>;
  using IB = Img<BN, TB, KB>;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * (IA::ELEMS + IB::ELEMS)];
  constexpr int BUF = IA::ELEMS + IB::ELEMS;  // buffer b: A image at b*BUF, B image after it

  int t = xcd_remap(blockIdx.x, g.nwg);
  const int tn = t % g.tiles_n;
  t /= g.tiles_n;
  const int tm = t % g.tiles_m;
  t /= g.tiles_m;
  const int sp = t % g.splits;
  const int p = t / g.splits;

  // (f32 operands: the trial stride counts f32 elements)
  const int64_t offA = boff(p, g.nin, g.a.batch, g.a_in);
  const int64_t offB = boff(p, g.nin, g.b.batch, g.b_in);
  const int64_t offC = boff(p, g.nin, g.sC, g.c_in);
  const bf16_t* A = KA == kDenseF32 ? (const bf16_t*)((const float*)g.a.ptr + offA)
                                    : g.a.ptr + offA;
  const bf16_t* B = KB == kDenseF32 ? (const bf16_t*)((const float*)g.b.ptr + offB)
                                    : g.b.ptr + offB;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kb = sp * g.k_per_split;
  const int ke = min(g.K, kb + g.k_per_split);
  const int nk = (ke - kb + BK - 1) / BK;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, gq = lane >> 4, q = li >> 2, pp = li & 3;
  const int wm = wave / WN, wn = wave % WN;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[IA::NC], rb[IB::NC];
  IA::load(ra, g.a, A, m0, kb, ke);
  IB::load(rb, g.b, B, n0, kb, ke);
  IA::store(ra, smem);
  IB::store(rb, smem + IA::ELEMS);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      IA::load(ra, g.a, A, m0, kb + (kt + 1) * BK, ke);
      IB::load(rb, g.b, B, n0, kb + (kt + 1) * BK, ke);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        a[i] = IA::frag(smem + cur * BUF, wm * 16 * FM + 16 * i, s, li, gq, q, pp);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        b[j] = IB::frag(smem + cur * BUF + IA::ELEMS, wn * 16 * FN + 16 * j, s, li, gq, q, pp);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
    }
    if (more) {
      IA::store(ra, smem + (cur ^ 1) * BUF);
      IB::store(rb, smem + (cur ^ 1) * BUF + IA::ELEMS);
    }
    __syncthreads();
  }

  // epilogue: lane holds C[row 4 gq + r][col li] of every fragment.  bf16 output is restaged
  // through LDS (the operand buffers are free after the loop's last barrier) so every lane
  // stores whole 16-byte row segments instead of scattered 2-byte elements.
  if (g.splits == 1 && g.C32 != nullptr) {  // f32 output: fragments stored as they are
    float* C = g.C32 + offC;
    const float* R = g.R32 == nullptr ? nullptr : g.R32 + offC;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * 16 * FN + 16 * j + li;
        if (n >= g.N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 16 * FM + 16 * i + 4 * gq + r;
          if (m < g.M) {
            const int64_t o = (int64_t)m * g.ldc + n;
            C[o] = R == nullptr ? acc[i][j][r] : acc[i][j][r] + R[o];
          }
        }
      }
  } else if (g.splits == 1) {
    constexpr int LSC = BN + 8;
    static_assert(BM * LSC <= 2 * BUF, "C tile must fit in the operand buffers");
    bf16_t* Cs = smem;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Cs[(wm * 16 * FM + 16 * i + 4 * gq + r) * LSC + wn * 16 * FN + 16 * j + li] =
              f2bf(acc[i][j][r]);
    __syncthreads();
    bf16_t* C = g.C + offC;
    constexpr int CPR = BN / 8;  // 16-byte chunks per tile row
#pragma unroll
    for (int c = threadIdx.x; c < BM * CPR; c += 256) {
      const int row = c / CPR, cc = c % CPR;
      const int m = m0 + row, n = n0 + 8 * cc;
      if (m < g.M && n < g.N)
        *(uint4*)(C + (int64_t)m * g.ldc + n) = *(const uint4*)(Cs + row * LSC + 8 * cc);
    }
  } else {
    float* C = g.part + ((int64_t)sp * g.P + p) * g.M * g.N;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * 16 * FN + 16 * j + li;
        if (n >= g.N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 16 * FM + 16 * i + 4 * gq + r;
          if (m < g.M) C[(int64_t)m * g.N + n] = acc[i][j][r];
        }
      }
  }
}

// ----------------------------------------------------------------------------------------------
// Large-tile dense GEMM (the LM's projections, head and their gradients): 512 threads = 8 waves
// arranged WM x (8/WM), each wave a 16*FM x 16*FN sub-tile; block tile 256 x 256 (or 256 x 192 / 256 x 128 /
// 128 x 256), BK = 64, one workgroup per CU.  Operand tiles go HBM/L2 -> LDS directly with
// global_load_lds_dwordx4 (no VGPR staging, no ds_write pass): every wave-instruction fills 1 KB
// of the LDS image lane-linearly, so the images are unpadded and bank conflicts are removed by
// XOR-swizzling 16-byte chunks -- the permutation is applied to the per-lane GLOBAL source
// address at the fill and to the ds_read address at the use (the same involution on both sides):
//   * k-contiguous image [rows][64] (128-B rows): chunk c of row r lives at c ^ ((r >> 1) & 7),
//     so the 16 rows of an A/B fragment read (ds_read_b128) hit 16 distinct 16-byte bank slots;
//   * row-contiguous image [64 k][rows]: chunk c of k-row kr lives at c ^ swz(kr), swz spreading
//     the 4 k-rows (and the two lane groups) of a ds_read_b64_tr_b16 over distinct bank slots.
// Two LDS stages: the fills of tile t+1 are in flight while tile t is multiplied; every wave
// waits for its own fills (vmcnt(0)) and the barrier publishes them.
// Preconditions (checked on the host): M % BM == 0, N % BN == 0, K % 64 == 0 (per split), row
// strides multiples of 8 elements, 16-byte aligned bases.
// ----------------------------------------------------------------------------------------------
constexpr int kGroupM = 8;   // row panels per tile group (4 / 16 measured slower, round 3)

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ int kc_swz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int rc_swz(int kr) { return ((kr & 3) << 1) | (((kr >> 3) & 1) << 3); }

// global_load_lds_dwordx4 as inline asm (M0 = the wave's LDS destination).  Through the builtin,
// hipcc (ROCm 7.2) tracks the fill as an LDS DMA and, unable to separate it from the transposed
// reads (ds_read_b64_tr_b16) of the other stage, waits vmcnt(0) before them -- draining the next
// tile's fills at the top of every K-step, which serialised loads and MFMAs on the NN / TN
// layouts (20-30 % slower than NT).  Issued from asm the fills are invisible to the waitcnt pass;
// the K loop waits for them itself (vmcnt(0) before its barrier).
__device__ __forceinline__ void glds16(const bf16_t* src, bf16_t* lds_dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((lds_void*)lds_dst));
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(src), "s"(m0)
               : "memory", "m0");
}

// k-contiguous image with 32-element (64-B) rows: 4 chunks per row; the swizzle keeps the 16
// rows of a fragment read on 16 distinct 16-byte slots of the 256-B bank line (and each 8-row
// half on 8 distinct slots of a 128-B line)
__device__ __forceinline__ int kc_swz32(int row) { return ((row >> 1) ^ (row >> 3)) & 3; }

template <int ROWS, bool KCONTIG, int KD = BK>
struct GImg {
  static_assert(KD == 64 || KD == 32, "image depth");
  static constexpr int ELEMS = ROWS * KD;          // unpadded
  static constexpr int BLOCKS = ELEMS * 2 / 1024;  // 1-KB wave-instruction fills
  static constexpr int NI = BLOCKS / 8;            // fills per wave (8 waves)
  static_assert(NI * 8 == BLOCKS, "tile must split into 8 waves of 1-KB fills");
  static constexpr int CPR = ROWS / 8;             // 16-B chunks per k-row (row-contiguous)
  static_assert(KCONTIG || (CPR >= 16 && CPR % 8 == 0),
                "row-contiguous swizzle needs >= 16 chunks per k-row, whole 8-chunk groups");
  static constexpr int KCH = KD / 8;               // 16-B chunks per row (k-contiguous)

  __device__ __forceinline__ static int kswz(int r) { return KD == 64 ? kc_swz(r) : kc_swz32(r); }
  // row-contiguous swizzle for a 192-wide image (24 chunks: the XOR must stay inside an 8-chunk
  // group).  Its 384-B k-rows shift odd rows by half a 256-B bank line, which already separates
  // k1 & 1; bits 1-2 of the slot then take k1 bit 1 and k1 bit 3, so the 32 lanes of each half
  // of a ds_read_b64_tr_b16 (4 k-rows x 2 lane groups x 2 chunks) hit 16 distinct 16-B slots
  __device__ __forceinline__ static int rswz(int kr) {
    return CPR % 16 == 0 ? rc_swz(kr) : ((((kr >> 1) & 1) << 1) | (((kr >> 3) & 1) << 2));
  }

  // fill this wave's share of the tile whose first row / k is (row0, k0)
  __device__ __forceinline__ static void fill(const bf16_t* __restrict__ base, int ld, int row0,
                                              int k0, bf16_t* img, int wave, int lane) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int blk = wave * NI + j;
      const bf16_t* src;
      if (KCONTIG) {
        const int r = blk * (64 / KCH) + lane / KCH, c = lane % KCH;
        src = base + (int64_t)(row0 + r) * ld + k0 + 8 * (c ^ kswz(r));
      } else {
        const int lin = blk * 64 + lane, kr = lin / CPR, c = lin % CPR;  // lane-linear image
        src = base + (int64_t)(k0 + kr) * ld + row0 + 8 * (c ^ rswz(kr));
      }
      glds16(src, img + blk * 512);
    }
  }

  // fragment of rows row16 .. row16+15, k = 32 s + 8 g .. + 7 (same lane map as Img::frag)
  __device__ __forceinline__ static bf16x8 frag(const bf16_t* img, int row16, int s, int li, int g,
                                                int q, int pp) {
    if (KCONTIG) {
      const int r = row16 + li;
      return lds_frag(img + r * KD + 8 * ((4 * s + g) ^ kswz(r)));
    }
    const int col = row16 + 4 * pp, k1 = 32 * s + 8 * g + q, k2 = k1 + 4;
    const s16x4 lo = lds_tr4(img + k1 * ROWS + 8 * ((col >> 3) ^ rswz(k1)) + (col & 7));
    const s16x4 hi = lds_tr4(img + k2 * ROWS + 8 * ((col >> 3) ^ rswz(k2)) + (col & 7));
    return cat_frag(lo, hi);
  }
};

__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }

// EPI 0: C = A B.  EPI 1, the SwiGLU of the LM's MLP (gate / up in interleaved 16-column
// groups [g0..g15 u0..u15 g16..], so a lane's fragments j (gate) and j + 1 (up) hold the two
// halves of the same four activation columns -- lm_ops.hip swiglu kernels, il = 1): C = gu = A B
// as usual, plus h = silu(g) u into g.H (row stride g.ldx = N / 2) from the bf16-rounded g and
// u -- the separate SwiGLU pass (reads gu, writes h) disappears.  (An EPI 2 writing dgu from the
// dh = dy wdown^T product, g and u loaded per fragment, doubled that GEMM's time and saved
// nothing; removed in round 4, profiles/round4.md.)
template <bool TA, bool TB, int WM, int FM, int FN, int EPI = 0>
__global__ __launch_bounds__(512) void pgemm_big_kernel(const GemmArgs g) {
  constexpr int WN = 8 / WM;
  constexpr int BM = WM * 16 * FM, BN = WN * 16 * FN;
  static_assert(FN % 2 == 0, "the epilogue pairs n-fragments");
  using IA = GImg<BM, !TA>;
  using IB = GImg<BN, TB>;
  constexpr int STAGE = IA::ELEMS + IB::ELEMS;
  __shared__ __attribute__((aligned(1024))) bf16_t smem[2 * STAGE];  // the only __shared__ object

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, gq = lane >> 4, q = li >> 2, pp = li & 3;
  const int wm = wave / WN, wn = wave % WN;
  const int nk = g.k_per_split / BK;

  // Persistent: workgroup b computes the tiles of virtual ids b, b + G, ... (G = grid size, a
  // multiple of 8, so every virtual id of b maps to b's XCD under xcd_remap).
  int vb = blockIdx.x;
  int p = 0, m0 = 0, n0 = 0, k0 = 0;
  // Tile order within a trial: groups of kGroupM row panels, m fastest inside a group, so the
  // tiles an XCD runs together share both their B column panels and a few A row panels in L2
  // (n-fastest order re-streams every B panel from HBM once per row panel).
  auto decode = [&](int v) {
    const int t = xcd_remap(v, g.nwg);
    const int per = g.tiles_m * g.tiles_n;
    const int pq = t / per;           // p * splits + K-split
    p = pq / g.splits;
    k0 = (pq - p * g.splits) * g.k_per_split;
    const int idx = t - pq * per, span = kGroupM * g.tiles_n;
    const int grp = idx / span, in = idx - grp * span;
    const int gm = min(kGroupM, g.tiles_m - grp * kGroupM);
    m0 = (grp * kGroupM + in % gm) * BM;
    n0 = (in / gm) * BN;
  };
  decode(vb);
  IA::fill(g.a.ptr + p * g.a.batch, g.a.ld, m0, k0, smem, wave, lane);
  IB::fill(g.b.ptr + p * g.b.batch, g.b.ld, n0, k0, smem + IA::ELEMS, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  int stage = 0;
  while (true) {
    const int nvb = vb + (int)gridDim.x;
    const bool has_next = nvb < g.nwg;
    int np = p, nm0 = m0, nn0 = n0, nk0 = k0;
    if (has_next) {
      const int cp = p, cm = m0, cn = n0, ck = k0;
      decode(nvb);
      np = p; nm0 = m0; nn0 = n0; nk0 = k0;
      p = cp; m0 = cm; n0 = cn; k0 = ck;
    }
    const bf16_t* A = g.a.ptr + p * g.a.batch;
    const bf16_t* B = g.b.ptr + p * g.b.batch;

    // acc holds C^T fragments (B is the MFMA's A operand): lane (li, gq), register r =
    // C[m = 16 i + li][n = 16 j + 4 gq + r] of the wave's sub-tile -- 4 consecutive columns
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int kt = 0; kt < nk; ++kt) {
      const bf16_t* cur = smem + stage * STAGE;
      bf16_t* nxt = smem + (stage ^ 1) * STAGE;
      // fill the other stage: this tile's next K-step, or the next tile's first one
      if (kt + 1 < nk) {
        IA::fill(A, g.a.ld, m0, k0 + (kt + 1) * BK, nxt, wave, lane);
        IB::fill(B, g.b.ld, n0, k0 + (kt + 1) * BK, nxt + IA::ELEMS, wave, lane);
      } else if (has_next) {
        IA::fill(g.a.ptr + np * g.a.batch, g.a.ld, nm0, nk0, nxt, wave, lane);
        IB::fill(g.b.ptr + np * g.b.batch, g.b.ld, nn0, nk0, nxt + IA::ELEMS, wave, lane);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 a[FM], b[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) a[i] = IA::frag(cur, wm * 16 * FM + 16 * i, s, li, gq, q, pp);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          b[j] = IB::frag(cur + IA::ELEMS, wn * 16 * FN + 16 * j, s, li, gq, q, pp);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(b[j], a[i], acc[i][j]);
      }
      // the fills of the other stage (and the previous tile's C stores) have landed, and every
      // wave is done reading this stage
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      stage ^= 1;
    }

    if (g.part != nullptr) {
      // K-split partial: f32 [splits][P][M][N], lane (li, gq) holds 4 consecutive columns
      const int64_t total = (int64_t)g.P * g.M * g.N;
      float* part = g.part + (k0 / g.k_per_split) * total + (int64_t)p * g.M * g.N +
                    (int64_t)(m0 + wm * 16 * FM + li) * g.N + n0 + wn * 16 * FN + 4 * gq;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) *(f32x4*)(part + (int64_t)(16 * i) * g.N + 16 * j) = acc[i][j];
      if (!has_next) break;
      vb = nvb;
      p = np; m0 = nm0; n0 = nn0; k0 = nk0;
      continue;
    }
    if constexpr (EPI == 3) {
      // lane (li, gq) holds qkv[m][n .. n + 3] of fragment (i, j), n = 16 j + 4 gq (+ origin):
      // section n / d (q, k, v), head (n % d) / 64, head column c = n % 64; the row is token t =
      // m % T of sequence m / T.  q and k are rotated by interleaved pairs (c, c+1), (c+2, c+3)
      // at angles c / 2, c / 2 + 1; out = C + sec (P M d) + ((b' H + head) T + t) 64 + c with
      // b' = p (M / T) + m / T -- the [3][B'][H][T][64] layout the attention kernels read.
      const int dm = g.nH * 64;
      const int64_t sec_stride = (int64_t)g.P * g.M * dm;
      const int bper = g.M / g.T;
      // each lane rotates its own 4 columns, then fragments j, j + 1 are exchanged between the
      // lane rows gq = 0|1 (2|3) by v_permlane16_swap as in the plain epilogue below: every lane
      // holds 8 consecutive columns (one head, 8-aligned) of one row -> one 16-byte store per
      // fragment pair instead of two 8-byte ones (round 6)
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = m0 + wm * 16 * FM + 16 * i + li;
        const int bl = m / g.T, t = m - bl * g.T;
        const int64_t bq = (int64_t)p * bper + bl;
#pragma unroll
        for (int j = 0; j < FN; j += 2) {
          uint32_t pk[2][2];
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const int n = n0 + wn * 16 * FN + 16 * (j + jj) + 4 * gq;
            const int sec = n / dm, c = (n - sec * dm) & 63;
            float x[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] = bf2f(f2bf(acc[i][j + jj][r]));   // qkv as stored
            if (sec < 2) {
              const float* cs = g.cosT + (int64_t)t * 32 + (c >> 1);
              const float* sn = g.sinT + (int64_t)t * 32 + (c >> 1);
#pragma unroll
              for (int q2 = 0; q2 < 2; ++q2) {
                const float a = x[2 * q2], b = x[2 * q2 + 1], co = cs[q2], si = sn[q2];
                x[2 * q2] = a * co - b * si;
                x[2 * q2 + 1] = b * co + a * si;
              }
            }
            pk[jj][0] = pack2bf(x[0], x[1]);
            pk[jj][1] = pack2bf(x[2], x[3]);
          }
          const auto s0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
          const int n8 = n0 + wn * 16 * FN + 16 * j + 16 * (gq & 1) + 8 * (gq >> 1);
          const int sec = n8 / dm, hc = n8 - sec * dm, hh = hc >> 6, c = hc & 63;
          bf16_t* o = g.C + sec * sec_stride + ((bq * g.nH + hh) * g.T + t) * 64 + c;
          *(uint4*)o = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        }
      }
      if (!has_next) break;
      vb = nvb;
      p = np; m0 = nm0; n0 = nn0; k0 = nk0;
      continue;
    }
    if constexpr (EPI == 1) {
      // h[m][(n0 + wn 16 FN) / 2 + 16 (j / 2) + 4 gq + r] from fragments j (gate), j + 1 (up)
      bf16_t* Hp = g.H + p * g.sX + (int64_t)(m0 + wm * 16 * FM + li) * g.ldx +
                   (n0 + wn * 16 * FN) / 2 + 4 * gq;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int j = 0; j < FN; j += 2) {
          float hv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r)
            hv[r] = silu_f(bf2f(f2bf(acc[i][j][r]))) * bf2f(f2bf(acc[i][j + 1][r]));
          *(uint2*)(Hp + (int64_t)(16 * i) * g.ldx + 8 * j) =
              make_uint2(pack2bf(hv[0], hv[1]), pack2bf(hv[2], hv[3]));
        }
      }
    }
    // Epilogue without LDS: pack 4 columns per fragment to bf16, then exchange between the lane
    // rows gq = 0|1 (and 2|3) with v_permlane16_swap so every lane holds 8 consecutive columns of
    // one row; per fragment pair (j, j+1) each row gets 64 contiguous bytes in one dwordx4 store.
    // The stores drain while the next tile's first K-step is multiplied.
    bf16_t* C = g.C + p * g.sC + (int64_t)(m0 + wm * 16 * FM + li) * g.ldc + n0 + wn * 16 * FN +
                16 * (gq & 1) + 8 * (gq >> 1);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int j = 0; j < FN; j += 2) {
        uint32_t x0 = pack2bf(acc[i][j][0], acc[i][j][1]);
        uint32_t x1 = pack2bf(acc[i][j][2], acc[i][j][3]);
        uint32_t y0 = pack2bf(acc[i][j + 1][0], acc[i][j + 1][1]);
        uint32_t y1 = pack2bf(acc[i][j + 1][2], acc[i][j + 1][3]);
        const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
        *(uint4*)(C + (int64_t)(16 * i) * g.ldc + 16 * j) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
      }
    }
    if (!has_next) break;
    vb = nvb;
    p = np; m0 = nm0; n0 = nn0; k0 = nk0;
  }
}

// ----------------------------------------------------------------------------------------------
// Phased 256 x 256 GEMM (cfg 12; round 6).  Same operand images, swizzles, persistent tile walk
// and epilogues as pgemm_big_kernel, but the K loop is cut into phases whose LDS-DMA fills stay
// in flight across the barriers (a counted vmcnt, never 0 in the loop) and whose fragment reads
// are issued before the barrier that precedes their MFMAs:
//
//   * the 256 x 64 A and B images of a K-tile are split into half-tiles of 128 rows (A0, A1 =
//     tile rows 0-127 / 128-255, B0, B1 = tile columns 0-127 / 128-255), 16 KB each, two LDS
//     buffers of four half-tiles (128 KB);
//   * wave (wm, wn) of the 2 x 4 waves owns rows {wm 64 + 0..63} of BOTH A halves and columns
//     {wn 32 + 0..31} of BOTH B halves, so each quarter of its 128 x 64 output (quadrant (mh, nh))
//     reads exactly one A half and one B half;
//   * one K-tile = 4 phases, one quadrant (16 MFMAs) each, in the order (A0,B0) (A0,B1) (A1,B1)
//     (A1,B0); A fragments are read at phases 1 and 3, B fragments at phases 2 and 4 into the
//     register set the NEXT phase pair uses -- phase 4 reads the next K-tile's B0 -- so two B
//     register sets alternate and two K-tiles make one loop iteration (8 phases);
//   * every phase issues one half-tile fill (2 x 1 KB LDS-DMA per lane) into a slot whose last
//     reads are two phases old -- phase 1: A1 of K-tile g+1, 2: B0 of g+2, 3: A0 of g+2, 4: B1 of
//     g+2 -- and waits vmcnt(8): the fill of four phases ago has landed (four half-tiles stay in
//     flight, ~2k SIMD cycles); it is read at the earliest one phase after that wait;
//   * phase = [fragment reads] [fill] [vmcnt] s_barrier lgkmcnt(0) [16 MFMA] s_barrier, and the
//     waves of row wm = 1 run one barrier behind those of wm = 0 (one extra barrier at the start,
//     wm = 0 one at the end): waves w and w + 4 share a SIMD, so one of them multiplies while the
//     other reads and fills.  With that offset a slot may be refilled two phases after its last
//     read (both rows' reads retired) and read one phase after its retiring wait -- the schedule
//     above keeps two phases of slack on the reads.
// The fills run through the persistent tile walk (the next tile's first K-tiles fill during the
// current tile's last ones).  Epilogue stores sit in the same vmcnt queue: the four phases after
// an epilogue wait vmcnt(8 + S) (S = the epilogue's store instructions per lane, a lower bound),
// and once no fills remain the waits are vmcnt(0).  Preconditions as pgemm_big_kernel, plus
// k_per_split a multiple of 128 (an even number of K-tiles).
// ----------------------------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void ph_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void ph_barrier() { asm volatile("s_barrier" ::: "memory"); }
__device__ __forceinline__ void ph_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <int S>
__device__ __forceinline__ void ph_wait(int mode) {  // 0 steady, 1 after an epilogue, 2 drain
  if (mode == 0) ph_vmcnt<8>();
  else if (mode == 1) ph_vmcnt<8 + S>();
  else ph_vmcnt<0>();
}

// Epilogue of one 256 x 256 tile of pgemm_ph_kernel (then the accumulators are zeroed): lane
// (li, gq) of wave (wm, wn) holds, in acc[mh][nh][i][j], C[m][n .. n + 3] with m = m0 + 128 mh +
// 64 wm + 16 i + li and n = n0 + 128 nh + 32 wn + 16 j + 4 gq -- pgemm_big_kernel's fragment
// layout (C^T fragments), so its store paths carry over with these row / column origins.
template <int EPI>
__device__ __forceinline__ void pgemm_ph_epilogue(const GemmArgs& g, f32x4 (&acc)[2][2][4][2],
                                                  int p, int m0, int n0, int k0, int wm, int wn,
                                                  int li, int gq) {
  if (g.part != nullptr) {  // K-split partial: f32 [splits][P][M][N]
    const int64_t total = (int64_t)g.P * g.M * g.N;
    float* part = g.part + (k0 / g.k_per_split) * total + (int64_t)p * g.M * g.N;
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int m = m0 + 128 * mh + 64 * wm + 16 * i + li;
            const int n = n0 + 128 * nh + 32 * wn + 16 * j + 4 * gq;
            *(f32x4*)(part + (int64_t)m * g.N + n) = acc[mh][nh][i][j];
          }
  } else if constexpr (EPI == 3) {  // QKV + RoPE into [3][B'][H][T][64] (pgemm_big_kernel)
    const int dm = g.nH * 64;
    const int64_t sec_stride = (int64_t)g.P * g.M * dm;
    const int bper = g.M / g.T;
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + 128 * mh + 64 * wm + 16 * i + li;
        const int bl = m / g.T, t = m - bl * g.T;
        const int64_t bq = (int64_t)p * bper + bl;
#pragma unroll
        for (int nh = 0; nh < 2; ++nh)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int n = n0 + 128 * nh + 32 * wn + 16 * j + 4 * gq;
            const int sec = n / dm, hc = n - sec * dm, hh = hc >> 6, c = hc & 63;
            float x[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] = bf2f(f2bf(acc[mh][nh][i][j][r]));
            if (sec < 2) {
              const float* cs = g.cosT + (int64_t)t * 32 + (c >> 1);
              const float* sn = g.sinT + (int64_t)t * 32 + (c >> 1);
#pragma unroll
              for (int q2 = 0; q2 < 2; ++q2) {
                const float a = x[2 * q2], b = x[2 * q2 + 1], co = cs[q2], si = sn[q2];
                x[2 * q2] = a * co - b * si;
                x[2 * q2 + 1] = b * co + a * si;
              }
            }
            bf16_t* o = g.C + sec * sec_stride + ((bq * g.nH + hh) * g.T + t) * 64 + c;
            *(uint2*)o = make_uint2(pack2bf(x[0], x[1]), pack2bf(x[2], x[3]));
          }
      }
  } else {
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int nh = 0; nh < 2; ++nh) {
        const int mr = m0 + 128 * mh + 64 * wm + li;   // row of fragment i = 0
        const int nc = n0 + 128 * nh + 32 * wn;        // first column of the j = 0, 1 pair
        if constexpr (EPI == 1) {  // SwiGLU: j = 0 gate, j = 1 up -> 16 columns of h
          bf16_t* Hp = g.H + p * g.sX + (int64_t)mr * g.ldx + nc / 2 + 4 * gq;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float hv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
              hv[r] = silu_f(bf2f(f2bf(acc[mh][nh][i][0][r]))) * bf2f(f2bf(acc[mh][nh][i][1][r]));
            *(uint2*)(Hp + (int64_t)(16 * i) * g.ldx) =
                make_uint2(pack2bf(hv[0], hv[1]), pack2bf(hv[2], hv[3]));
          }
        }
        // 4 columns per fragment packed, rows gq = 0|1 (2|3) exchanged by v_permlane16_swap:
        // 8 consecutive columns of one row per lane, one 16-byte store per fragment pair
        bf16_t* C = g.C + p * g.sC + (int64_t)mr * g.ldc + nc + 16 * (gq & 1) + 8 * (gq >> 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          uint32_t x0 = pack2bf(acc[mh][nh][i][0][0], acc[mh][nh][i][0][1]);
          uint32_t x1 = pack2bf(acc[mh][nh][i][0][2], acc[mh][nh][i][0][3]);
          uint32_t y0 = pack2bf(acc[mh][nh][i][1][0], acc[mh][nh][i][1][1]);
          uint32_t y1 = pack2bf(acc[mh][nh][i][1][2], acc[mh][nh][i][1][3]);
          const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
          *(uint4*)(C + (int64_t)(16 * i) * g.ldc) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        }
      }
  }
#pragma unroll
  for (int mh = 0; mh < 2; ++mh)
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mh][nh][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

template <bool TA, bool TB, int EPI = 0>
__global__ __launch_bounds__(512) void pgemm_ph_kernel(const GemmArgs g) {
  constexpr int H = 128;                          // rows of a half-tile
  using IA = GImg<H, !TA>;
  using IB = GImg<H, TB>;
  constexpr int SL = H * BK;                      // elements of one half-tile image (16 KB)
  // slot s of buffer b at smem + (2 s + b) SL: s = 0 A0, 1 A1, 2 B0, 3 B1 (both buffers of an
  // operand within 64 KB of its first slot: every fragment read of the kernel is a base
  // register + a 16-bit immediate offset)
  __shared__ __attribute__((aligned(1024))) bf16_t smem[8 * SL];  // the only __shared__ object

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, gq = lane >> 4, q = li >> 2, pp = li & 3;
  const int wm = wave >> 2, wn = wave & 3;
  const int nk = g.k_per_split / BK;              // >= 2 (host check)

  auto decode = [&](int v, int& p, int& m0, int& n0, int& k0) {
    const int t = xcd_remap(v, g.nwg);
    const int per = g.tiles_m * g.tiles_n;
    const int pq = t / per;
    p = pq / g.splits;
    k0 = (pq - p * g.splits) * g.k_per_split;
    const int idx = t - pq * per, span = kGroupM * g.tiles_n;
    const int grp = idx / span, in = idx - grp * span;
    const int gm = min(kGroupM, g.tiles_m - grp * kGroupM);
    m0 = (grp * kGroupM + in % gm) * 256;
    n0 = (in / gm) * 256;
  };
  int vb = blockIdx.x;
  int p, m0, n0, k0;
  decode(vb, p, m0, n0, k0);
  int vn = vb + (int)gridDim.x;
  bool has_next = vn < g.nwg;
  int np = 0, nm0 = 0, nn0 = 0, nk0 = 0;
  if (has_next) decode(vn, np, nm0, nn0, nk0);

  // fill slot s of buffer b with K-tile kt of the current (nx = false) or next tile
  auto fill = [&](int s, int b, bool nx, int kt) {
    const int fp = nx ? np : p, fm = nx ? nm0 : m0, fn = nx ? nn0 : n0;
    const int fk = (nx ? nk0 : k0) + kt * BK;
    bf16_t* img = smem + (2 * s + b) * SL;
    if (s < 2) IA::fill(g.a.ptr + fp * g.a.batch, g.a.ld, fm + s * H, fk, img, wave, lane);
    else IB::fill(g.b.ptr + fp * g.b.batch, g.b.ld, fn + (s - 2) * H, fk, img, wave, lane);
  };
  // the K-tile d ahead of kt: (exists, in the next tile, its k index)
  auto ahead = [&](int kt, int d, bool& nx, int& kk) {
    kk = kt + d;
    nx = kk >= nk;
    if (nx) kk -= nk;
    return !nx || has_next;
  };

  const int S = g.part != nullptr ? 32 : (EPI == 0 ? 16 : 32);  // epilogue stores per lane

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a0 = 0; a0 < 2; ++a0)
#pragma unroll
    for (int a1 = 0; a1 < 2; ++a1)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a0][a1][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[2][4], bx[2][2], by[2][2];  // A fragments [k-sub][i], two B sets [k-sub][j]

  // prologue: the fills a steady state would have issued before K-tile 0's first phase --
  // B0(0) A0(0) B1(0) A1(0) B0(1) A0(1) B1(1) -- the first three retired, B0(0) read into bx
  fill(2, 0, false, 0);
  fill(0, 0, false, 0);
  fill(3, 0, false, 0);
  fill(1, 0, false, 0);
  fill(2, 1, false, 1);
  fill(0, 1, false, 1);
  fill(3, 1, false, 1);
  ph_vmcnt<8>();
  ph_barrier();
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      bx[ks][j] = IB::frag(smem + 4 * SL, wn * 32 + 16 * j, ks, li, gq, q, pp);
  if (wm == 1) ph_barrier();                     // row 1 runs one barrier behind

  int kt = 0;
  int post = 0;                                   // phases left that follow an epilogue

#define PH_READ_A(BUF, HALF)                                                                   \
  _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                             \
    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                              \
      fa[ks][i] = IA::frag(smem + (2 * (HALF) + (BUF)) * SL, wm * 64 + 16 * i, ks, li, gq, q, pp);
#define PH_READ_B(BUF, HALF, BR)                                                               \
  _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                             \
    _Pragma("unroll") for (int j = 0; j < 2; ++j)                                              \
      BR[ks][j] = IB::frag(smem + (2 * (2 + (HALF)) + (BUF)) * SL, wn * 32 + 16 * j, ks, li, gq, q, pp);
  // s_setprio around the cluster: without it hipcc moves MFMAs across the raw barriers in among
  // the next phase's reads and fills, which undoes the ping-pong of the two wave rows
#define PH_MFMA(MH, NH, BR)                                                                    \
  __builtin_amdgcn_s_setprio(1);                                                               \
  _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                             \
    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                              \
      _Pragma("unroll") for (int j = 0; j < 2; ++j)                                            \
        acc[MH][NH][i][j] = mfma16(BR[ks][j], fa[ks][i], acc[MH][NH][i][j]);                   \
  __builtin_amdgcn_s_setprio(0);
  // one phase: FILL is (slot, buffer, K-tiles ahead); the wait mode follows from what is queued
#define PH_STEP(FSLOT, FBUF, FD, MH, NH, BR)                                                   \
  {                                                                                            \
    bool fnx;                                                                                  \
    int fkk;                                                                                   \
    const bool fok = ahead(kt, FD, fnx, fkk);                                                  \
    if (fok) fill(FSLOT, FBUF, fnx, fkk);                                                      \
    const int mode = !fok ? 2 : (post > 0 ? 1 : 0);                                            \
    if (S == 16) ph_wait<16>(mode); else ph_wait<32>(mode);                                    \
    if (post > 0) --post;                                                                      \
    ph_barrier();                                                                              \
    ph_lgkm0();                                                                                \
    PH_MFMA(MH, NH, BR)                                                                        \
    ph_barrier();                                                                              \
  }
  // K-tile in buffer CB (its B0 already in BX): quadrants (0,0) (0,1) (1,1) (1,0); phase 4 reads
  // the next K-tile's B0 into BY.  nk is even (host check): a tile's K-tiles start in buffer 0
  // and its last one is an odd instance, after which the epilogue runs (one code copy)
#define PH_KTILE(CB, BX, BY)                                                                   \
  {                                                                                            \
    PH_READ_A(CB, 0)                                                                           \
    PH_STEP(1, (CB) ^ 1, 1, 0, 0, BX)                                                          \
    PH_READ_B(CB, 1, BY)                                                                       \
    PH_STEP(2, CB, 2, 0, 1, BY)                                                                \
    PH_READ_A(CB, 1)                                                                           \
    PH_STEP(0, CB, 2, 1, 1, BY)                                                                \
    {                                                                                          \
      bool nx1;                                                                                \
      int kk1;                                                                                 \
      if (ahead(kt, 1, nx1, kk1)) { PH_READ_B((CB) ^ 1, 0, BY) }                               \
    }                                                                                          \
    PH_STEP(3, CB, 2, 1, 0, BX)                                                                \
  }
  while (true) {
    PH_KTILE(0, bx, by)
    ++kt;
    PH_KTILE(1, by, bx)
    if (++kt < nk) continue;
    pgemm_ph_epilogue<EPI>(g, acc, p, m0, n0, k0, wm, wn, li, gq);
    if (!has_next) break;
    vb = vn; p = np; m0 = nm0; n0 = nn0; k0 = nk0;
    vn = vb + (int)gridDim.x;
    has_next = vn < g.nwg;
    if (has_next) decode(vn, np, nm0, nn0, nk0);
    kt = 0;
    post = 4;
  }
#undef PH_KTILE
#undef PH_STEP
#undef PH_MFMA
#undef PH_READ_B
#undef PH_READ_A
  if (wm == 0) ph_barrier();                     // equal barrier counts in both rows
}

// (Round 5, two deeper-pipelined variants of this kernel, both correct on every GEMM test and
// both removed (profiles/round5.md): a 3-stage 64-deep LDS ring at 256 x 128 / 128 x 256 (fills
// two K-steps ahead behind counted vmcnt waits, one raw s_barrier per K-step, C stores in inline
// asm so the counts were exact) ran 670-860 TFLOP/s, and a 4-stage 32-deep ring at 256 x 256
// (fills three steps ahead) 610-1009, against 900-1200 for this kernel's best tile on every LM
// shape.  The fill latency is not what holds this loop back: with 32 MFMAs per wave between
// barriers the exposed LDS-read latency after each barrier grew instead.)
// (Round 4: a register-pipelined variant -- the operands of K-step t + 3 loaded into one of two
// register sets while step t is multiplied, written to the free LDS stage two steps later --
// was correct but 2.5-4x slower: the two register sets on top of the accumulators exceed the
// 256 VGPRs of two waves per SIMD and spill; profiles/round4.md.)
// (A multi-stage variant -- BK = 32 images in 4-5 LDS stages, fills 3-4 K-steps ahead -- was
// correct on every layout but 5-25 % slower than this 2-stage kernel on every LM shape; it was
// removed in round 4, the A/B is in profiles/round3.md "LM GEMMs".)

// ----------------------------------------------------------------------------------------------
// The big-tile kernel on v_mfma_f32_32x32x16_bf16 (cfg 13: 256 x 256, cfg 14: 256 x 192; round 6,
// VERDICT r5 item 1), NT layout (A [M][K], B [N][K]: both images k-contiguous) -- the same LDS-DMA
// fills, swizzle, 2-stage loop and persistent tile walk as pgemm_big_kernel, each wave a 32 FM x
// 32 FN sub-tile of 32 x 32 accumulator blocks.  Fragment of a 32-row block for k-sub-step kk
// (16 deep): lane l reads row (l & 31), k = 16 kk + 8 (l >> 5) .. + 7 -- one ds_read_b128 of
// chunk 2 kk + (l >> 5); 16 lanes of one read hit 16 rows of one chunk column, which the
// (r >> 1) & 7 XOR spreads over 16 bank slots, as for the 16x16x32 reads.  The LDS bytes a wave
// reads per K-step are those of its sub-tile's A and B panels under either MFMA shape (a fragment
// is reused across the other operand's blocks); what changes is half the MFMA instructions (32
// cycles each instead of 16) and the C layout: acc (C^T, B the MFMA's A operand) lane l, register
// 4 q + r = C[m = 32 i + (l & 31)][n = 32 j + 8 q + 4 (l >> 5) + r].
// ----------------------------------------------------------------------------------------------
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <int WM, int FM, int FN>
__global__ __launch_bounds__(512) void pgemm_big32_kernel(const GemmArgs g) {
  constexpr int WN = 8 / WM;
  constexpr int BM = WM * 32 * FM, BN = WN * 32 * FN;
  static_assert(FN * 4 % 2 == 0, "stores pair the 8-column groups");
  using IA = GImg<BM, true>;
  using IB = GImg<BN, true>;
  constexpr int STAGE = IA::ELEMS + IB::ELEMS;
  __shared__ __attribute__((aligned(1024))) bf16_t smem[2 * STAGE];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int wm = wave / WN, wn = wave % WN;
  const int nk = g.k_per_split / BK;

  int vb = blockIdx.x;
  int p = 0, m0 = 0, n0 = 0, k0 = 0;
  auto decode = [&](int v) {
    const int t = xcd_remap(v, g.nwg);
    const int per = g.tiles_m * g.tiles_n;
    const int pq = t / per;
    p = pq / g.splits;
    k0 = (pq - p * g.splits) * g.k_per_split;
    const int idx = t - pq * per, span = kGroupM * g.tiles_n;
    const int grp = idx / span, in = idx - grp * span;
    const int gm = min(kGroupM, g.tiles_m - grp * kGroupM);
    m0 = (grp * kGroupM + in % gm) * BM;
    n0 = (in / gm) * BN;
  };
  // fragment of the 32-row block starting at row32, k-sub-step kk
  auto frag = [&](const bf16_t* img, int row32, int kk) {
    const int r = row32 + lr;
    return lds_frag(img + r * BK + 8 * ((2 * kk + lh) ^ kc_swz(r)));
  };
  decode(vb);
  IA::fill(g.a.ptr + p * g.a.batch, g.a.ld, m0, k0, smem, wave, lane);
  IB::fill(g.b.ptr + p * g.b.batch, g.b.ld, n0, k0, smem + IA::ELEMS, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  int stage = 0;
  while (true) {
    const int nvb = vb + (int)gridDim.x;
    const bool has_next = nvb < g.nwg;
    int np = p, nm0 = m0, nn0 = n0, nk0 = k0;
    if (has_next) {
      const int cp = p, cm = m0, cn = n0, ck = k0;
      decode(nvb);
      np = p; nm0 = m0; nn0 = n0; nk0 = k0;
      p = cp; m0 = cm; n0 = cn; k0 = ck;
    }
    const bf16_t* A = g.a.ptr + p * g.a.batch;
    const bf16_t* B = g.b.ptr + p * g.b.batch;
    f32x16 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    for (int kt = 0; kt < nk; ++kt) {
      const bf16_t* cur = smem + stage * STAGE;
      bf16_t* nxt = smem + (stage ^ 1) * STAGE;
      if (kt + 1 < nk) {
        IA::fill(A, g.a.ld, m0, k0 + (kt + 1) * BK, nxt, wave, lane);
        IB::fill(B, g.b.ld, n0, k0 + (kt + 1) * BK, nxt + IA::ELEMS, wave, lane);
      } else if (has_next) {
        IA::fill(g.a.ptr + np * g.a.batch, g.a.ld, nm0, nk0, nxt, wave, lane);
        IB::fill(g.b.ptr + np * g.b.batch, g.b.ld, nn0, nk0, nxt + IA::ELEMS, wave, lane);
      }
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        bf16x8 a[FM], b[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) a[i] = frag(cur, wm * 32 * FM + 32 * i, kk);
#pragma unroll
        for (int j = 0; j < FN; ++j) b[j] = frag(cur + IA::ELEMS, wn * 32 * FN + 32 * j, kk);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = mfma32(b[j], a[i], acc[i][j]);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      stage ^= 1;
    }

    const int mrow = m0 + wm * 32 * FM + lr;
    const int ncol = n0 + wn * 32 * FN;
    if (g.part != nullptr) {
      const int64_t total = (int64_t)g.P * g.M * g.N;
      float* part = g.part + (k0 / g.k_per_split) * total + (int64_t)p * g.M * g.N +
                    (int64_t)mrow * g.N + ncol + 4 * lh;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            *(f32x4*)(part + (int64_t)(32 * i) * g.N + 32 * j + 8 * q) =
                f32x4{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2],
                      acc[i][j][4 * q + 3]};
    } else {
      // groups q (lane half h holds columns 8 q + 4 h .. + 3): v_permlane32_swap of the packed
      // groups q, q + 1 gives lane l < 32 columns 8 q .. + 7 and lane l + 32 columns 8 (q + 1)
      // .. + 7 of row l -- one 16-byte store per lane per group pair
      bf16_t* C = g.C + p * g.sC + (int64_t)mrow * g.ldc + ncol + 8 * lh;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int q = 0; q < 4; q += 2) {
            const uint32_t x0 = pack2bf(acc[i][j][4 * q], acc[i][j][4 * q + 1]);
            const uint32_t x1 = pack2bf(acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]);
            const uint32_t y0 = pack2bf(acc[i][j][4 * q + 4], acc[i][j][4 * q + 5]);
            const uint32_t y1 = pack2bf(acc[i][j][4 * q + 6], acc[i][j][4 * q + 7]);
            const auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
            const auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
            *(uint4*)(C + (int64_t)(32 * i) * g.ldc + 32 * j + 8 * q) =
                make_uint4(s0[0], s1[0], s0[1], s1[1]);
          }
    }
    if (!has_next) break;
    vb = nvb;
    p = np; m0 = nm0; n0 = nn0; k0 = nk0;
  }
}

// sum of the split-K partials [splits][P][M][N] -> C[p][m][n * ldc] bf16
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part,
                                                            bf16_t* __restrict__ C,
                                                            float* C32, const float* R32,
                                                            int64_t sC, int ldc, int P, int M,
                                                            int N, int splits, int nin,
                                                            int64_t c_in) {
  const int64_t total = (int64_t)P * M * N;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += part[k * total + i];
  const int64_t n = i % N, m = (i / N) % M, p = i / ((int64_t)M * N);
  const int64_t o = boff((int)p, nin, sC, c_in) + m * ldc + n;
  if (C32 != nullptr) C32[o] = R32 == nullptr ? s : s + R32[o];
  else C[o] = f2bf(s);
}

template <int KA, int KB, bool TA, bool TB, int WM, int FM, int FN>
int launch(GemmArgs g, hipStream_t st) {
  constexpr int BM = WM * 16 * FM, BN = (4 / WM) * 16 * FN;
  g.tiles_m = (g.M + BM - 1) / BM;
  g.tiles_n = (g.N + BN - 1) / BN;
  const int64_t nwg = (int64_t)g.P * g.splits * g.tiles_m * g.tiles_n;
  if (nwg <= 0 || nwg > 0x7FFFFFFF) return (int)hipErrorInvalidValue;
  g.nwg = (int)nwg;
  hipLaunchKernelGGL((pgemm_kernel<KA, KB, TA, TB, WM, FM, FN>), dim3(g.nwg), dim3(256), 0, st,
                     g);
  return (int)hipGetLastError();
}

template <bool TA, bool TB, int WM, int FM, int FN, int EPI = 0>
int launch_big(GemmArgs g, hipStream_t st) {
  constexpr int BM = WM * 16 * FM, BN = (8 / WM) * 16 * FN;
  if (g.M % BM || g.N % BN || g.k_per_split % BK || g.k_per_split < BK ||
      (int64_t)g.k_per_split * g.splits != g.K || (g.splits > 1 && g.part == nullptr) ||
      g.nin > 1 || (EPI != 0 && g.splits != 1) || (EPI == 1 && g.H == nullptr) ||
      (EPI == 3 && (g.cosT == nullptr || g.T <= 0 || g.M % g.T || g.N != 3 * 64 * g.nH)))
    return (int)hipErrorInvalidValue;
  g.tiles_m = g.M / BM;
  g.tiles_n = g.N / BN;
  const int64_t nwg = (int64_t)g.P * g.splits * g.tiles_m * g.tiles_n;
  if (nwg <= 0 || nwg > 0x7FFFFFFF) return (int)hipErrorInvalidValue;
  g.nwg = (int)nwg;
  // persistent: one workgroup per CU (the LDS stages allow no second one), a multiple of 8
  constexpr int kGrid = 256;
  const int grid = nwg < kGrid ? (int)nwg : kGrid;
  hipLaunchKernelGGL((pgemm_big_kernel<TA, TB, WM, FM, FN, EPI>), dim3(grid), dim3(512), 0, st, g);
  return (int)hipGetLastError();
}

template <bool TA, bool TB, int WM, int FM, int FN>
int launch_big32(GemmArgs g, hipStream_t st) {
  if constexpr (TA || !TB) {
    return (int)hipErrorNotSupported;          // NT only (both images k-contiguous)
  } else {
    constexpr int BM = WM * 32 * FM, BN = (8 / WM) * 32 * FN;
    if (g.M % BM || g.N % BN || g.k_per_split % BK || g.k_per_split < BK ||
        (int64_t)g.k_per_split * g.splits != g.K || (g.splits > 1 && g.part == nullptr) ||
        g.nin > 1)
      return (int)hipErrorInvalidValue;
    g.tiles_m = g.M / BM;
    g.tiles_n = g.N / BN;
    const int64_t nwg = (int64_t)g.P * g.splits * g.tiles_m * g.tiles_n;
    if (nwg <= 0 || nwg > 0x7FFFFFFF) return (int)hipErrorInvalidValue;
    g.nwg = (int)nwg;
    constexpr int kGrid = 256;
    const int grid = nwg < kGrid ? (int)nwg : kGrid;
    hipLaunchKernelGGL((pgemm_big32_kernel<WM, FM, FN>), dim3(grid), dim3(512), 0, st, g);
    return (int)hipGetLastError();
  }
}

template <bool TA, bool TB, int EPI = 0>
int launch_ph(GemmArgs g, hipStream_t st) {
  if (g.M % 256 || g.N % 256 || g.k_per_split % (2 * BK) || g.k_per_split < 2 * BK ||
      (int64_t)g.k_per_split * g.splits != g.K || (g.splits > 1 && g.part == nullptr) ||
      g.nin > 1 || (EPI != 0 && g.splits != 1) || (EPI == 1 && g.H == nullptr) ||
      (EPI == 3 && (g.cosT == nullptr || g.T <= 0 || g.M % g.T || g.N != 3 * 64 * g.nH)))
    return (int)hipErrorInvalidValue;
  g.tiles_m = g.M / 256;
  g.tiles_n = g.N / 256;
  const int64_t nwg = (int64_t)g.P * g.splits * g.tiles_m * g.tiles_n;
  if (nwg <= 0 || nwg > 0x7FFFFFFF) return (int)hipErrorInvalidValue;
  g.nwg = (int)nwg;
  constexpr int kGrid = 256;   // persistent, one workgroup per CU (128 KB of LDS)
  const int grid = nwg < kGrid ? (int)nwg : kGrid;
  hipLaunchKernelGGL((pgemm_ph_kernel<TA, TB, EPI>), dim3(grid), dim3(512), 0, st, g);
  return (int)hipGetLastError();
}

template <int KA, int KB, bool TA, bool TB>
int dispatch_tile(const GemmArgs& g, int cfg, hipStream_t st) {
  if constexpr (KA == kDense && KB == kDense) {
    switch (cfg) {
      case 12: return launch_ph<TA, TB>(g, st);                // 256 x 256, phased
      case 5: return launch_big<TA, TB, 2, 8, 4>(g, st);  // 256 x 256
      case 6: return launch_big<TA, TB, 4, 4, 4>(g, st);  // 256 x 128
      case 7: return launch_big<TA, TB, 2, 4, 4>(g, st);  // 128 x 256
      case 11: return launch_big<TA, TB, 4, 4, 6>(g, st);     // 256 x 192
      case 13: return launch_big32<TA, TB, 2, 4, 2>(g, st);   // 256 x 256, 32x32x16 MFMA
      case 14: return launch_big32<TA, TB, 4, 2, 3>(g, st);   // 256 x 192, 32x32x16 MFMA
      default: break;
    }
  }
  switch (cfg) {
    case 0: return launch<KA, KB, TA, TB, 2, 4, 4>(g, st);  // 128 x 128
    case 1: return launch<KA, KB, TA, TB, 4, 2, 1>(g, st);  // 128 x 16
    case 2: return launch<KA, KB, TA, TB, 4, 2, 2>(g, st);  // 128 x 32
    case 3: return launch<KA, KB, TA, TB, 4, 1, 4>(g, st);  // 64 x 64
    case 4: return launch<KA, KB, TA, TB, 2, 2, 4>(g, st);  // 64 x 128
    // (256 x 128 and 128 x 256 at one workgroup per CU measured 10-35 % slower on the LM
    //  shapes: this register-staged loop needs the second resident workgroup to hide latency)
    default: return (int)hipErrorInvalidValue;
  }
}

template <int KA, int KB, bool TA, bool TB>
int dispatch_conv_tile(const GemmArgs& g, int cfg, hipStream_t st) {
  switch (cfg) {  // convolution GEMMs have N = channels <= 64
    case 1: return launch<KA, KB, TA, TB, 4, 2, 1>(g, st);
    case 2: return launch<KA, KB, TA, TB, 4, 2, 2>(g, st);
    case 3: return launch<KA, KB, TA, TB, 4, 1, 4>(g, st);
    default: return (int)hipErrorInvalidValue;
  }
}

int finish_splitk(const GemmArgs& g, hipStream_t st) {
  const int64_t total = (int64_t)g.P * g.M * g.N;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     st, (const float*)g.part, g.C, g.C32, g.R32, g.sC, g.ldc, g.P, g.M, g.N,
                     g.splits, g.nin, g.c_in);
  return (int)hipGetLastError();
}

Src dense(const void* ptr, int64_t batch, int ld, int n_outer, int n_inner) {
  Src s{};
  s.ptr = (const bf16_t*)ptr;
  s.batch = batch;
  s.ld = ld;
  s.n_outer = n_outer;
  s.n_inner = n_inner;
  return s;
}

int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return (1 << l) == v ? l : -1;
}

}  // namespace

extern "C" {

// Tile of configuration ``cfg`` (rows, cols): lets the host size grids and split-K.
int mopt_pgemm_tile(int cfg, int* bm, int* bn) {
  static const int t[15][2] = {{128, 128}, {128, 16},  {128, 32},  {64, 64},
                               {64, 128},  {256, 256}, {256, 128}, {128, 256},
                               {256, 256}, {256, 256}, {256, 128}, {256, 192},
                               {256, 256}, {256, 256}, {256, 192}};
  if (cfg < 0 || cfg > 14) return (int)hipErrorInvalidValue;
  *bm = t[cfg][0];
  *bn = t[cfg][1];
  return 0;
}

// C[p] = op(A[p]) . op(B[p]); ta: A stored [K][M] (else [M][K]); tb: B stored [N][K] (else
// [K][N]).  Contiguous-dimension extents must be multiples of 8 and every row 16-byte aligned;
// k_per_split a multiple of 64 (splits > 1 needs ``part`` = f32 [splits][P][M][N]).
int mopt_pgemm(const void* A, const void* B, void* C, void* part, int P, int M, int N, int K,
               int lda, int ldb, int ldc, int64_t sA, int64_t sB, int64_t sC, int ta, int tb,
               int cfg, int splits, int k_per_split, void* stream) {
  if (P <= 0 || M <= 0 || N <= 0 || K <= 0) return 0;
  if (splits < 1 || (splits > 1 && (part == nullptr || k_per_split % BK))) {
    return (int)hipErrorInvalidValue;
  }
  hipStream_t st = (hipStream_t)stream;
  GemmArgs g{};
  g.a = ta ? dense(A, sA, lda, K, M) : dense(A, sA, lda, M, K);
  g.b = tb ? dense(B, sB, ldb, N, K) : dense(B, sB, ldb, K, N);
  g.C = (bf16_t*)C;
  g.part = (float*)part;
  g.sC = sC;
  g.P = P; g.M = M; g.N = N; g.K = K; g.ldc = ldc;
  g.splits = splits;
  g.k_per_split = splits > 1 ? k_per_split : K;
  int err;
  if (!ta && !tb) err = dispatch_tile<kDense, kDense, false, false>(g, cfg, st);
  else if (!ta && tb) err = dispatch_tile<kDense, kDense, false, true>(g, cfg, st);
  else if (ta && !tb) err = dispatch_tile<kDense, kDense, true, false>(g, cfg, st);
  else err = dispatch_tile<kDense, kDense, true, true>(g, cfg, st);
  if (err || splits == 1) return err;
  return finish_splitk(g, st);
}

// The SwiGLU epilogue of the big-tile kernel (pgemm_big_kernel EPI 1): C = A B (the gate / up
// product [M][N], interleaved 16-column groups) and X = h [M][N / 2] (row stride ldx, batch
// stride sX).  Big-tile configurations (5, 6, 7, 11) of an NN product without K splits only --
// hipErrorNotSupported otherwise (the caller then runs pgemm + the swiglu kernel with il = 1).
int mopt_pgemm_swiglu(const void* A, const void* B, void* C, void* X, int P, int M, int N, int K,
                      int lda, int ldb, int ldc, int ldx, int64_t sA, int64_t sB, int64_t sC,
                      int64_t sX, int cfg, void* stream) {
  if (P <= 0 || M <= 0 || N <= 0 || K <= 0) return 0;
  if (N % 32) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  GemmArgs g{};
  g.a = dense(A, sA, lda, M, K);
  g.b = dense(B, sB, ldb, K, N);
  g.C = (bf16_t*)C;
  g.sC = sC;
  g.P = P; g.M = M; g.N = N; g.K = K; g.ldc = ldc;
  g.splits = 1;
  g.k_per_split = K;
  g.H = (bf16_t*)X;
  g.sX = sX;
  g.ldx = ldx;
  switch (cfg) {
    case 5: return launch_big<false, false, 2, 8, 4, 1>(g, st);
    case 6: return launch_big<false, false, 4, 4, 4, 1>(g, st);
    case 7: return launch_big<false, false, 2, 4, 4, 1>(g, st);
    case 11: return launch_big<false, false, 4, 4, 6, 1>(g, st);
    case 12: return launch_ph<false, false, 1>(g, st);
    default: return (int)hipErrorNotSupported;
  }
}

// The QKV projection with RoPE in the big-tile GEMM's epilogue (pgemm_big_kernel EPI 3):
// out [3][P (M / T)][H][T][64] = the q, k, v heads of A [P][M][d] @ B [P][d][3 d] (d = 64 H),
// q and k rotated by interleaved pairs (cos / sin [T][32]).  NN, big tiles without K splits
// (M a multiple of T) -- hipErrorNotSupported otherwise (the caller runs pgemm + mopt_rope_fwd
// with il = 1).
int mopt_pgemm_qkv_rope(const void* A, const void* B, void* out, const void* cosT,
                        const void* sinT, int P, int M, int K, int T, int nH, int lda, int ldb,
                        int64_t sA, int64_t sB, int cfg, void* stream) {
  const int N = 3 * 64 * nH;
  if (P <= 0 || M <= 0 || K <= 0) return 0;
  if (T <= 0 || M % T) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  GemmArgs g{};
  g.a = dense(A, sA, lda, M, K);
  g.b = dense(B, sB, ldb, K, N);
  g.C = (bf16_t*)out;
  g.P = P; g.M = M; g.N = N; g.K = K; g.ldc = N;
  g.splits = 1;
  g.k_per_split = K;
  g.cosT = (const float*)cosT;
  g.sinT = (const float*)sinT;
  g.T = T;
  g.nH = nH;
  switch (cfg) {
    case 5: return launch_big<false, false, 2, 8, 4, 3>(g, st);
    case 6: return launch_big<false, false, 4, 4, 4, 3>(g, st);
    case 7: return launch_big<false, false, 2, 4, 4, 3>(g, st);
    case 11: return launch_big<false, false, 4, 4, 6, 3>(g, st);
    case 12: return launch_ph<false, false, 3>(g, st);
    default: return (int)hipErrorNotSupported;
  }
}

// mopt_pgemm with f32 operands and f32 output (a32/b32/c32 all 1; the register-staged tiles
// only, cfg 0..4): operands are rounded to bf16 as they are staged, accumulation f32.
// ``res``: C = product + res (res laid out as C; res == C accumulates in place), or nullptr.
// Two-level batch (nin > 1): P counts outer x inner problems, problem p = po * nin + pi reads
// A + po * sA + pi * sA_in (likewise B, C / res); strides may be 0 (a broadcast operand).
int mopt_pgemm_f32b(const void* A, const void* B, void* C, const void* res, void* part, int P,
                    int M, int N, int K, int lda, int ldb, int ldc, int64_t sA, int64_t sB,
                    int64_t sC, int ta, int tb, int cfg, int splits, int k_per_split, int nin,
                    int64_t sA_in, int64_t sB_in, int64_t sC_in, void* stream) {
  if (P <= 0 || M <= 0 || N <= 0 || K <= 0) return 0;
  if (cfg < 0 || cfg > 4 || splits < 1 ||
      (splits > 1 && (part == nullptr || k_per_split % BK))) {
    return (int)hipErrorInvalidValue;
  }
  hipStream_t st = (hipStream_t)stream;
  GemmArgs g{};
  g.a = ta ? dense(A, sA, lda, K, M) : dense(A, sA, lda, M, K);
  g.b = tb ? dense(B, sB, ldb, N, K) : dense(B, sB, ldb, K, N);
  g.C32 = (float*)C;
  g.R32 = (const float*)res;
  g.nin = nin;
  g.a_in = sA_in;
  g.b_in = sB_in;
  g.c_in = sC_in;
  g.part = (float*)part;
  g.sC = sC;
  g.P = P; g.M = M; g.N = N; g.K = K; g.ldc = ldc;
  g.splits = splits;
  g.k_per_split = splits > 1 ? k_per_split : K;
  int err;
  if (!ta && !tb) err = dispatch_tile<kDenseF32, kDenseF32, false, false>(g, cfg, st);
  else if (!ta && tb) err = dispatch_tile<kDenseF32, kDenseF32, false, true>(g, cfg, st);
  else if (ta && !tb) err = dispatch_tile<kDenseF32, kDenseF32, true, false>(g, cfg, st);
  else err = dispatch_tile<kDenseF32, kDenseF32, true, true>(g, cfg, st);
  if (err || splits == 1) return err;
  return finish_splitk(g, st);
}

int mopt_pgemm_f32r(const void* A, const void* B, void* C, const void* res, void* part, int P,
                    int M, int N, int K, int lda, int ldb, int ldc, int64_t sA, int64_t sB,
                    int64_t sC, int ta, int tb, int cfg, int splits, int k_per_split,
                    void* stream) {
  return mopt_pgemm_f32b(A, B, C, res, part, P, M, N, K, lda, ldb, ldc, sA, sB, sC, ta, tb, cfg,
                         splits, k_per_split, 1, 0, 0, 0, stream);
}

int mopt_pgemm_f32(const void* A, const void* B, void* C, void* part, int P, int M, int N, int K,
                   int lda, int ldb, int ldc, int64_t sA, int64_t sB, int64_t sC, int ta, int tb,
                   int cfg, int splits, int k_per_split, void* stream) {
  return mopt_pgemm_f32r(A, B, C, nullptr, part, P, M, N, K, lda, ldb, ldc, sA, sB, sC, ta, tb,
                         cfg, splits, k_per_split, stream);
}

// Implicit-GEMM 3x3 convolution (pad 1, stride 1|2) of a population, NHWC bf16:
//   kind 0 forward  out y [P*Bn, OH, OW, Co] = conv(x [P*Bn, H, W, Ci], w [P, 9 Ci, Co])
//   kind 1 dgrad    out dx [P*Bn, H, W, Ci]  from dy [P*Bn, OH, OW, Co] and w
//   kind 2 wgrad    out dw [P, 9 Ci, Co]     from x and dy (split-K over pixels: ``part``)
// a / b are (x, w), (dy, w), (x, dy).  H, W, Ci, Co powers of two, Ci >= 8, OH = H / stride.
int mopt_pconv(int kind, const void* a, const void* b, void* out, void* part, int P, int Bn,
               int H, int W, int Ci, int Co, int stride, int cfg, int splits, int k_per_split,
               void* stream) {
  const int hl = ilog2(H), wl = ilog2(W), cil = ilog2(Ci), col = ilog2(Co);
  if (hl < 0 || wl < 0 || cil < 3 || col < 3 || (stride != 1 && stride != 2) ||
      (stride == 2 && (hl < 1 || wl < 1)) || splits < 1 ||
      (splits > 1 && (part == nullptr || k_per_split % BK))) {
    return (int)hipErrorInvalidValue;
  }
  const int ohl = hl - (stride == 2), owl = wl - (stride == 2);
  const int64_t x_batch = (int64_t)Bn << (hl + wl + cil);
  const int64_t y_batch = (int64_t)Bn << (ohl + owl + col);
  const int64_t w_batch = (int64_t)9 * Ci * Co;
  const int out_pix = Bn << (ohl + owl), in_pix = Bn << (hl + wl);
  hipStream_t st = (hipStream_t)stream;
  GemmArgs g{};
  g.C = (bf16_t*)out;
  g.part = (float*)part;
  g.P = P;
  g.splits = splits;
  Src im{};  // x gathered over the output grid
  im.ptr = (const bf16_t*)a;
  im.batch = x_batch;
  im.hl2 = ohl; im.wl2 = owl; im.sh_l2 = hl; im.sw_l2 = wl; im.cl2 = cil; im.stride = stride;
  int err;
  if (kind == 0) {
    g.M = out_pix; g.N = Co; g.K = 9 * Ci; g.ldc = Co; g.sC = y_batch;
    im.n_outer = g.M; im.n_inner = g.K;
    g.a = im;
    g.b = dense(b, w_batch, Co, g.K, Co);
    g.k_per_split = g.K;
    g.splits = 1;
    err = dispatch_conv_tile<kIm2col, kDense, false, false>(g, cfg, st);
    return err;
  }
  if (kind == 1) {
    g.M = in_pix; g.N = Ci; g.K = 9 * Co; g.ldc = Ci; g.sC = x_batch;
    Src dg{};
    dg.ptr = (const bf16_t*)a;
    dg.batch = y_batch;
    dg.n_outer = g.M; dg.n_inner = g.K;
    dg.hl2 = hl; dg.wl2 = wl; dg.sh_l2 = ohl; dg.sw_l2 = owl; dg.cl2 = col; dg.stride = stride;
    Src wd{};
    wd.ptr = (const bf16_t*)b;
    wd.batch = w_batch;
    wd.n_outer = Ci; wd.n_inner = g.K; wd.cl2 = col; wd.cin = Ci;
    g.a = dg;
    g.b = wd;
    g.k_per_split = g.K;
    g.splits = 1;
    return dispatch_conv_tile<kDgrad, kWdgrad, false, true>(g, cfg, st);
  }
  if (kind == 2) {
    g.M = 9 * Ci; g.N = Co; g.K = out_pix; g.ldc = Co; g.sC = w_batch;
    im.n_outer = g.K; im.n_inner = g.M;  // stored [pixel][tap * Ci + c] = [K][M]
    g.a = im;
    g.b = dense(b, y_batch, Co, g.K, Co);
    g.k_per_split = splits > 1 ? k_per_split : g.K;
    err = dispatch_conv_tile<kIm2col, kDense, true, false>(g, cfg, st);
    if (err || splits == 1) return err;
    return finish_splitk(g, st);
  }
  return (int)hipErrorInvalidValue;
}

}  // extern "C"
