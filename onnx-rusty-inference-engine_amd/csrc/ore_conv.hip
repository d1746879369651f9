// Conv (convolution_op.rs:94-517) and MatMul (mul_op.rs:23) on the gfx950 f32 MFMA
// (v_mfma_f32_32x32x2_f32: exact f32, k-ordered fma chain, 157.3 TFLOP/s dense peak).
//
// Implicit GEMM:  Y[m][n] = sum_k Wp[k][m] * B[k][n] (+ bias[m], optional Relu)
//   m = output channel, n = (image, output pixel) flattened, k = (cin, r, s).
//   Weights are packed once into K-major, zero-padded Wp[Kp][Mp] (Kp % 32 == 0, Mp % 128 == 0)
//   so the A tile is a plain 16-B-vectorised copy with no bounds checks.
//   B (the im2col of the input) is never materialised: each K tile gathers it straight from
//   the NCHW input (B1X1: contiguous rows k*x_ps + pix; BGATHER: a per-layer (cin, r, s) offset
//   table read with scalar loads, plus per-column image/row/col bases).
//   Block = 256 threads = 4 waves (WM x WN); block tile BM x BN x BK; LDS double-buffered, the
//   next K tile prefetched into registers while the current one feeds the MFMAs.
//   Fragment maps (cdna_hip_programming.md §3): lane l holds A[l&31][k=l>>5] and
//   B[k=l>>5][l&31]; accumulator register e of lane l is row (e&3)+8*(e>>2)+4*(l>>5), column
//   l&31 -> one register = two 128-B runs of consecutive output pixels.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "ore_kernels.h"

namespace ore {

typedef float floatx16 __attribute__((ext_vector_type(16)));

enum { B1X1 = 0, BGATHER = 1, BGATHER_LDS = 2 };  // BGATHER_LDS: whole gather table in LDS

constexpr int KTAB_LDS = 1024;  // gather-table entries staged in LDS (larger K reads it from global)

template <int BM, int BN, int WM, int WN, int BK, int BMODE>
__global__ __launch_bounds__(256, 2) void conv_gemm_kernel(ConvParams p) {
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 32, FN = TN / 32;
  constexpr int AS = BM + 4;                 // LDS row stride of the A tile (16-B aligned rows)
  constexpr int BROWS = 256 / BN;            // B rows loaded per pass
  constexpr int BLOADS = BK / BROWS;         // B elements per thread per tile
  constexpr int AF4 = BM * BK / 4;           // float4s in the A tile
  constexpr int AVEC = (AF4 + 255) / 256;    // float4 A loads per thread per tile
  static_assert(WM * WN == 4 && FM >= 1 && FN >= 1 && BK % BROWS == 0 && AVEC >= 1, "tile");

  __shared__ __attribute__((aligned(16))) float As[2][BK][AS];
  __shared__ float Bs[2][BK][BN];
  __shared__ float sbias[BM];
  __shared__ int2 ktab_s[BMODE == BGATHER_LDS ? KTAB_LDS : 1];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm0 = (wave / WN) * TM;
  const int wn0 = (wave % WN) * TN;

  // XCD-aware bijective remap (cdna_hip_programming.md §5): consecutive tile ids (M fastest,
  // i.e. the M tiles sharing one B tile) land on one XCD and share its L2.
  const int nwg = p.mtiles * p.ntiles;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, rr8 = nwg & 7;
  const int wgid = (xcd < rr8 ? xcd * (q + 1) : rr8 * (q + 1) + (xcd - rr8) * q) + (bid >> 3);
  const int mt = wgid % p.mtiles;
  const int nt = wgid / p.mtiles;
  const int m0 = mt * BM;
  const int n0 = nt * BN;
  const int K = p.K;
  const int XPS = p.x_ps;  // channel-plane stride of x (>= H*W: planes may be padded)
  const int YPS = p.y_ps;  // channel-plane stride of y = columns iterated per image (>= Ho*Wo)

  for (int i = tid; i < BM; i += 256) sbias[i] = (p.bias && m0 + i < p.M) ? p.bias[m0 + i] : 0.0f;
  const int Kp = (K + 31) & ~31;
  if (BMODE == BGATHER_LDS)
    for (int i = tid; i < Kp; i += 256) ktab_s[i] = p.ktab[i];
  __syncthreads();

  // ---- this thread's B column (Ntot < 2^31 is checked on the host)
  const int bcol = tid % BN;
  const int krow = __builtin_amdgcn_readfirstlane(tid / BN);
  const int bn = n0 + bcol;
  const bool bn_ok = bn < p.Ntot;
  // element offsets fit in 32 bits (checked on the host): uniform base + 32-bit lane offset
  int xoff;
  int ih0 = 0, iw0 = 0;
  {
    const int nn = bn_ok ? bn : 0;
    const int img = nn / YPS;
    const int pix = nn - img * YPS;  // pix >= Ho*Wo: a pad column, computed and never read
    xoff = img * (int)p.x_nstride;
    if (BMODE == B1X1) {
      xoff += pix;
    } else {
      const int oh = pix / p.Wo, ow = pix - oh * p.Wo;
      ih0 = oh * p.sh - p.pt;
      iw0 = ow * p.sw - p.pl;
      xoff += ih0 * p.W + iw0;
    }
  }
  const float* __restrict__ x = p.x;
  const float* __restrict__ wp = p.wp;
  const int2* __restrict__ ktab = p.ktab;

  static_assert(AVEC <= 2, "A tile prefetch holds at most two float4 per thread");

  // Branch-free loads: every lane loads (masked lanes from x[0]) and selects 0 afterwards, so
  // the whole tile's loads issue back to back.
#define ORE_LOAD_TILE(RA0, RA1, RB, ROK, K0)                                                                         \
  {                                                                                                  \
    const int k0_ = (K0);                                                                            \
    {                                                                                                \
      const int kk = tid / (BM / 4), mm = (tid % (BM / 4)) * 4;                                      \
      if (AF4 >= 256 || tid < AF4)                                                                   \
        RA0 = *reinterpret_cast<const float4*>(wp + (unsigned)((k0_ + kk) * p.Mp + m0 + mm));       \
      if (AVEC > 1 && (AF4 >= 512 || tid + 256 < AF4)) {                                             \
        const int e1 = tid + 256, kk1 = e1 / (BM / 4), mm1 = (e1 % (BM / 4)) * 4;                    \
        RA1 = *reinterpret_cast<const float4*>(wp + (unsigned)((k0_ + kk1) * p.Mp + m0 + mm1));     \
      }                                                                                              \
    }                                                                                                \
    _Pragma("unroll") for (int j = 0; j < BLOADS; ++j) {                                             \
      const int k = k0_ + krow + j * BROWS;                                                          \
      bool ok;                                                                                       \
      int off;                                                                                       \
      if (BMODE == B1X1) {                                                                           \
        ok = bn_ok & (k < K);                                                                        \
        off = xoff + k * XPS;                                                                        \
      } else {                                                                                       \
        const int2 e = BMODE == BGATHER_LDS ? ktab_s[k] : ktab[__builtin_amdgcn_readfirstlane(k)];  \
        const int r = e.y >> 16, s = e.y & 0xffff;                                                   \
        ok = bn_ok & ((unsigned)(ih0 + r) < (unsigned)p.H) & ((unsigned)(iw0 + s) < (unsigned)p.W);  \
        off = xoff + e.x;                                                                            \
      }                                                                                              \
      RB[j] = x[(unsigned)(ok ? off : 0)];                                                           \
      ROK[j] = ok;  /* the zero select happens at the LDS store, after the MFMAs */                  \
    }                                                                                                \
  }
#define ORE_STORE_TILE(RA0, RA1, RB, ROK, BUF)                                                                       \
  {                                                                                                  \
    {                                                                                                \
      const int kk = tid / (BM / 4), mm = (tid % (BM / 4)) * 4;                                      \
      if (AF4 >= 256 || tid < AF4) *reinterpret_cast<float4*>(&As[BUF][kk][mm]) = RA0;              \
      if (AVEC > 1 && (AF4 >= 512 || tid + 256 < AF4)) {                                             \
        const int e1 = tid + 256, kk1 = e1 / (BM / 4), mm1 = (e1 % (BM / 4)) * 4;                    \
        *reinterpret_cast<float4*>(&As[BUF][kk1][mm1]) = RA1;                                       \
      }                                                                                              \
    }                                                                                                \
    _Pragma("unroll") for (int j = 0; j < BLOADS; ++j)                                               \
      Bs[BUF][krow + j * BROWS][bcol] = ROK[j] ? RB[j] : 0.0f;                                       \
  }

  floatx16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  const int ntk = (K + BK - 1) / BK;
  {
    float4 ra0, ra1;
    float rb[BLOADS];
    bool rok[BLOADS];
    ORE_LOAD_TILE(ra0, ra1, rb, rok, 0);
    ORE_STORE_TILE(ra0, ra1, rb, rok, 0);
  }
  __syncthreads();
  const int lrow = lane >> 5, lcol = lane & 31;
// fragments for k-step kk+2 are read from LDS before the MFMAs of k-step kk are issued
#define ORE_COMPUTE_TILE(BUF)                                                                        \
  {                                                                                                  \
    float af[2][FM], bf[2][FN];                                                                      \
    _Pragma("unroll") for (int i = 0; i < FM; ++i) af[0][i] = As[BUF][lrow][wm0 + i * 32 + lcol];    \
    _Pragma("unroll") for (int j = 0; j < FN; ++j) bf[0][j] = Bs[BUF][lrow][wn0 + j * 32 + lcol];    \
    _Pragma("unroll") for (int kk = 0; kk < BK; kk += 2) {                                           \
      const int cur = (kk >> 1) & 1;                                                                 \
      if (kk + 2 < BK) {                                                                             \
        _Pragma("unroll") for (int i = 0; i < FM; ++i)                                               \
          af[cur ^ 1][i] = As[BUF][kk + 2 + lrow][wm0 + i * 32 + lcol];                              \
        _Pragma("unroll") for (int j = 0; j < FN; ++j)                                               \
          bf[cur ^ 1][j] = Bs[BUF][kk + 2 + lrow][wn0 + j * 32 + lcol];                              \
      }                                                                                              \
      _Pragma("unroll") for (int i = 0; i < FM; ++i)                                                 \
      _Pragma("unroll") for (int j = 0; j < FN; ++j)                                                 \
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[cur][i], bf[cur][j], acc[i][j], 0, 0, 0); \
    }                                                                                                \
  }
  // steady state: prefetch tile t+1 into registers, MFMAs on tile t, publish t+1 to LDS
  for (int t = 0; t < ntk - 1; ++t) {
    const int buf = t & 1;
    float4 ra0, ra1;
    float rb[BLOADS];
    bool rok[BLOADS];
    ORE_LOAD_TILE(ra0, ra1, rb, rok, (t + 1) * BK);
    __builtin_amdgcn_sched_barrier(0);  // keep the next tile's loads ahead of this tile's MFMAs
    ORE_COMPUTE_TILE(buf);
    ORE_STORE_TILE(ra0, ra1, rb, rok, buf ^ 1);
    __syncthreads();
  }
  ORE_COMPUTE_TILE((ntk - 1) & 1);
#undef ORE_COMPUTE_TILE
#undef ORE_LOAD_TILE
#undef ORE_STORE_TILE

  // ---- epilogue: + bias, optional Relu, scatter to NCHW (possibly a channel slice)
  float* __restrict__ y = p.y;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn0 + j * 32 + lcol;
    if (n >= p.Ntot) continue;
    const int img = n / YPS;
    const int pix = n - img * YPS;
    const unsigned yb = (unsigned)(img * (int)p.y_nstride + pix);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int ml = wm0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * lrow;
        if (m0 + ml < p.M) {
          float v = acc[i][j][e] + sbias[ml];
          if (p.relu) v = fmaxf(v, 0.0f);
          y[yb + (unsigned)((m0 + ml) * YPS)] = v;
        }
      }
    }
  }
}

// ------------------------------------------------------------------ gather table
// ktab[k] = {c*x_ps + r*W + s, (r << 16) | s} for k = (c, r, s) < K; padded entries (k >= K)
// carry r = 1 << 14 so the bounds test of the gather fails and they read as zero.
__global__ __launch_bounds__(256) void ktab_kernel(int2* __restrict__ ktab, int K, int Kp, int kh, int kw, int ps,
                                                   int W) {
  for (int k = blockIdx.x * 256 + threadIdx.x; k < Kp; k += gridDim.x * 256) {
    int2 e = make_int2(0, (1 << 14) << 16);
    if (k < K) {
      const int KK = kh * kw;
      const int c = k / KK, rs = k - c * KK, r = rs / kw, s = rs - r * kw;
      e = make_int2(c * ps + r * W + s, (r << 16) | s);
    }
    ktab[k] = e;
  }
}

void launch_ktab(int2* ktab, int K, int kh, int kw, int x_ps, int W, hipStream_t s) {
  const int Kp = conv_packed_kp(K);
  hipLaunchKernelGGL(ktab_kernel, dim3((Kp + 255) / 256), dim3(256), 0, s, ktab, K, Kp, kh, kw, x_ps, W);
}

// ------------------------------------------------------------------ weight packing
// src ONNX [M][K] (kmajor_src = 0) or MatMul [K][M] (kmajor_src = 1) -> Wp[Kp][Mp], zero padded.
__global__ __launch_bounds__(256) void pack_weights_kernel(const float* __restrict__ w, float* __restrict__ wp,
                                                           int M, int K, int Mp, int Kp, int kmajor_src) {
  const long long total = (long long)Kp * Mp;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int k = (int)(i / Mp), m = (int)(i - (long long)k * Mp);
    float v = 0.0f;
    if (k < K && m < M) v = kmajor_src ? w[(long long)k * M + m] : w[(long long)m * K + k];
    wp[i] = v;
  }
}

int conv_packed_mp(int M) { return (M + 127) / 128 * 128; }
int conv_packed_kp(int K) { return (K + 31) / 32 * 32; }

void launch_pack_weights(const float* w, bool kmajor_src, int M, int K, float* wp, hipStream_t s) {
  const int Mp = conv_packed_mp(M), Kp = conv_packed_kp(K);
  long long total = (long long)Mp * Kp;
  long long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pack_weights_kernel, dim3((unsigned)blocks), dim3(256), 0, s, w, wp, M, K, Mp, Kp,
                     kmajor_src ? 1 : 0);
}

template <int BM, int BN, int WM, int WN, int BK>
static void launch_conv_cfg(const ConvParams& p0, hipStream_t s) {
  ConvParams p = p0;
  p.mtiles = (p.M + BM - 1) / BM;
  p.ntiles = (int)((p.Ntot + BN - 1) / BN);
  dim3 grid(p.mtiles * p.ntiles), block(256);
  if (p.is1x1)
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, BK, B1X1>), grid, block, 0, s, p);
  else if (conv_packed_kp(p.K) <= KTAB_LDS)
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, BK, BGATHER_LDS>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, BK, BGATHER>), grid, block, 0, s, p);
}

// Block tiles, chosen per layer to minimise the padded output channels (MFMA work on rows
// >= M is wasted): BM = 128 (2x2 waves of 64x64), 96 (1x4 waves of 96x32), 64 (2x2 of 32x64),
// 32 (1x4 of 32x64).  Ties go to the larger tile (more reuse of each B element).
int conv_tile_config(int M) {
  static const int bms[4] = {128, 96, 64, 32};
  int best = 0;
  long long best_rows = 1LL << 60;
  for (int i = 0; i < 4; ++i) {
    const long long rows = (long long)((M + bms[i] - 1) / bms[i]) * bms[i];
    if (rows < best_rows) { best_rows = rows; best = i; }
  }
  return best;
}

void launch_conv(const ConvParams& p, hipStream_t s) {
  static int forced = -2;
  if (forced == -2) {
    const char* e = getenv("ORE_CONV_CFG");  // tuning knob: force a tile config (0..3)
    forced = e ? atoi(e) : -1;
  }
  int cfg = conv_tile_config(p.M);
  // short-K layers (SqueezeNet's expand1x1, K <= 64) are epilogue/write bound: the 1x4-wave
  // 96-row tile measured fastest for them even with padded rows (tools/bench_ops.py)
  if (p.K <= 64 && p.M >= 64 && p.is1x1) cfg = 1;
  switch (forced >= 0 ? forced : cfg) {
    case 0: launch_conv_cfg<128, 128, 2, 2, 16>(p, s); break;
    case 1: launch_conv_cfg<96, 128, 1, 4, 16>(p, s); break;
    case 2: launch_conv_cfg<64, 128, 2, 2, 16>(p, s); break;
    default: launch_conv_cfg<32, 256, 1, 4, 16>(p, s); break;
  }
}

}  // namespace ore
