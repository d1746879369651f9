// fp16 variant: f16 activations stored channels-last (NHWC), f16
// weights, f32 accumulation on the CDNA4 f16 matrix cores (v_mfma_f32_32x32x16_f16, 16x the f32
// MFMA rate).  The reference is f32 NCHW only (convolution_op.rs:422-480); the f16 path is ours to
// lay out, and NHWC is what makes its operand gather cheap: with k ordered (r, s, c) -- c fastest --
// the 8 consecutive k of one MFMA fragment lane are 8 consecutive channels of one input pixel,
// i.e. ONE 16-B load, where an NCHW gather needs 8 scattered 2-byte loads with 8 bounds checks.
//
//   conv_f16_kernel<..., F16_X_NHWC_VEC>   every conv on an f16 activation with C % 8 == 0
//   conv_f16_kernel<..., F16_X_NCHW32>     the first conv: the f32 NCHW model input, per-element
//                                          gather in the reference's (c, r, s) order, rounded to f16
//                                          while staging
//   conv_f16_kernel<..., F16_X_NHWC_ELEM>  f16 NHWC input with C % 8 != 0 (per-element, (r, s, c))
//   maxpool_nhwc_kernel / gap_nhwc_kernel / concat_nhwc_kernel: the other f16 steps
//
// Storage of an NHWC value: element (n, c, h, w) at n * nstride + (h * W + w) * cs + c, cs (the
// pixel stride) = the channel count of the root buffer; a Concat slice is the root pointer advanced
// by its first channel.  MFMA operand layouts: lane l holds A[row l&31][k = 8(l>>5) .. +7] and
// B[k = 8(l>>5) .. +7][col l&31]; both LDS tiles are k-contiguous ([row][k], [pixel][k], 80-B
// rows: conflict-free 16-B fragment reads).  Same implicit GEMM as conv_gemm_kernel (M = Cout, N =
// images x output pixels, K = Cin*kh*kw), XCD remap, bias + Relu epilogue in f32, one rounding.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include <type_traits>

#include "ore_kernels.h"

namespace ore {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float floatx16h __attribute__((ext_vector_type(16)));

template <int BM, int BN, int WM, int WN, int XMODE>
__global__ __launch_bounds__(256, 2) void conv_f16_kernel(ConvParams p) {
  constexpr int BK = 32;                 // k per stage: two 32x32x16 k-steps, four 8-k groups
  constexpr int LR = 40;                 // LDS row: 32 halves + 8 pad = 80 B
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 32, FN = TN / 32;
  constexpr int ACH = BM * 4;            // 16-B chunks of one A stage (BM rows x 4 groups)
  constexpr int AV = (ACH + 255) / 256;  // A chunks per thread
  constexpr int BV = BN * 4 / 256;       // B tasks (one pixel x one 8-k group) per thread
  constexpr int QS = 256 / BN;           // per-element modes: k-group stride between a thread's tasks
  constexpr int SR = TM + 8;             // epilogue staging row: one pixel's TM channels + pad (halves)
  constexpr bool VEC = XMODE == F16_X_NHWC_VEC;
  static_assert(WM * WN == 4 && FM >= 1 && FN >= 1 && BN % 64 == 0 && 256 % BN == 0, "tile");
  typedef typename std::conditional<XMODE == F16_X_NCHW32, float, _Float16>::type XT;
  constexpr int MAIN_HALVES = 2 * (BM + BN) * LR, EPI_HALVES = 4 * TN * SR;
  __shared__ __attribute__((aligned(16))) _Float16 smem[MAIN_HALVES > EPI_HALVES ? MAIN_HALVES : EPI_HALVES];
  __shared__ float sbias[BM];
  _Float16(*As)[BM][LR] = reinterpret_cast<_Float16(*)[BM][LR]>(smem);
  _Float16(*Bs)[BN][LR] = reinterpret_cast<_Float16(*)[BN][LR]>(smem + 2 * BM * LR);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm0 = (wave / WN) * TM, wn0 = (wave % WN) * TN;
  const int lrow = lane >> 5, lcol = lane & 31;

  const int nwg = p.mtiles * p.ntiles;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, rr8 = nwg & 7;
  const int wgid = (xcd < rr8 ? xcd * (q8 + 1) : rr8 * (q8 + 1) + (xcd - rr8) * q8) + (bid >> 3);
  const int mt = wgid % p.mtiles, nt = wgid / p.mtiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int Kp = (p.K + 31) & ~31;
  const int P = p.P;  // output pixels per image (columns are dense over pixels)

  for (int i = tid; i < BM; i += 256) sbias[i] = (p.bias && m0 + i < p.M) ? p.bias[m0 + i] : 0.0f;

  // B tasks.  VEC: lane group g = tid & 3 (fixed), pixels (tid >> 2) + 64u: four lanes read 64
  // contiguous bytes of one pixel.  Per-element: pixel tid % BN, k groups qbase + QS*u (uniform).
  constexpr int NPX = VEC ? BV : 1;
  const int g = tid & 3;
  const int bcol0 = VEC ? (tid >> 2) : (tid % BN);
  const int qbase = __builtin_amdgcn_readfirstlane(tid / BN);
  int xoff[NPX], ih0[NPX], iw0[NPX];
  bool nok[NPX];
#pragma unroll
  for (int u = 0; u < NPX; ++u) {
    const int bn = n0 + bcol0 + 64 * u;
    nok[u] = bn < p.Ntot;
    const int nn = nok[u] ? bn : 0;
    const int img = nn / P;
    const int pix = nn - img * P;
    const int oh = pix / p.Wo, ow = pix - oh * p.Wo;
    ih0[u] = oh * p.sh - p.pt;
    iw0[u] = ow * p.sw - p.pl;
    xoff[u] = img * (int)p.x_nstride + (ih0[u] * p.W + iw0[u]) * (XMODE == F16_X_NCHW32 ? 1 : p.x_ps);
  }
  const XT* __restrict__ x = reinterpret_cast<const XT*>(p.x);
  const _Float16* __restrict__ wh = reinterpret_cast<const _Float16*>(p.wp);  // [Mp][Kp]
  typedef const __attribute__((address_space(4))) long long* ktab_cptr;
  const ktab_cptr ktab = (ktab_cptr)p.ktab;  // per k, or per 8-k group (VEC)

#define ORE_H_LOADA(RA, K0)                                                                          \
  _Pragma("unroll") for (int v_ = 0; v_ < AV; ++v_) {                                                \
    const int c_ = (ACH % 256 == 0 || tid + v_ * 256 < ACH) ? tid + v_ * 256 : 0;                    \
    RA[v_] = *reinterpret_cast<const half8*>(wh + (unsigned)((m0 + (c_ >> 2)) * Kp + (K0) + (c_ & 3) * 8)); \
  }
#define ORE_H_STOREA(RA, BUF)                                                                        \
  _Pragma("unroll") for (int v_ = 0; v_ < AV; ++v_) {                                                \
    const int c_ = tid + v_ * 256;                                                                   \
    if (ACH % 256 == 0 || c_ < ACH) *reinterpret_cast<half8*>(&As[BUF][c_ >> 2][(c_ & 3) * 8]) = RA[v_]; \
  }
  // VEC B: the four group entries of the stage by scalar loads, this lane's picked by g; a tap
  // outside the image (or a group past K: r = 1 << 14) is stored as zeros
#define ORE_H_LOADB_VEC(RB, ROK, K0)                                                                 \
  {                                                                                                  \
    const int kb_ = (K0) >> 3;                                                                       \
    const long long e0_ = ktab[kb_], e1_ = ktab[kb_ + 1], e2_ = ktab[kb_ + 2], e3_ = ktab[kb_ + 3];  \
    const long long w_ = g == 0 ? e0_ : g == 1 ? e1_ : g == 2 ? e2_ : e3_;                           \
    const int ex_ = (int)w_, ey_ = (int)(w_ >> 32);                                                  \
    const int r_ = ey_ >> 16, s_ = ey_ & 0xffff;                                                     \
    _Pragma("unroll") for (int u_ = 0; u_ < BV; ++u_) {                                              \
      const bool ok_ = nok[u_] & ((unsigned)(ih0[u_] + r_) < (unsigned)p.H) &                        \
                       ((unsigned)(iw0[u_] + s_) < (unsigned)p.W);                                   \
      RB[u_] = *reinterpret_cast<const half8*>(x + (unsigned)(ok_ ? xoff[u_] + ex_ : 0));            \
      ROK[u_] = ok_;                                                                                 \
    }                                                                                                \
  }
#define ORE_H_STOREB_VEC(RB, ROK, BUF)                                                               \
  _Pragma("unroll") for (int u_ = 0; u_ < BV; ++u_) {                                                \
    const half8 z_ = {};                                                                             \
    *reinterpret_cast<half8*>(&Bs[BUF][bcol0 + 64 * u_][g * 8]) = ROK[u_] ? RB[u_] : z_;             \
  }
  // per-element B: 8 scattered loads per task through the per-k table (uniform k)
#define ORE_H_LOADB_ELEM(RB, ROK, K0)                                                                \
  _Pragma("unroll") for (int u_ = 0; u_ < BV; ++u_) {                                                \
    const int kg_ = (K0) + (qbase + u_ * QS) * 8;                                                    \
    _Pragma("unroll") for (int e_ = 0; e_ < 8; ++e_) {                                               \
      const long long w_ = ktab[kg_ + e_];                                                           \
      const int ex_ = (int)w_, ey_ = (int)(w_ >> 32);                                                \
      const int r_ = ey_ >> 16, s_ = ey_ & 0xffff;                                                   \
      const bool ok_ = nok[0] & ((unsigned)(ih0[0] + r_) < (unsigned)p.H) &                          \
                       ((unsigned)(iw0[0] + s_) < (unsigned)p.W);                                    \
      RB[u_ * 8 + e_] = x[(unsigned)(ok_ ? xoff[0] + ex_ : 0)];                                      \
      ROK[u_ * 8 + e_] = ok_;                                                                        \
    }                                                                                                \
  }
#define ORE_H_STOREB_ELEM(RB, ROK, BUF)                                                              \
  _Pragma("unroll") for (int u_ = 0; u_ < BV; ++u_) {                                                \
    half8 h_;                                                                                        \
    _Pragma("unroll") for (int e_ = 0; e_ < 8; ++e_)                                                 \
      h_[e_] = ROK[u_ * 8 + e_] ? (_Float16)RB[u_ * 8 + e_] : (_Float16)0.0f;                        \
    *reinterpret_cast<half8*>(&Bs[BUF][bcol0][(qbase + u_ * QS) * 8]) = h_;                          \
  }
#define ORE_H_COMPUTE(BUF)                                                                           \
  _Pragma("unroll") for (int ks = 0; ks < BK; ks += 16) {                                            \
    half8 af[FM], bf[FN];                                                                            \
    _Pragma("unroll") for (int i = 0; i < FM; ++i)                                                   \
      af[i] = *reinterpret_cast<const half8*>(&As[BUF][wm0 + i * 32 + lcol][ks + 8 * lrow]);         \
    _Pragma("unroll") for (int j = 0; j < FN; ++j)                                                   \
      bf[j] = *reinterpret_cast<const half8*>(&Bs[BUF][wn0 + j * 32 + lcol][ks + 8 * lrow]);         \
    _Pragma("unroll") for (int i = 0; i < FM; ++i)                                                   \
    _Pragma("unroll") for (int j = 0; j < FN; ++j)                                                   \
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[j], acc[i][j], 0, 0, 0);          \
  }

  floatx16h acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  __syncthreads();  // sbias
  const int ntk = Kp / BK;
  if constexpr (VEC) {
    {
      half8 ra[AV], rb[BV];
      bool rok[BV];
      ORE_H_LOADA(ra, 0);
      ORE_H_LOADB_VEC(rb, rok, 0);
      ORE_H_STOREA(ra, 0);
      ORE_H_STOREB_VEC(rb, rok, 0);
    }
    __syncthreads();
    for (int t = 0; t < ntk - 1; ++t) {
      const int buf = t & 1;
      half8 ra[AV], rb[BV];
      bool rok[BV];
      ORE_H_LOADA(ra, (t + 1) * BK);
      ORE_H_LOADB_VEC(rb, rok, (t + 1) * BK);
      __builtin_amdgcn_sched_barrier(0);  // the next stage's loads issue ahead of this stage's MFMAs
      ORE_H_COMPUTE(buf);
      ORE_H_STOREA(ra, buf ^ 1);
      ORE_H_STOREB_VEC(rb, rok, buf ^ 1);
      __syncthreads();
    }
  } else {
    {
      half8 ra[AV];
      XT rb[8 * BV];
      bool rok[8 * BV];
      ORE_H_LOADA(ra, 0);
      ORE_H_LOADB_ELEM(rb, rok, 0);
      ORE_H_STOREA(ra, 0);
      ORE_H_STOREB_ELEM(rb, rok, 0);
    }
    __syncthreads();
    for (int t = 0; t < ntk - 1; ++t) {
      const int buf = t & 1;
      half8 ra[AV];
      XT rb[8 * BV];
      bool rok[8 * BV];
      ORE_H_LOADA(ra, (t + 1) * BK);
      ORE_H_LOADB_ELEM(rb, rok, (t + 1) * BK);
      __builtin_amdgcn_sched_barrier(0);
      ORE_H_COMPUTE(buf);
      ORE_H_STOREA(ra, buf ^ 1);
      ORE_H_STOREB_ELEM(rb, rok, buf ^ 1);
      __syncthreads();
    }
  }
  ORE_H_COMPUTE((ntk - 1) & 1);
#undef ORE_H_LOADA
#undef ORE_H_STOREA
#undef ORE_H_LOADB_VEC
#undef ORE_H_STOREB_VEC
#undef ORE_H_LOADB_ELEM
#undef ORE_H_STOREB_ELEM
#undef ORE_H_COMPUTE

  // epilogue: + bias (f32), optional Relu, one rounding to f16, NHWC store.  Each wave stages its
  // TM channels x TN pixels in its own LDS slice as [pixel][channel] (accumulator rows 8q + 4 lrow
  // + 0..3 are four consecutive channels: one 8-B write), then stores every pixel's channel run
  // with 16-B stores (host: y_ps % 8 == 0, M % 8 == 0, 16-B aligned y) or 2-byte stores.
  __syncthreads();  // every wave is done with the operand tiles
  _Float16* stg = smem + wave * (TN * SR);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ch = i * 32 + 8 * q + 4 * lrow;
        half4 h;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = acc[i][j][4 * q + e] + sbias[wm0 + ch + e];
          if (p.relu) v = fmaxf(v, 0.0f);
          h[e] = (_Float16)v;
        }
        *reinterpret_cast<half4*>(stg + (j * 32 + lcol) * SR + ch) = h;
      }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  _Float16* __restrict__ y = reinterpret_cast<_Float16*>(p.y);
  const int yps = p.y_ps;
  if (p.vec_out) {
    constexpr int CG = TM / 8;  // 16-B channel groups per staged pixel
#pragma unroll
    for (int idx = lane; idx < TN * CG; idx += 64) {
      const int px = idx / CG, cg = idx - px * CG;
      const int n = n0 + wn0 + px;
      const int m = m0 + wm0 + cg * 8;
      if (n < p.Ntot && m < p.M) {
        const int img = n / P, pix = n - img * P;
        *reinterpret_cast<half8*>(y + (unsigned)(img * (int)p.y_nstride + pix * yps + m)) =
            *reinterpret_cast<const half8*>(stg + px * SR + cg * 8);
      }
    }
  } else {
    for (int idx = lane; idx < TN * TM; idx += 64) {
      const int px = idx / TM, ch = idx - px * TM;
      const int n = n0 + wn0 + px, m = m0 + wm0 + ch;
      if (n < p.Ntot && m < p.M) {
        const int img = n / P, pix = n - img * P;
        y[(unsigned)(img * (int)p.y_nstride + pix * yps + m)] = stg[px * SR + ch];
      }
    }
  }
}

// Wh[m][k] = f16(W[m][c][r][s]) zero padded to Mp x Kp; k = (c, r, s) (the reference's order, the
// f32 NCHW input) or k = (r, s, c) (NHWC inputs: c fastest).
__global__ __launch_bounds__(256) void pack_weights_f16_kernel(const float* __restrict__ w, int rsc, int M, int C,
                                                               int KK, int Mp, int Kp, _Float16* __restrict__ wh) {
  const int K = C * KK;
  const long long total = (long long)Mp * Kp;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int m = (int)(i / Kp), k = (int)(i - (long long)m * Kp);
    float v = 0.0f;
    if (m < M && k < K) v = rsc ? w[((long long)m * C + (k % C)) * KK + k / C] : w[(long long)m * K + k];
    wh[i] = (_Float16)v;
  }
}

void launch_pack_weights_f16(const float* w, int xmode, int M, int C, int kh, int kw, int Mp, void* wh,
                             hipStream_t s) {
  const int Kp = conv_packed_kp(C * kh * kw);
  long long blocks = ((long long)Mp * Kp + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pack_weights_f16_kernel, dim3((unsigned)blocks), dim3(256), 0, s, w,
                     xmode == F16_X_NCHW32 ? 0 : 1, M, C, kh * kw, Mp, Kp, static_cast<_Float16*>(wh));
}

// Gather table over an NHWC input, k = (r, s, c): entry {(r * W + s) * cs + c, (r << 16) | s} per k
// (vec = false) or per group of 8 k (vec: c = the group's first channel); entries past K carry
// r = 1 << 14, which no bounds check passes (read as zeros).
__global__ __launch_bounds__(256) void ktab_nhwc_kernel(int2* __restrict__ ktab, int C, int K, int n, int step, int kw,
                                                        int cs, int W) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    int2 e = make_int2(0, (1 << 14) << 16);
    const int k = i * step;
    if (k < K) {
      const int rs = k / C, c = k - rs * C, r = rs / kw, s = rs - r * kw;
      e = make_int2((r * W + s) * cs + c, (r << 16) | s);
    }
    ktab[i] = e;
  }
}

void launch_ktab_nhwc(int2* ktab, int C, int kh, int kw, int cs, int W, bool vec, hipStream_t s) {
  const int K = C * kh * kw, step = vec ? 8 : 1;
  const int n = conv_packed_kp(K) / step;
  hipLaunchKernelGGL(ktab_nhwc_kernel, dim3((n + 255) / 256), dim3(256), 0, s, ktab, C, K, n, step, kw, cs, W);
}

template <int BM, int BN, int WM, int WN>
static void launch_f16_cfg(const ConvParams& p0, int xmode, hipStream_t s) {
  ConvParams p = p0;
  p.mtiles = (p.M + BM - 1) / BM;
  p.ntiles = (int)((p.Ntot + BN - 1) / BN);
  dim3 grid((unsigned)(p.mtiles * p.ntiles)), block(256);
  switch (xmode) {
    case F16_X_NCHW32: hipLaunchKernelGGL((conv_f16_kernel<BM, BN, WM, WN, F16_X_NCHW32>), grid, block, 0, s, p); break;
    case F16_X_NHWC_ELEM: hipLaunchKernelGGL((conv_f16_kernel<BM, BN, WM, WN, F16_X_NHWC_ELEM>), grid, block, 0, s, p); break;
    default: hipLaunchKernelGGL((conv_f16_kernel<BM, BN, WM, WN, F16_X_NHWC_VEC>), grid, block, 0, s, p); break;
  }
}

void launch_conv_f16(const ConvParams& p, int cfg, int xmode, hipStream_t s) {
  switch (cfg) {
    case 0: launch_f16_cfg<128, 128, 2, 2>(p, xmode, s); break;
    case 1: launch_f16_cfg<96, 128, 1, 4>(p, xmode, s); break;
    case 2: launch_f16_cfg<64, 128, 2, 2>(p, xmode, s); break;
    default: launch_f16_cfg<32, 256, 1, 4>(p, xmode, s); break;
  }
}

// ------------------------------------------------------------------ NHWC MaxPool / GAP / Concat
// MaxPool over NHWC f16: one thread per (output pixel, 8-channel group), 16-B loads when channel
// counts, pixel strides and pointers allow, else one thread per (pixel, channel).  Taps outside the
// image read 0 (max_pool_op.rs:265-276) and the running max starts at -FLT_MAX (:337).  Exact.
template <int VEC>
__global__ __launch_bounds__(256) void maxpool_nhwc_kernel(NhwcPoolParams p) {
  const int CG = VEC ? p.C / 8 : p.C;
  const long long total = (long long)p.N * p.Ho * p.Wo * CG;
  for (long long idx = (long long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    const int cg = (int)(idx % CG);
    long long t = idx / CG;
    const int ow = (int)(t % p.Wo);
    t /= p.Wo;
    const int oh = (int)(t % p.Ho);
    const int n = (int)(t / p.Ho);
    const int ih0 = oh * p.sh - p.pt, iw0 = ow * p.sw - p.pl;
    const _Float16* xn = p.x + (long long)n * p.x_nstride;
    _Float16* yp = p.y + (long long)n * p.y_nstride + (long long)(oh * p.Wo + ow) * p.y_cs;
    if (VEC) {
      float m[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) m[e] = -FLT_MAX;
      for (int r = 0; r < p.kh; ++r) {
        const int ih = ih0 + r;
        for (int s = 0; s < p.kw; ++s) {
          const int iw = iw0 + s;
          half8 v = {};
          if ((unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W)
            v = *reinterpret_cast<const half8*>(xn + (long long)(ih * p.W + iw) * p.x_cs + cg * 8);
#pragma unroll
          for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], (float)v[e]);
        }
      }
      half8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (_Float16)m[e];
      *reinterpret_cast<half8*>(yp + cg * 8) = o;
    } else {
      float m = -FLT_MAX;
      for (int r = 0; r < p.kh; ++r) {
        const int ih = ih0 + r;
        for (int s = 0; s < p.kw; ++s) {
          const int iw = iw0 + s;
          const bool in = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
          m = fmaxf(m, in ? (float)xn[(long long)(ih * p.W + iw) * p.x_cs + cg] : 0.0f);
        }
      }
      yp[cg] = (_Float16)m;
    }
  }
}

static unsigned grid_for(long long work) {
  long long b = (work + 255) / 256;
  if (b > 256 * 32) b = 256 * 32;
  return (unsigned)(b < 1 ? 1 : b);
}

void launch_maxpool_nhwc(const NhwcPoolParams& p, hipStream_t s) {
  const bool vec = p.C % 8 == 0 && p.x_cs % 8 == 0 && p.y_cs % 8 == 0 && p.x_nstride % 8 == 0 &&
                   p.y_nstride % 8 == 0 &&
                   ((reinterpret_cast<uintptr_t>(p.x) | reinterpret_cast<uintptr_t>(p.y)) & 15) == 0;
  const long long total = (long long)p.N * p.Ho * p.Wo * (vec ? p.C / 8 : p.C);
  if (total <= 0) return;
  if (vec)
    hipLaunchKernelGGL(maxpool_nhwc_kernel<1>, dim3(grid_for(total)), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(maxpool_nhwc_kernel<0>, dim3(grid_for(total)), dim3(256), 0, s, p);
}

// GlobalAveragePool of NHWC f16 -> f32 y[n][c]: one lane per (n, c) summing the pixels in row-major
// order in f32, then / (H*W) -- the reference's sequential Iterator::sum
// (global_average_pool_op.rs:44-48) over the f16 values.  Lanes are consecutive channels, so each
// pixel step is one coalesced run of the image.
__global__ __launch_bounds__(256) void gap_nhwc_kernel(const _Float16* __restrict__ x, float* __restrict__ y, int N,
                                                       int C, int HW, int cs, long long nstride) {
  const long long total = (long long)N * C;
  for (long long idx = (long long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    const int n = (int)(idx / C), c = (int)(idx - (long long)n * C);
    const _Float16* xp = x + (long long)n * nstride + c;
    float s = 0.0f;
    for (int i = 0; i < HW; ++i) s = s + (float)xp[(long long)i * cs];
    y[idx] = s / (float)HW;
  }
}

void launch_gap_nhwc(const void* x, float* y, int N, int C, int HW, int cs, long long nstride, hipStream_t s) {
  const long long total = (long long)N * C;
  if (total <= 0) return;
  hipLaunchKernelGGL(gap_nhwc_kernel, dim3(grid_for(total)), dim3(256), 0, s, static_cast<const _Float16*>(x), y, N, C,
                     HW, cs, nstride);
}

// Concat along channels of two dense NHWC values into a dense y (Ca + Cb channels per pixel).
__global__ __launch_bounds__(256) void concat_nhwc_kernel(const _Float16* __restrict__ a, const _Float16* __restrict__ b,
                                                          _Float16* __restrict__ y, long long pixels, int Ca, int Cb) {
  const int Cy = Ca + Cb;
  const long long total = pixels * Cy;
  for (long long idx = (long long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    const long long px = idx / Cy;
    const int c = (int)(idx - px * Cy);
    y[idx] = c < Ca ? a[px * Ca + c] : b[px * Cb + (c - Ca)];
  }
}

void launch_concat_nhwc(const void* a, const void* b, void* y, long long pixels, int Ca, int Cb, hipStream_t s) {
  if (pixels * (Ca + Cb) <= 0) return;
  hipLaunchKernelGGL(concat_nhwc_kernel, dim3(grid_for(pixels * (Ca + Cb))), dim3(256), 0, s,
                     static_cast<const _Float16*>(a), static_cast<const _Float16*>(b), static_cast<_Float16*>(y), pixels,
                     Ca, Cb);
}

}  // namespace ore
