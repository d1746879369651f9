// fp16 variant of the Conv op: f16 activations and weights, f32
// accumulation on the CDNA4 f16 matrix cores (v_mfma_f32_32x32x16_f16, 16x the f32 MFMA
// rate).  Same implicit GEMM as conv_gemm_kernel (ore_conv.hip) -- M = Cout, N = images x
// plane, K = Cin*kh*kw in the reference's (cin, r, s) order, gather table ktab, XCD remap, bias +
// Relu epilogue into (possibly sliced, padded) NCHW -- with the operand layouts the f16 MFMA
// wants: lane l holds A[row l&31][k = 8(l>>5) .. +7] and B[k = 8(l>>5) .. +7][col l&31], so both
// LDS tiles are stored k-contiguous ([row][k] and [pixel][k]) and every fragment is one 16-B read.
//
// The first conv of a network reads the f32 model input (XF32) and rounds to f16 while staging.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ore_kernels.h"

namespace ore {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16h __attribute__((ext_vector_type(16)));

enum { H1X1 = 0, HGATHER = 1, HPOOL = 2 };  // HPOOL: B = 3x3 window max of the pre-pool tensor

template <int BM, int BN, int WM, int WN, int XF32, int BMODE>
__global__ __launch_bounds__(256, 2) void conv_f16_kernel(ConvParams p) {
  constexpr int BK = 32;                 // k per stage: two 32x32x16 k-steps
  constexpr int LR = 40;                 // LDS row: 32 halves + 8 pad = 80 B (16-B reads conflict-free)
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 32, FN = TN / 32;
  constexpr int ACH = BM * 4;            // 16-B chunks of one A stage (BM rows x 4)
  constexpr int AV = (ACH + 255) / 256;  // A chunks per thread
  constexpr int BV = BN * 4 / 256;       // B tasks (one pixel x 8 consecutive k) per thread
  constexpr int QS = 256 / BN;           // k-group stride between a thread's tasks
  static_assert(WM * WN == 4 && FM >= 1 && FN >= 1 && (BN * 4) % 256 == 0 && 256 % BN == 0, "tile");
  typedef typename std::conditional<XF32, float, _Float16>::type XT;

  // operand tiles; the epilogue reuses the array for a per-wave [32][TN] f32 staging tile
  constexpr int MAIN_HALVES = 2 * (BM + BN) * LR, EPI_HALVES = 4 * 32 * TN * 2;
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
  const int K = p.K, Kp = (K + 31) & ~31;
  const int XPS = p.x_ps, YPS = p.y_ps;

  for (int i = tid; i < BM; i += 256) sbias[i] = (p.bias && m0 + i < p.M) ? p.bias[m0 + i] : 0.0f;

  // this thread's B column and k groups (wave-uniform)
  const int bcol = tid % BN;
  const int qbase = __builtin_amdgcn_readfirstlane(tid / BN);
  const int bn = n0 + bcol;
  const bool bn_ok = bn < p.Ntot;
  int xoff, ih0 = 0, iw0 = 0;
  int pmask = 0;
  {
    const int nn = bn_ok ? bn : 0;
    const int img = nn / YPS;
    const int pix = nn - img * YPS;
    xoff = img * (int)p.x_nstride;
    if (BMODE == H1X1) {
      xoff += pix;
    } else if (BMODE == HPOOL) {
      const int oh = pix / p.Wo, ow = pix - oh * p.Wo;
      ih0 = oh * p.pool_sh - p.pool_pt;
      iw0 = ow * p.pool_sw - p.pool_pl;
      xoff += ih0 * p.pool_W + iw0;
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s)
          if ((unsigned)(ih0 + r) < (unsigned)p.pool_H && (unsigned)(iw0 + s) < (unsigned)p.pool_W) pmask |= 1 << (r * 3 + s);
    } else {
      const int oh = pix / p.Wo, ow = pix - oh * p.Wo;
      ih0 = oh * p.sh - p.pt;
      iw0 = ow * p.sw - p.pl;
      xoff += ih0 * p.W + iw0;
    }
  }
  const XT* __restrict__ x = reinterpret_cast<const XT*>(p.x);
  const _Float16* __restrict__ wh = reinterpret_cast<const _Float16*>(p.wp);  // [Mp][Kp]
  typedef const __attribute__((address_space(4))) long long* ktab_cptr;
  const ktab_cptr ktab = (ktab_cptr)p.ktab;

#define ORE_H_LOAD(RA, RB, ROK, K0)                                                                  \
  {                                                                                                  \
    const int k0_ = (K0);                                                                            \
    _Pragma("unroll") for (int v_ = 0; v_ < AV; ++v_) {                                              \
      const int c_ = (ACH % 256 == 0 || tid + v_ * 256 < ACH) ? tid + v_ * 256 : 0;                  \
      const int row_ = c_ >> 2, q_ = c_ & 3;                                                         \
      RA[v_] = *reinterpret_cast<const half8*>(wh + (unsigned)((m0 + row_) * Kp + k0_ + q_ * 8));    \
    }                                                                                                \
    _Pragma("unroll") for (int u_ = 0; u_ < BV; ++u_) {                                              \
      const int kg_ = k0_ + (qbase + u_ * QS) * 8;                                                   \
      _Pragma("unroll") for (int e_ = 0; e_ < 8; ++e_) {                                             \
        const int k = kg_ + e_;                                                                      \
        bool ok;                                                                                     \
        int off;                                                                                     \
        if (BMODE == H1X1 || BMODE == HPOOL) {                                                       \
          ok = bn_ok & (k < K);                                                                      \
          off = xoff + k * XPS;                                                                      \
        } else {                                                                                     \
          const long long w_ = ktab[k];                                                              \
          const int ex_ = (int)w_, ey_ = (int)(w_ >> 32);                                            \
          const int r = ey_ >> 16, s = ey_ & 0xffff;                                                 \
          ok = bn_ok & ((unsigned)(ih0 + r) < (unsigned)p.H) & ((unsigned)(iw0 + s) < (unsigned)p.W); \
          off = xoff + ex_;                                                                          \
        }                                                                                            \
        if (BMODE == HPOOL) {                                                                        \
          float m_ = -3.402823466e38f;                                                               \
          _Pragma("unroll") for (int t_ = 0; t_ < 9; ++t_) {                                         \
            const bool in_ = ok & (((pmask >> t_) & 1) != 0);                                        \
            const float v_ = (float)x[(unsigned)(in_ ? off + (t_ / 3) * p.pool_W + (t_ % 3) : 0)];    \
            m_ = fmaxf(m_, in_ ? v_ : 0.0f);                                                         \
          }                                                                                          \
          RB[u_ * 8 + e_] = (XT)m_;                                                                  \
        } else {                                                                                     \
          RB[u_ * 8 + e_] = x[(unsigned)(ok ? off : 0)];                                             \
        }                                                                                            \
        ROK[u_ * 8 + e_] = ok;                                                                       \
      }                                                                                              \
    }                                                                                                \
  }
#define ORE_H_STORE(RA, RB, ROK, BUF)                                                                \
  {                                                                                                  \
    _Pragma("unroll") for (int v_ = 0; v_ < AV; ++v_) {                                              \
      const int c_ = tid + v_ * 256;                                                                 \
      if (ACH % 256 == 0 || c_ < ACH)                                                                \
        *reinterpret_cast<half8*>(&As[BUF][c_ >> 2][(c_ & 3) * 8]) = RA[v_];                         \
    }                                                                                                \
    _Pragma("unroll") for (int u_ = 0; u_ < BV; ++u_) {                                              \
      half8 h_;                                                                                      \
      _Pragma("unroll") for (int e_ = 0; e_ < 8; ++e_)                                               \
        h_[e_] = ROK[u_ * 8 + e_] ? (_Float16)RB[u_ * 8 + e_] : (_Float16)0.0f;                      \
      *reinterpret_cast<half8*>(&Bs[BUF][bcol][(qbase + u_ * QS) * 8]) = h_;                         \
    }                                                                                                \
  }
#define ORE_H_COMPUTE(BUF)                                                                           \
  {                                                                                                  \
    _Pragma("unroll") for (int ks = 0; ks < BK; ks += 16) {                                          \
      half8 af[FM], bf[FN];                                                                          \
      _Pragma("unroll") for (int i = 0; i < FM; ++i)                                                 \
        af[i] = *reinterpret_cast<const half8*>(&As[BUF][wm0 + i * 32 + lcol][ks + 8 * lrow]);       \
      _Pragma("unroll") for (int j = 0; j < FN; ++j)                                                 \
        bf[j] = *reinterpret_cast<const half8*>(&Bs[BUF][wn0 + j * 32 + lcol][ks + 8 * lrow]);       \
      _Pragma("unroll") for (int i = 0; i < FM; ++i)                                                 \
      _Pragma("unroll") for (int j = 0; j < FN; ++j)                                                 \
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[j], acc[i][j], 0, 0, 0);        \
    }                                                                                                \
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
  {
    half8 ra[AV];
    XT rb[8 * BV];
    bool rok[8 * BV];
    ORE_H_LOAD(ra, rb, rok, 0);
    ORE_H_STORE(ra, rb, rok, 0);
  }
  __syncthreads();
  for (int t = 0; t < ntk - 1; ++t) {
    const int buf = t & 1;
    half8 ra[AV];
    XT rb[8 * BV];
    bool rok[8 * BV];
    ORE_H_LOAD(ra, rb, rok, (t + 1) * BK);
    __builtin_amdgcn_sched_barrier(0);  // the next stage's loads issue ahead of this stage's MFMAs
    ORE_H_COMPUTE(buf);
    ORE_H_STORE(ra, rb, rok, buf ^ 1);
    __syncthreads();
  }
  ORE_H_COMPUTE((ntk - 1) & 1);
#undef ORE_H_LOAD
#undef ORE_H_STORE
#undef ORE_H_COMPUTE

  // epilogue: + bias (f32), optional Relu, round to f16, store NCHW (possibly a channel slice)
  _Float16* __restrict__ y = reinterpret_cast<_Float16*>(p.y);
  if (p.vec_out) {
    // 16-B stores of 8 pixels: each wave stages 32 rows x TN pixels (f32) in its own LDS slice
    // (rows r and r + 4 in opposite bank halves), then converts and writes whole pixel runs.
    // Host guarantees y_ps % 8 == 0, y_nstride % 8 == 0 and a 16-B aligned y.
    __syncthreads();  // every wave is done with the A/B tiles
    float* stg = reinterpret_cast<float*>(smem) + wave * (32 * TN);
    constexpr int V8 = TN / 8;   // 8-pixel groups per staged row
    constexpr int RPI = 64 / V8; // rows per wave-instruction
#define ORE_HSTG(R, C) (TN >= 64 ? (R) * TN + ((C) ^ ((((R) >> 2) & 1) * 32)) : ((R) ^ (((R) >> 2) & 1)) * TN + (C))
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int r = (e & 3) + 8 * (e >> 2) + 4 * lrow;
          float v = acc[i][j][e] + sbias[wm0 + i * 32 + r];
          if (p.relu) v = fmaxf(v, 0.0f);
          stg[ORE_HSTG(r, j * 32 + lcol)] = v;
        }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int c8 = (lane % V8) * 8;
      const int n = n0 + wn0 + c8;
      const int img = n / YPS;
      const int pix = n - img * YPS;
      const bool nok = n < p.Ntot;
#pragma unroll
      for (int rr = 0; rr < 32; rr += RPI) {
        const int r = rr + lane / V8;
        const int m = m0 + wm0 + i * 32 + r;
        half8 h;
#pragma unroll
        for (int u = 0; u < 8; ++u) h[u] = (_Float16)stg[ORE_HSTG(r, c8 + u)];
        if (nok && m < p.M) *reinterpret_cast<half8*>(y + (unsigned)(img * (int)p.y_nstride + m * YPS + pix)) = h;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#undef ORE_HSTG
    return;
  }
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
          y[yb + (unsigned)((m0 + ml) * YPS)] = (_Float16)v;
        }
      }
    }
  }
}

// Wh[m][k] = f16(W[m][k]) for m < M, k < K (zero padding to Mp x Kp); kmajor_src: W is [K][M].
__global__ __launch_bounds__(256) void pack_weights_f16_kernel(const float* __restrict__ w, int kmajor_src, int M,
                                                               int K, int Mp, int Kp, _Float16* __restrict__ wh) {
  const long long total = (long long)Mp * Kp;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int m = (int)(i / Kp), k = (int)(i - (long long)m * Kp);
    float v = 0.0f;
    if (m < M && k < K) v = kmajor_src ? w[(long long)k * M + m] : w[(long long)m * K + k];
    wh[i] = (_Float16)v;
  }
}

void launch_pack_weights_f16(const float* w, bool kmajor_src, int M, int K, int Mp, void* wh, hipStream_t s) {
  const int Kp = conv_packed_kp(K);
  long long blocks = ((long long)Mp * Kp + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pack_weights_f16_kernel, dim3((unsigned)blocks), dim3(256), 0, s, w, kmajor_src ? 1 : 0, M, K,
                     Mp, Kp, static_cast<_Float16*>(wh));
}

template <int BM, int BN, int WM, int WN>
static void launch_f16_cfg(const ConvParams& p0, hipStream_t s) {
  ConvParams p = p0;
  p.mtiles = (p.M + BM - 1) / BM;
  p.ntiles = (int)((p.Ntot + BN - 1) / BN);
  dim3 grid((unsigned)(p.mtiles * p.ntiles)), block(256);
  const bool xf32 = p.x_f32 != 0;
  if (p.pool) {
    if (xf32)
      hipLaunchKernelGGL((conv_f16_kernel<BM, BN, WM, WN, 1, HPOOL>), grid, block, 0, s, p);
    else
      hipLaunchKernelGGL((conv_f16_kernel<BM, BN, WM, WN, 0, HPOOL>), grid, block, 0, s, p);
  } else if (p.is1x1) {
    if (xf32)
      hipLaunchKernelGGL((conv_f16_kernel<BM, BN, WM, WN, 1, H1X1>), grid, block, 0, s, p);
    else
      hipLaunchKernelGGL((conv_f16_kernel<BM, BN, WM, WN, 0, H1X1>), grid, block, 0, s, p);
  } else {
    if (xf32)
      hipLaunchKernelGGL((conv_f16_kernel<BM, BN, WM, WN, 1, HGATHER>), grid, block, 0, s, p);
    else
      hipLaunchKernelGGL((conv_f16_kernel<BM, BN, WM, WN, 0, HGATHER>), grid, block, 0, s, p);
  }
}

void launch_conv_f16(const ConvParams& p, int cfg, hipStream_t s) {
  switch (cfg) {
    case 0: launch_f16_cfg<128, 128, 2, 2>(p, s); break;
    case 1: launch_f16_cfg<96, 128, 1, 4>(p, s); break;
    case 2: launch_f16_cfg<64, 128, 2, 2>(p, s); break;
    default: launch_f16_cfg<32, 256, 1, 4>(p, s); break;
  }
}

}  // namespace ore
