// LDS-free, barrier-free implicit-GEMM Conv (f32): every wave loads its own MFMA fragments
// straight from global memory (L1/L2) and runs independently of the other waves of its block.
//
// The same GEMM as conv_gemm_kernel (ore_conv.hip; M = Cout, N = images x plane, K = Cin*kh*kw
// in the reference's (cin, r, s) order, convolution_op.rs:422-480): the k-ordered MFMA chain per
// output is identical, so results are bit-identical to it.  What changes is the staging:
//   * A fragment (lane l: A[m = l&31][k = l>>5]) = one dword of the K-major packed weights per
//     lane -- two 128-B rows per wave-instruction.
//   * B fragment (lane l: B[k = l>>5][n = l&31]) = one gathered activation per lane through a
//     buffer resource: a tap outside the image gets an out-of-range offset and reads 0 (the
//     reference's zero padding) with no select.
//   * P k-steps of fragments are in flight (a register ring), so global latency is covered by the
//     wave's own MFMAs; no __syncthreads anywhere in the K loop.
// Tiles 4-7, selectable with ORE_CONV_CFG; not autotune candidates: on every SqueezeNet layer
// they measured 15-80 % slower than the LDS-staged kernel (profiles/r01l_direct_vs_lds.txt) --
// one VMEM instruction per MFMA operand costs more than the LDS round trip and barriers save.
#include <hip/hip_runtime.h>
#include <float.h>

#include "ore_kernels.h"

namespace ore {

typedef float floatx16d __attribute__((ext_vector_type(16)));

enum { D1X1 = 0, DGATHER = 1 };

template <int BM, int BN, int WM, int WN, int BMODE, int P>
__global__ __launch_bounds__(256, 2) void conv_direct_kernel(ConvParams p) {
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 32, FN = TN / 32;
  static_assert(WM * WN == 4 && FM >= 1 && FN >= 1 && 16 % P == 0, "tile");
  __shared__ float sbias[BM];

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

  // this lane's B columns (one per fragment j)
  int xoff[FN], ih0[FN], iw0[FN];
  bool nok[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int bn = n0 + wn0 + j * 32 + lcol;
    nok[j] = bn < p.Ntot;
    const int nn = nok[j] ? bn : 0;
    const int img = nn / YPS;
    const int pix = nn - img * YPS;
    xoff[j] = img * (int)p.x_nstride;
    ih0[j] = 0;
    iw0[j] = 0;
    if (BMODE == D1X1) {
      xoff[j] += pix;
    } else {
      const int oh = pix / p.Wo, ow = pix - oh * p.Wo;
      ih0[j] = oh * p.sh - p.pt;
      iw0[j] = ow * p.sw - p.pl;
      xoff[j] += ih0[j] * p.W + iw0[j];
    }
  }
  const __amdgpu_buffer_rsrc_t xrsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.x), (short)0, (int)p.x_bytes, 0x00020000);
  const float* __restrict__ wp = p.wp;
  typedef const __attribute__((address_space(4))) long long* ktab_cptr;
  const ktab_cptr ktab = (ktab_cptr)p.ktab;
  const int mA = m0 + wm0 + lcol;  // A fragment row of fragment i: mA + 32 i

  // one k-step (2 k values) of fragments: lane reads k = KK + lrow
#define ORE_D_LOAD(AF, BF, KK)                                                                       \
  {                                                                                                  \
    const int kk_ = (KK);                                                                            \
    const int k_ = kk_ + lrow;                                                                       \
    _Pragma("unroll") for (int i = 0; i < FM; ++i)                                                   \
      AF[i] = wp[(unsigned)(k_ * p.Mp + mA + i * 32)];                                               \
    int ex_, r_ = 0, s_ = 0;                                                                         \
    if (BMODE == D1X1) {                                                                             \
      ex_ = k_ * XPS;                                                                                \
    } else {                                                                                         \
      const long long w0_ = ktab[kk_], w1_ = ktab[kk_ + 1];                                          \
      const long long w_ = lrow ? w1_ : w0_;                                                         \
      ex_ = (int)w_;                                                                                 \
      const int ey_ = (int)(w_ >> 32);                                                               \
      r_ = ey_ >> 16;                                                                                \
      s_ = ey_ & 0xffff;                                                                             \
    }                                                                                                \
    _Pragma("unroll") for (int j = 0; j < FN; ++j) {                                                 \
      bool ok_ = nok[j] & (k_ < K);                                                                  \
      if (BMODE != D1X1)                                                                             \
        ok_ = ok_ & ((unsigned)(ih0[j] + r_) < (unsigned)p.H) & ((unsigned)(iw0[j] + s_) < (unsigned)p.W); \
      BF[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(                        \
          xrsrc, ok_ ? (xoff[j] + ex_) * 4 : (int)0x80000000, 0, 0));                                 \
    }                                                                                                \
  }

  floatx16d acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  // register ring of P k-steps in flight
  float ra[P][FM], rb[P][FN];
#pragma unroll
  for (int q = 0; q < P; ++q) ORE_D_LOAD(ra[q], rb[q], 2 * q);
  const int nsteps = Kp / 2;  // Kp % 32 == 0, P divides 16: whole rounds of P
  for (int base = 0; base < nsteps; base += P) {
#pragma unroll
    for (int q = 0; q < P; ++q) {
      float ca[FM], cb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) ca[i] = ra[q][i];
#pragma unroll
      for (int j = 0; j < FN; ++j) cb[j] = rb[q][j];
      const int nx = base + q + P;  // refill this ring slot with k-step nx (clamped past the end)
      ORE_D_LOAD(ra[q], rb[q], 2 * (nx < nsteps ? nx : nsteps - 1));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ca[i], cb[j], acc[i][j], 0, 0, 0);
    }
  }
#undef ORE_D_LOAD

  __syncthreads();  // sbias
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

template <int BM, int BN, int WM, int WN>
static void launch_direct_cfg(const ConvParams& p0, hipStream_t s) {
  constexpr int P = 4;
  ConvParams p = p0;
  p.mtiles = (p.M + BM - 1) / BM;
  p.ntiles = (int)((p.Ntot + BN - 1) / BN);
  dim3 grid(p.mtiles * p.ntiles), block(256);
  if (p.is1x1)
    hipLaunchKernelGGL((conv_direct_kernel<BM, BN, WM, WN, D1X1, P>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((conv_direct_kernel<BM, BN, WM, WN, DGATHER, P>), grid, block, 0, s, p);
}

// tile 4: 128x128 (2x2 waves of 64x64), 5: 96x128 (1x4 of 96x32), 6: 64x128 (2x2 of 32x64),
// 7: 128x64 (4x1 of 32x64)
void launch_conv_direct(const ConvParams& p, int tile, hipStream_t s) {
  switch (tile) {
    case 4: launch_direct_cfg<128, 128, 2, 2>(p, s); break;
    case 5: launch_direct_cfg<96, 128, 1, 4>(p, s); break;
    case 6: launch_direct_cfg<64, 128, 2, 2>(p, s); break;
    default: launch_direct_cfg<128, 64, 4, 1>(p, s); break;
  }
}

}  // namespace ore
