// fp16 variant: f16 activations stored channels-last (NHWC), f16
// weights, f32 accumulation on the CDNA4 f16 matrix cores (v_mfma_f32_32x32x16_f16, 16x the f32
// MFMA rate).  The reference is f32 NCHW only (convolution_op.rs:422-480); the f16 path is ours to
// lay out, and NHWC is what makes its operand gather cheap: with k ordered (r, s, c) -- c fastest --
// the 8 consecutive k of one MFMA fragment lane are 8 consecutive channels of one input pixel,
// i.e. ONE 16-B load, where an NCHW gather needs 8 scattered 2-byte loads with 8 bounds checks.
//
//   conv_f16_kernel<..., F16_X_NHWC_VEC>   every conv on an f16 activation with C % 8 == 0
//   conv_f16_kernel<..., F16_X_NHWC_PAIR>  the first conv (<= 4 input channels): the f32 NCHW model
//                                          input converted to NHWC with 4 channels per pixel
//                                          (nchw_to_nhwc4_kernel); one 8-B load per (tap, 4 channels),
//                                          the 16-B fragment group = two horizontally adjacent taps
//   conv_f16_kernel<..., F16_X_NCHW32>     a conv on an f32 NCHW value with > 4 channels: per-element
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
#include <stdlib.h>

#include <type_traits>

#include "ore_kernels.h"


namespace ore {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float floatx16h __attribute__((ext_vector_type(16)));

// B-operand registers of one K stage per thread, by operand mode
template <int XMODE, int BV>
struct BStage;
template <int BV>
struct BStage<F16_X_NHWC_VEC, BV> {  // one 16-B (pixel, 8-channel) load per task
  half8 v[BV];
  bool ok[BV];
};
template <int BV>
struct BStage<F16_X_NHWC_PAIR, BV> {  // two 8-B (pixel, 4-channel) taps per task
  half4 v[2 * BV];
  bool ok[2 * BV];
};
template <int BV>
struct BStage<F16_X_NCHW32, BV> {  // 8 scattered f32 elements per task
  float v[8 * BV];
  bool ok[8 * BV];
};
template <int BV>
struct BStage<F16_X_NHWC_ELEM, BV> {  // 8 scattered f16 elements per task
  _Float16 v[8 * BV];
  bool ok[8 * BV];
};

// EP (ORE_FUSE_CONV_POOL on an f16 model): the block's BN = 256 columns are a 13 x 19 patch of conv
// outputs (ConvParams ep_*; as conv_gemm_kernel's pooled epilogue) and only the 6 x 9 tile of
// 3x3 / stride-2 pooled outputs is stored (NHWC f16).  The conv values are rounded to f16 first, as
// the separate conv stores them, so the pooled result is the separate pool's bit for bit.
constexpr int H_EP_PR = EPOOL_TILE_PR, H_EP_PC = EPOOL_TILE_PC, H_EP_RC = 2 * H_EP_PR + 1, H_EP_CC = 2 * H_EP_PC + 1;

template <int BM, int BN, int WM, int WN, int XMODE, int EP = 0>
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
  constexpr bool LANEG = XMODE == F16_X_NHWC_VEC || XMODE == F16_X_NHWC_PAIR;  // lane-varying k group
  static_assert(WM * WN == 4 && FM >= 1 && FN >= 1 && BN % 64 == 0 && 256 % BN == 0, "tile");
  typedef typename std::conditional<XMODE == F16_X_NCHW32, float, _Float16>::type XT;
  constexpr int SRE = BM + 8;            // EP staging row: one conv position's BM channels + pad (halves)
  constexpr int MAIN_HALVES = 2 * (BM + BN) * LR, EPI_HALVES = EP ? BN * SRE : 4 * TN * SR;
  static_assert(!EP || (WM == 1 && BN == 256 && H_EP_RC * H_EP_CC <= BN), "pooled epilogue tile");
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

  // B tasks.  VEC / PAIR: lane group g = tid & 3 (fixed), pixels (tid >> 2) + 64u: four lanes
  // read 64 contiguous bytes of one pixel.  Per-element: pixel tid % BN, k groups qbase + QS*u
  // (uniform).
  constexpr int NPX = LANEG ? BV : 1;
  const int g = tid & 3;
  const int bcol0 = LANEG ? (tid >> 2) : (tid % BN);
  const int qbase = __builtin_amdgcn_readfirstlane(tid / BN);
  int xoff[NPX], ih0[NPX], iw0[NPX];
  bool nok[NPX];
  // EP: N tile nt = (image, pooled tile row, pooled tile column)
  int ep_img = 0, ep_ph0 = 0, ep_pw0 = 0;
  if constexpr (EP) {
    const int tpi = p.ep_tr * p.ep_tc;
    ep_img = nt / tpi;
    const int t = nt - ep_img * tpi;
    ep_ph0 = (t / p.ep_tc) * H_EP_PR;
    ep_pw0 = (t - (t / p.ep_tc) * p.ep_tc) * H_EP_PC;
  }
#pragma unroll
  for (int u = 0; u < NPX; ++u) {
    int img, oh, ow;
    if constexpr (EP) {
      const int bcol = bcol0 + 64 * u;
      const int prc = bcol / H_EP_CC, pcc = bcol - prc * H_EP_CC;
      img = ep_img;
      oh = ep_ph0 * 2 - p.ep_pt + prc;
      ow = ep_pw0 * 2 - p.ep_pl + pcc;
      nok[u] = img < p.N && bcol < H_EP_RC * H_EP_CC && (unsigned)oh < (unsigned)p.Ho && (unsigned)ow < (unsigned)p.Wo;
      if (!nok[u]) img = oh = ow = 0;
    } else {
      const int bn = n0 + bcol0 + 64 * u;
      nok[u] = bn < p.Ntot;
      const int nn = nok[u] ? bn : 0;
      img = nn / P;
      const int pix = nn - img * P;
      oh = pix / p.Wo;
      ow = pix - oh * p.Wo;
    }
    ih0[u] = oh * p.sh - p.pt;
    iw0[u] = ow * p.sw - p.pl;
    xoff[u] = img * (int)p.x_nstride + (ih0[u] * p.W + iw0[u]) * (XMODE == F16_X_NCHW32 ? 1 : p.x_ps);
  }
  const XT* __restrict__ x = reinterpret_cast<const XT*>(p.x);
  const _Float16* __restrict__ wh = reinterpret_cast<const _Float16*>(p.wp);  // [Mp][Kp]
  typedef const __attribute__((address_space(4))) long long* ktab_cptr;
  const ktab_cptr ktab = (ktab_cptr)p.ktab;  // per k, or per 8-k group (VEC, PAIR)

  // one K stage into registers: A (16-B weight chunks) and B per mode; a tap outside the image
  // (or a group past K: ktab r = 1 << 14) loads from x[0] and is zeroed at the LDS store
  auto load_stage = [&](half8 (&ra)[AV], BStage<XMODE, BV>& rb, int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      const int c = (ACH % 256 == 0 || tid + v * 256 < ACH) ? tid + v * 256 : 0;
      ra[v] = *reinterpret_cast<const half8*>(wh + (unsigned)((m0 + (c >> 2)) * Kp + k0 + (c & 3) * 8));
    }
    if constexpr (LANEG) {
      // the stage's four group entries by scalar loads; this lane's picked by g
      const int kb = k0 >> 3;
      const long long e0 = ktab[kb], e1 = ktab[kb + 1], e2 = ktab[kb + 2], e3 = ktab[kb + 3];
      const long long w = g == 0 ? e0 : g == 1 ? e1 : g == 2 ? e2 : e3;
      const int ex = (int)w, ey = (int)(w >> 32);
      const int r = ey >> 16, s = ey & 0x7fff;
#pragma unroll
      for (int u = 0; u < BV; ++u) {
        const bool rin = nok[u] & ((unsigned)(ih0[u] + r) < (unsigned)p.H);
        const bool ok0 = rin & ((unsigned)(iw0[u] + s) < (unsigned)p.W);
        if constexpr (XMODE == F16_X_NHWC_VEC) {
          rb.v[u] = *reinterpret_cast<const half8*>(x + (unsigned)(ok0 ? xoff[u] + ex : 0));
          rb.ok[u] = ok0;
        } else {  // PAIR: taps s and s + 1 (the latter absent past kw: ey bit 15)
          const bool ok1 = rin & ((ey & 0x8000) == 0) & ((unsigned)(iw0[u] + s + 1) < (unsigned)p.W);
          rb.v[2 * u] = *reinterpret_cast<const half4*>(x + (unsigned)(ok0 ? xoff[u] + ex : 0));
          rb.v[2 * u + 1] = *reinterpret_cast<const half4*>(x + (unsigned)(ok1 ? xoff[u] + ex + p.x_ps : 0));
          rb.ok[2 * u] = ok0;
          rb.ok[2 * u + 1] = ok1;
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < BV; ++u) {
        const int kg = k0 + (qbase + u * QS) * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const long long w = ktab[kg + e];
          const int ex = (int)w, ey = (int)(w >> 32);
          const int r = ey >> 16, s = ey & 0xffff;
          const bool ok = nok[0] & ((unsigned)(ih0[0] + r) < (unsigned)p.H) & ((unsigned)(iw0[0] + s) < (unsigned)p.W);
          rb.v[u * 8 + e] = x[(unsigned)(ok ? xoff[0] + ex : 0)];
          rb.ok[u * 8 + e] = ok;
        }
      }
    }
  };
  auto store_stage = [&](const half8 (&ra)[AV], const BStage<XMODE, BV>& rb, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      const int c = tid + v * 256;
      if (ACH % 256 == 0 || c < ACH) *reinterpret_cast<half8*>(&As[buf][c >> 2][(c & 3) * 8]) = ra[v];
    }
#pragma unroll
    for (int u = 0; u < BV; ++u) {
      if constexpr (XMODE == F16_X_NHWC_VEC) {
        const half8 z = {};
        *reinterpret_cast<half8*>(&Bs[buf][bcol0 + 64 * u][g * 8]) = rb.ok[u] ? rb.v[u] : z;
      } else if constexpr (XMODE == F16_X_NHWC_PAIR) {
        const half4 z = {};
        *reinterpret_cast<half4*>(&Bs[buf][bcol0 + 64 * u][g * 8]) = rb.ok[2 * u] ? rb.v[2 * u] : z;
        *reinterpret_cast<half4*>(&Bs[buf][bcol0 + 64 * u][g * 8 + 4]) = rb.ok[2 * u + 1] ? rb.v[2 * u + 1] : z;
      } else {
        half8 h;
#pragma unroll
        for (int e = 0; e < 8; ++e) h[e] = rb.ok[u * 8 + e] ? (_Float16)rb.v[u * 8 + e] : (_Float16)0.0f;
        *reinterpret_cast<half8*>(&Bs[buf][bcol0][(qbase + u * QS) * 8]) = h;
      }
    }
  };

  floatx16h acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  auto compute = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < BK; ks += 16) {
      half8 af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = *reinterpret_cast<const half8*>(&As[buf][wm0 + i * 32 + lcol][ks + 8 * lrow]);
#pragma unroll
      for (int j = 0; j < FN; ++j) bf[j] = *reinterpret_cast<const half8*>(&Bs[buf][wn0 + j * 32 + lcol][ks + 8 * lrow]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  };

  const int ntk = Kp / BK;
  __syncthreads();  // sbias
  // stage t + 1 is loaded into registers ahead of stage t's MFMAs and published to the other
  // LDS buffer after them
  half8 ra[AV];
  BStage<XMODE, BV> rb;
  load_stage(ra, rb, 0);
  store_stage(ra, rb, 0);
  __syncthreads();
  for (int t = 0; t < ntk; ++t) {
    const bool more = t + 1 < ntk;
    if (more) load_stage(ra, rb, (t + 1) * BK);
    __builtin_amdgcn_sched_barrier(0);  // the next stage's loads issue ahead of this stage's MFMAs
    compute(t & 1);
    if (more) {
      store_stage(ra, rb, (t + 1) & 1);
      __syncthreads();
    }
  }

  if constexpr (EP) {
    // pooled epilogue: every conv position of the patch goes to LDS as [position][channel] f16
    // (bias, Relu, one rounding; 0 outside the conv plane = the pool's zero padding,
    // max_pool_op.rs:265-276), then each (pooled output, 8-channel group) takes the 3x3 max from
    // -FLT_MAX (:337) and leaves by one 16-B NHWC store
    __syncthreads();  // every wave is done with the operand tiles
    const int ohb = ep_ph0 * 2 - p.ep_pt, owb = ep_pw0 * 2 - p.ep_pl;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = wn0 + j * 32 + lcol;
      const int prc = col / H_EP_CC, pcc = col - prc * H_EP_CC;
      const bool cok = col < H_EP_RC * H_EP_CC && (unsigned)(ohb + prc) < (unsigned)p.Ho &&
                       (unsigned)(owb + pcc) < (unsigned)p.Wo;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int ch = i * 32 + 8 * q + 4 * lrow;
          half4 h;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float v = acc[i][j][4 * q + e] + sbias[ch + e];
            if (p.relu) v = fmaxf(v, 0.0f);
            h[e] = cok ? (_Float16)v : (_Float16)0.0f;
          }
          *reinterpret_cast<half4*>(smem + col * SRE + ch) = h;
        }
    }
    __syncthreads();
    _Float16* __restrict__ y = reinterpret_cast<_Float16*>(p.y);
    constexpr int CGN = BM / 8;  // 8-channel groups
    for (int task = tid; task < H_EP_PR * H_EP_PC * CGN; task += 256) {
      const int pp = task / CGN, cg = task - pp * CGN;
      const int a = pp / H_EP_PC, b = pp - a * H_EP_PC;
      float mx[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) mx[e] = -FLT_MAX;
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const half8 v = *reinterpret_cast<const half8*>(smem + ((2 * a + r) * H_EP_CC + 2 * b + s) * SRE + cg * 8);
#pragma unroll
          for (int e = 0; e < 8; ++e) mx[e] = fmaxf(mx[e], (float)v[e]);
        }
      const int ph = ep_ph0 + a, pw = ep_pw0 + b, m = m0 + cg * 8;
      if (ph >= p.ep_Ho || pw >= p.ep_Wo || ep_img >= p.N || m >= p.M) continue;
      _Float16* dst = y + (unsigned)(ep_img * (int)p.y_nstride + (ph * p.ep_Wo + pw) * p.y_ps + m);
      if (p.vec_out) {
        half8 h;
#pragma unroll
        for (int e = 0; e < 8; ++e) h[e] = (_Float16)mx[e];
        *reinterpret_cast<half8*>(dst) = h;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (m + e < p.M) dst[e] = (_Float16)mx[e];
      }
    }
    return;
  }
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

// ------------------------------------------------------------------ LDS-DMA variant (16-B NHWC)
// conv_f16_kernel spends most of its time moving the staged operands from VGPRs into LDS
// (ds_write_b128: ablating those stores alone took 35-45 % off the 3x3 layers, the MFMAs 10 %).
// Here every 16-B operand chunk goes global -> LDS by buffer_load_dwordx4 ... lds (no VGPR round
// trip, no store instruction), into a ring of three K stages, each its own __shared__ array so
// the compiler's wait for an LDS-DMA write only covers reads of the same stage:
//   * stage layout: BMA rows of A (weights) then BN rows of B (pixels), 64 B (one 32-k stage) per
//     row, no padding; a wave-instruction fills 64 consecutive 16-B slots.  Slot (row, q) holds
//     k-chunk q ^ ((row >> 2) & 3), which makes the MFMA fragment reads (ds_read_b128, lane l:
//     row l & 31, chunk ks/8 + (l >> 5)) bank-conflict free.
//   * a tap outside the image (or a group past K) gets an out-of-range buffer offset: the load
//     returns zeros, which is the reference's zero padding.
//   * stage t + 2 is issued after the barrier that publishes stage t; each wave waits with a counted
//     vmcnt for its own chunks of stage t only, so two stages of loads stay in flight.
// Same GEMM, k order, MFMA chain and epilogue arithmetic as conv_f16_kernel<..., F16_X_NHWC_VEC>:
// bit-identical results.
typedef int int4v __attribute__((ext_vector_type(4)));

// buffer descriptor {base, stride 0, num_records bytes, raw-buffer flags}: offsets >= num_records
// (0x80000000) read as zeros
__device__ __forceinline__ int4v buffer_desc(const void* base, int bytes) {
  const unsigned long long b = reinterpret_cast<unsigned long long>(base);
  return int4v{(int)(unsigned)b, (int)((b >> 32) & 0xffff), bytes, 0x00020000};
}

// One 16-B-per-lane LDS-DMA (lane i -> lds_addr + 16 i).  Inline asm rather than the builtin so
// the compiler does not guard later LDS reads with its own conservative vmcnt(0) (it cannot tell
// which ring stage a DMA writes); the kernel waits with counted vmcnt itself.  M0 is restored.
__device__ __forceinline__ void lds_dma16(int4v rsrc, unsigned lds_addr, int voffset) {
  int m0save;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(m0save)
      : "s"(__builtin_amdgcn_readfirstlane(lds_addr)), "v"(voffset), "s"(rsrc)
      : "memory");
}

__device__ __forceinline__ unsigned lds_addr_of(const _Float16* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) _Float16*)p;
}

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256, 2) void conv_f16_dma_kernel(ConvParams p) {
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 32, FN = TN / 32;
  constexpr int AV = (BM * 4 + 255) / 256;  // A DMA instructions per thread per stage (rows padded to AV*64)
  constexpr int BMA = AV * 64;              // A rows in the stage (rows >= BM load zeros)
  constexpr int BV = BN * 4 / 256;          // B DMA instructions per thread per stage
  constexpr int NQ = AV + BV;               // DMA instructions per wave per stage (uniform)
  constexpr int SH = (BMA + BN) * 32;       // halves per stage
  constexpr int SR = 40;                    // epilogue staging row (32 channels + 8 pad, halves)
  static_assert(WM * WN == 4 && FM >= 1 && FN >= 1 && BN % 64 == 0 && 256 % BN == 0, "tile");
  static_assert(2 * TN * SR <= SH, "epilogue staging of two waves fits one stage array");
  __shared__ __attribute__((aligned(16))) _Float16 S0[SH];
  __shared__ __attribute__((aligned(16))) _Float16 S1[SH];
  __shared__ __attribute__((aligned(16))) _Float16 S2[SH];
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
  const int Kp = (p.K + 31) & ~31;
  const int P = p.P;

  for (int i = tid; i < BM; i += 256) sbias[i] = (p.bias && m0 + i < p.M) ? p.bias[m0 + i] : 0.0f;

  // this thread's slots: row (tid >> 2) + 64v, slot tid & 3 -> k-chunk g (same for A and B rows)
  const int g = (tid & 3) ^ ((tid >> 4) & 3);
  const int prow = tid >> 2;
  int aoff[AV];
#pragma unroll
  for (int v = 0; v < AV; ++v) {
    const int row = prow + 64 * v;
    aoff[v] = row < BM ? ((m0 + row) * Kp + g * 8) * 2 : (int)0x80000000;
  }
  int xoff[BV], ih0[BV], iw0[BV];
  bool nok[BV];
#pragma unroll
  for (int u = 0; u < BV; ++u) {
    const int bn = n0 + prow + 64 * u;
    nok[u] = bn < p.Ntot;
    const int nn = nok[u] ? bn : 0;
    const int img = nn / P;
    const int pix = nn - img * P;
    const int oh = pix / p.Wo, ow = pix - oh * p.Wo;
    ih0[u] = oh * p.sh - p.pt;
    iw0[u] = ow * p.sw - p.pl;
    xoff[u] = img * (int)p.x_nstride + (ih0[u] * p.W + iw0[u]) * p.x_ps;
  }
  const int4v wrsrc = buffer_desc(p.wp, p.Mp * Kp * 2);
  const int4v xrsrc = buffer_desc(p.x, (int)p.x_bytes);
  typedef const __attribute__((address_space(4))) long long* ktab_cptr;
  const ktab_cptr ktab = (ktab_cptr)p.ktab;

  // issue stage `st` (k0 = st * 32) into stage array SA: every wave NQ DMA instructions
#define ORE_HD_ISSUE(SA, K0)                                                                         \
  {                                                                                                  \
    const int k0_ = (K0);                                                                            \
    _Pragma("unroll") for (int v_ = 0; v_ < AV; ++v_)                                                \
      lds_dma16(wrsrc, lds_addr_of((SA) + (v_ * 256 + wave * 64) * 8), aoff[v_] < 0 ? aoff[v_] : aoff[v_] + k0_ * 2); \
    const int kb_ = k0_ >> 3;                                                                        \
    const long long e0_ = ktab[kb_], e1_ = ktab[kb_ + 1], e2_ = ktab[kb_ + 2], e3_ = ktab[kb_ + 3];  \
    const long long w_ = g == 0 ? e0_ : g == 1 ? e1_ : g == 2 ? e2_ : e3_;                           \
    const int ex_ = (int)w_, ey_ = (int)(w_ >> 32);                                                  \
    const int r_ = ey_ >> 16, s_ = ey_ & 0x7fff;                                                     \
    _Pragma("unroll") for (int u_ = 0; u_ < BV; ++u_) {                                              \
      const bool ok_ = nok[u_] & ((unsigned)(ih0[u_] + r_) < (unsigned)p.H) &                        \
                       ((unsigned)(iw0[u_] + s_) < (unsigned)p.W);                                   \
      lds_dma16(xrsrc, lds_addr_of((SA) + (BMA * 4 + u_ * 256 + wave * 64) * 8),                     \
                ok_ ? (xoff[u_] + ex_) * 2 : (int)0x80000000);                                       \
    }                                                                                                \
  }

  floatx16h acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  const int sw = (lcol >> 2) & 3;  // fragment rows R have (R >> 2) & 3 == (lcol >> 2) & 3
#define ORE_HD_COMPUTE(SA)                                                                           \
  _Pragma("unroll") for (int ks = 0; ks < 32; ks += 16) {                                            \
    const int q_ = ((ks >> 3) + lrow) ^ sw;                                                          \
    half8 af[FM], bf[FN];                                                                            \
    _Pragma("unroll") for (int i = 0; i < FM; ++i)                                                   \
      af[i] = *reinterpret_cast<const half8*>((SA) + (wm0 + i * 32 + lcol) * 32 + q_ * 8);           \
    _Pragma("unroll") for (int j = 0; j < FN; ++j)                                                   \
      bf[j] = *reinterpret_cast<const half8*>((SA) + (BMA + wn0 + j * 32 + lcol) * 32 + q_ * 8);     \
    _Pragma("unroll") for (int i = 0; i < FM; ++i)                                                   \
    _Pragma("unroll") for (int j = 0; j < FN; ++j)                                                   \
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[j], acc[i][j], 0, 0, 0);          \
  }
  // stage t in CUR; NX2 receives stage t + 2 (read last at stage t - 1, before this barrier)
#define ORE_HD_STEP(CUR, NX2)                                                                        \
  {                                                                                                  \
    if (t + 1 < ntk)                                                                                 \
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NQ) : "memory"); /* stage t + 1 may stay in flight */ \
    else                                                                                             \
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                               \
    __builtin_amdgcn_s_barrier();                                                                    \
    if (t + 2 < ntk) ORE_HD_ISSUE(NX2, (t + 2) * 32);                                                \
    ORE_HD_COMPUTE(CUR);                                                                             \
    if (++t >= ntk) break;                                                                           \
  }

  const int ntk = Kp / 32;
  ORE_HD_ISSUE(S0, 0);
  if (ntk > 1) ORE_HD_ISSUE(S1, 32);
  __syncthreads();  // sbias (the DMA stays in flight: the barrier's own wait is vmcnt-free here)
  for (int t = 0;;) {
    ORE_HD_STEP(S0, S2);
    ORE_HD_STEP(S1, S0);
    ORE_HD_STEP(S2, S1);
  }
#undef ORE_HD_STEP
#undef ORE_HD_COMPUTE
#undef ORE_HD_ISSUE

  // epilogue: + bias (f32), optional Relu, one rounding, NHWC store.  Per 32-channel fragment
  // row i each wave stages [TN pixels][32 channels] (80-B rows) in half of S0 / S1 (waves 0-1 /
  // 2-3), then writes each pixel's 64-B channel run with 16-B stores (host: M % 8 == 0,
  // y_ps % 8 == 0, aligned y) or 2-byte stores.
  __syncthreads();  // every wave is done with the stage arrays
  _Float16* stg = (wave < 2 ? S0 : S1) + (wave & 1) * (TN * SR);
  _Float16* __restrict__ y = reinterpret_cast<_Float16*>(p.y);
  const int yps = p.y_ps;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ch = 8 * q + 4 * lrow;
        half4 h;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = acc[i][j][4 * q + e] + sbias[wm0 + i * 32 + ch + e];
          if (p.relu) v = fmaxf(v, 0.0f);
          h[e] = (_Float16)v;
        }
        *reinterpret_cast<half4*>(stg + (j * 32 + lcol) * SR + ch) = h;
      }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int mb = m0 + wm0 + i * 32;
    if (p.vec_out) {
#pragma unroll
      for (int idx = lane; idx < TN * 4; idx += 64) {
        const int px = idx >> 2, cg = idx & 3;
        const int n = n0 + wn0 + px, m = mb + cg * 8;
        if (n < p.Ntot && m < p.M) {
          const int img = n / P, pix = n - img * P;
          *reinterpret_cast<half8*>(y + (unsigned)(img * (int)p.y_nstride + pix * yps + m)) =
              *reinterpret_cast<const half8*>(stg + px * SR + cg * 8);
        }
      }
    } else {
      for (int idx = lane; idx < TN * 32; idx += 64) {
        const int px = idx >> 5, ch = idx & 31;
        const int n = n0 + wn0 + px, m = mb + ch;
        if (n < p.Ntot && m < p.M) {
          const int img = n / P, pix = n - img * P;
          y[(unsigned)(img * (int)p.y_nstride + pix * yps + m)] = stg[px * SR + ch];
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// Wh[m][k] = f16(W[m][c][r][s]) zero padded to Mp x Kp, k in the order the operand mode gathers:
//   F16_X_NCHW32: (c, r, s) (the reference's); F16_X_NHWC_*: (r, s, c), c fastest;
//   F16_X_NHWC_PAIR: (r, s', c') with s' < kw rounded up to even and c' < 4 (zero weights for the
//   padding tap and channels).
__global__ __launch_bounds__(256) void pack_weights_f16_kernel(const float* __restrict__ w, int xmode, int M, int C,
                                                               int kh, int kw, int Mp, int Kp, _Float16* __restrict__ wh) {
  const int KK = kh * kw, K = C * KK, kwp = (kw + 1) & ~1;
  const long long total = (long long)Mp * Kp;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int m = (int)(i / Kp), k = (int)(i - (long long)m * Kp);
    float v = 0.0f;
    if (m < M) {
      if (xmode == F16_X_NHWC_PAIR) {
        const int c = k & 3, t = k >> 2, r = t / kwp, sx = t - r * kwp;
        if (r < kh && sx < kw && c < C) v = w[(((long long)m * C + c) * kh + r) * kw + sx];
      } else if (k < K) {
        v = xmode == F16_X_NCHW32 ? w[(long long)m * K + k] : w[((long long)m * C + (k % C)) * KK + k / C];
      }
    }
    wh[i] = (_Float16)v;
  }
}

int f16_conv_k(int xmode, int C, int kh, int kw) {
  return xmode == F16_X_NHWC_PAIR ? kh * ((kw + 1) & ~1) * 4 : C * kh * kw;
}

void launch_pack_weights_f16(const float* w, int xmode, int M, int C, int kh, int kw, int Mp, void* wh,
                             hipStream_t s) {
  const int Kp = conv_packed_kp(f16_conv_k(xmode, C, kh, kw));
  long long blocks = ((long long)Mp * Kp + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pack_weights_f16_kernel, dim3((unsigned)blocks), dim3(256), 0, s, w, xmode, M, C, kh, kw, Mp, Kp,
                     static_cast<_Float16*>(wh));
}

// Gather tables over an NHWC input with pixel stride cs, one entry {x offset, (r << 16) | s} per k
// (F16_X_NHWC_ELEM, k = (r, s, c)) or per group of 8 k (F16_X_NHWC_VEC: c = the group's first
// channel; F16_X_NHWC_PAIR: taps s (even) and s + 1 of 4 channels, bit 15 set when s + 1 is the
// padding tap).  Entries past K carry r = 1 << 14, which no bounds check passes (read as zeros).
__global__ __launch_bounds__(256) void ktab_nhwc_kernel(int2* __restrict__ ktab, int xmode, int C, int kh, int kw, int n,
                                                        int cs, int W) {
  const int K = C * kh * kw, kwp = (kw + 1) & ~1;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    int2 e = make_int2(0, (1 << 14) << 16);
    if (xmode == F16_X_NHWC_PAIR) {
      const int t = 2 * i, r = t / kwp, sx = t - r * kwp;
      if (r < kh) e = make_int2((r * W + sx) * cs, (r << 16) | sx | (sx + 1 >= kw ? 0x8000 : 0));
    } else {
      const int k = xmode == F16_X_NHWC_VEC ? 8 * i : i;
      if (k < K) {
        const int rs = k / C, c = k - rs * C, r = rs / kw, sx = rs - r * kw;
        e = make_int2((r * W + sx) * cs + c, (r << 16) | sx);
      }
    }
    ktab[i] = e;
  }
}

void launch_ktab_nhwc(int2* ktab, int xmode, int C, int kh, int kw, int cs, int W, hipStream_t s) {
  const int n = conv_packed_kp(f16_conv_k(xmode, C, kh, kw)) / (xmode == F16_X_NHWC_ELEM ? 1 : 8);
  hipLaunchKernelGGL(ktab_nhwc_kernel, dim3((n + 255) / 256), dim3(256), 0, s, ktab, xmode, C, kh, kw, n, cs, W);
}

// f32 NCHW (plane stride x_ps, image stride x_nstride) -> f16 NHWC with CS channels per pixel
// (channels >= C zero): the operand of F16_X_NHWC_PAIR (CS = 4) for the first conv.  One thread per
// pixel: coalesced plane reads, one 8-B store.
template <int CS>
__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(const float* __restrict__ x, _Float16* __restrict__ y,
                                                           long long pixels, int HW, int C, long long x_nstride,
                                                           int x_ps) {
  typedef _Float16 hv __attribute__((ext_vector_type(CS)));
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < pixels; i += (long long)gridDim.x * 256) {
    const long long n = i / HW;
    const int q = (int)(i - n * HW);
    const float* xp = x + n * x_nstride + q;
    hv h;
#pragma unroll
    for (int c = 0; c < CS; ++c) h[c] = c < C ? (_Float16)xp[(long long)c * x_ps] : (_Float16)0.0f;
    *reinterpret_cast<hv*>(y + i * CS) = h;
  }
}

void launch_nchw_to_nhwc(const float* x, void* y, int N, int C, int HW, long long x_nstride, int x_ps, int cs,
                         hipStream_t s) {
  const long long pixels = (long long)N * HW;
  if (pixels <= 0) return;
  long long b = (pixels + 255) / 256;
  if (b > 256 * 32) b = 256 * 32;
  (void)cs;  // 4 (F16_X_NHWC_PAIR)
  hipLaunchKernelGGL(nchw_to_nhwc_kernel<4>, dim3((unsigned)b), dim3(256), 0, s, x, static_cast<_Float16*>(y), pixels,
                     HW, C, x_nstride, x_ps);
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
    case F16_X_NHWC_PAIR: hipLaunchKernelGGL((conv_f16_kernel<BM, BN, WM, WN, F16_X_NHWC_PAIR>), grid, block, 0, s, p); break;
    default:
      // LDS-DMA B tiles (run_conv_f16 launches image chunks whose extent fits the buffer resource)
      hipLaunchKernelGGL((conv_f16_dma_kernel<BM, BN, WM, WN>), grid, block, 0, s, p);
      break;
  }
}

// pooled epilogue (EP): BM x 256 tiles of 1 x 4 waves, the N tile a 13 x 19 conv patch
template <int BM>
static void launch_f16_epool_cfg(const ConvParams& p0, int xmode, hipStream_t s) {
  ConvParams p = p0;
  p.mtiles = (p.M + BM - 1) / BM;
  p.ntiles = p.N * p.ep_tr * p.ep_tc;
  dim3 grid((unsigned)(p.mtiles * p.ntiles)), block(256);
  switch (xmode) {
    case F16_X_NCHW32: hipLaunchKernelGGL((conv_f16_kernel<BM, 256, 1, 4, F16_X_NCHW32, 1>), grid, block, 0, s, p); break;
    case F16_X_NHWC_ELEM: hipLaunchKernelGGL((conv_f16_kernel<BM, 256, 1, 4, F16_X_NHWC_ELEM, 1>), grid, block, 0, s, p); break;
    case F16_X_NHWC_PAIR: hipLaunchKernelGGL((conv_f16_kernel<BM, 256, 1, 4, F16_X_NHWC_PAIR, 1>), grid, block, 0, s, p); break;
    default: hipLaunchKernelGGL((conv_f16_kernel<BM, 256, 1, 4, F16_X_NHWC_VEC, 1>), grid, block, 0, s, p); break;
  }
}

void launch_conv_f16_epool(const ConvParams& p, int xmode, hipStream_t s) {
  // rows per tile as launch_conv_epool: 96 when it divides the channel count (conv1's 96), else 128,
  // or 32 for M <= 32
  if (p.M <= 32)
    launch_f16_epool_cfg<32>(p, xmode, s);
  else if (p.M % 96 == 0 || p.M < 96)
    launch_f16_epool_cfg<96>(p, xmode, s);
  else
    launch_f16_epool_cfg<128>(p, xmode, s);
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
    int i = 0;
    for (; i + 8 <= HW; i += 8) {  // 8 loads in flight ahead of the (sequential) adds
      _Float16 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = xp[(long long)(i + u) * cs];
#pragma unroll
      for (int u = 0; u < 8; ++u) s = s + (float)v[u];
    }
    for (; i < HW; ++i) s = s + (float)xp[(long long)i * cs];
    y[idx] = s / (float)HW;
  }
}

void launch_gap_nhwc(const void* x, float* y, int N, int C, int HW, int cs, long long nstride, hipStream_t s) {
  const long long total = (long long)N * C;
  if (total <= 0) return;
  // (two channels per lane with 4-B loads measured slower: 20 -> 23.5 us for SqueezeNet's pool10 --
  // half the lanes, each with two dependent sums)
  hipLaunchKernelGGL(gap_nhwc_kernel, dim3(grid_for(total)), dim3(256), 0, s, static_cast<const _Float16*>(x), y, N, C,
                     HW, cs, nstride);
}

// ------------------------------------------------------------------ 1x1 conv + Relu + GAP (f16)
// SqueezeNet's conv10 (512 -> 1000, 13 x 13) -> relu10 -> pool10 in one launch.  The separate path is
// conv_f16_dma_kernel (128 x 128 tiles, a barrier per 32 k: 8 MFMAs per wave between barriers) writing
// the 87 MB f16 map, then gap_nhwc_kernel reading it back.  Here one workgroup owns one image's P <= 32 NF
// pixels x 128 output channels (4 waves x 32): per 64-channel K chunk the image's pixels are staged
// in LDS (double-buffered, the next chunk's loads in flight) and each wave runs 4 k-steps x NF
// v_mfma_f32_32x32x16_f16 (A = its 32 weight rows from L2, one chunk ahead) -- 24 MFMAs per barrier.
// Epilogue: bias + Relu + one rounding to f16 (what conv_f16 stores), the wave's [pixels][32 channels]
// tile to LDS, then lane c < 32 sums its channel over the pixels in order in f32 and divides by P
// (gap_nhwc_kernel's arithmetic).  Same operands, k order and MFMA chain as the separate conv, the
// same f16 values in the same order into the same sum: bit-identical.
template <int NF>
__global__ __launch_bounds__(256, 2) void conv1x1_gap_f16_kernel(Conv1x1GapF16 p) {
  constexpr int KC = 64, BS = KC + 8;      // K chunk; LDS pixel stride (halves, 144 B)
  constexpr int NPX = 32 * NF, STAGE = NPX * BS, TS = 36;  // staged pixels; GAP tile pixel stride
  static_assert(4 * NPX * TS <= 2 * STAGE, "the GAP tiles fit the stage buffers");
  extern __shared__ __attribute__((aligned(16))) _Float16 gsm[];
  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-grouped ids: the channel blocks of one image are consecutive on one XCD, so the image's
  // staged input is fetched from HBM once and re-read from that XCD's L2 (with the plain block id
  // they were spread over the eight XCDs: 343 MB fetched for a 44 MB input at B = 256)
  const int mblocks = (p.M + 127) / 128, wg = xcd_block_id();
  const int img = wg / mblocks, m0 = (wg - img * mblocks) * 128 + 32 * wave;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<_Float16*>(static_cast<const _Float16*>(p.x) + (long long)img * p.x_nstride), (short)0,
      p.P * p.x_cs * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.wp), (short)0, p.Mp * p.Kp * 2, 0x00020000);
  // this thread's staged 16-B groups q = tid + 256 u: pixel q >> 3 (>= P: zeros), channels 8 (q & 7)
  int xo[NF], so[NF];
#pragma unroll
  for (int u = 0; u < NF; ++u) {
    const int q = tid + 256 * u, px = q >> 3, g = q & 7;
    xo[u] = px < p.P ? (px * p.x_cs + 8 * g) * 2 : (int)0x80000000;
    so[u] = px * BS + 8 * g;
  }
  const int aoff = ((m0 + lr) * p.Kp + 8 * h) * 2;  // rows past Mp read 0 (buffer range)
  half8 xv[NF], a[2][4];
  auto load = [&](int c, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NF; ++u)
      xv[u] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(xr, xo[u], c * KC * 2, 0));
#pragma unroll
    for (int t = 0; t < 4; ++t)
      a[slot][t] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(wr, aoff, (c * KC + 16 * t) * 2, 0));
  };
  auto store = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NF; ++u) *reinterpret_cast<half8*>(gsm + buf * STAGE + so[u]) = xv[u];
  };
  floatx16h acc[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.0f;
  const int nch = p.C / KC;
  // chunk c from stage buffer BUF (a compile-time constant after inlining: the register rings stay
  // statically indexed)
  auto chunk = [&](int c, int BUF) __attribute__((always_inline)) {
    if (c + 1 < nch) load(c + 1, BUF ^ 1);  // in flight during this chunk's MFMAs
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      half8 b[NF];
#pragma unroll
      for (int j = 0; j < NF; ++j) b[j] = *reinterpret_cast<const half8*>(gsm + BUF * STAGE + (32 * j + lr) * BS + 16 * t + 8 * h);
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[BUF][t], b[j], acc[j], 0, 0, 0);
    }
    if (c + 1 < nch) store(BUF ^ 1);  // that buffer was last read in chunk c - 1 (the barrier below it)
    __syncthreads();
  };
  load(0, 0);
  store(0);
  __syncthreads();
  for (int c = 0; c < nch; c += 2) {
    chunk(c, 0);
    if (c + 1 < nch) chunk(c + 1, 1);
  }
  // epilogue: element i of lane (lr, h) in fragment j = channel m0 + 8 (i >> 2) + 4 h + (i & 3) at
  // pixel 32 j + lr; the wave's tile [pixel][32 channels] (f16) in the stage buffers
  _Float16* tl = gsm + wave * NPX * TS;
  float bv[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int m = m0 + 8 * (i >> 2) + 4 * h + (i & 3);
    bv[i] = (p.bias && m < p.M) ? p.bias[m] : 0.0f;
  }
#pragma unroll
  for (int j = 0; j < NF; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      half4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc[j][4 * q + e] + bv[4 * q + e];
        if (p.relu) v = fmaxf(v, 0.0f);
        o[e] = (_Float16)v;
      }
      *reinterpret_cast<half4*>(tl + (32 * j + lr) * TS + 8 * q + 4 * h) = o;
    }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane < 32 && m0 + lane < p.M) {  // one lane per channel: the pixels in order, as gap_nhwc_kernel
    float s = 0.0f;
    int px = 0;
    for (; px + 8 <= p.P; px += 8) {  // 8 LDS reads in flight ahead of the (sequential) adds
      _Float16 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = tl[(px + u) * TS + lane];
#pragma unroll
      for (int u = 0; u < 8; ++u) s = s + (float)v[u];
    }
    for (; px < p.P; ++px) s = s + (float)tl[px * TS + lane];
    p.y[(long long)img * p.y_nstride + m0 + lane] = s / (float)p.P;
  }
}

bool conv1x1_gap_f16_eligible(const Conv1x1GapF16& p) {
  return p.N > 0 && p.C > 0 && p.C % 64 == 0 && p.P >= 1 && p.P <= 256 && p.M >= 1 && p.x_cs % 8 == 0 &&
         p.x_cs >= p.C && p.x_nstride % 8 == 0 && (reinterpret_cast<uintptr_t>(p.x) & 15) == 0 && p.Kp >= p.C &&
         p.Kp % 8 == 0 && p.Mp >= p.M && (long long)p.P * p.x_cs * 2 < (1LL << 31) &&
         (long long)p.Mp * p.Kp * 2 < (1LL << 31) && p.y_nstride >= p.M;
}

template <int NF>
static void launch_cg(const Conv1x1GapF16& p, hipStream_t s) {
  const size_t lds = size_t(2) * 32 * NF * (64 + 8) * 2;
  const unsigned grid = (unsigned)(p.N * ((p.M + 127) / 128));
  hipLaunchKernelGGL((conv1x1_gap_f16_kernel<NF>), dim3(grid), dim3(256), lds, s, p);
}

void launch_conv1x1_gap_f16(const Conv1x1GapF16& p, hipStream_t s) {
  switch ((p.P + 31) / 32) {
    case 1: launch_cg<1>(p, s); break;
    case 2: launch_cg<2>(p, s); break;
    case 3: launch_cg<3>(p, s); break;
    case 4: launch_cg<4>(p, s); break;
    case 5: launch_cg<5>(p, s); break;
    case 6: launch_cg<6>(p, s); break;
    case 7: launch_cg<7>(p, s); break;
    default: launch_cg<8>(p, s); break;
  }
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
