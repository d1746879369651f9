// First conv + its 3x3 / stride-2 MaxPool for f16 models (config 5): SqueezeNet's conv1 (3 -> 96,
// 7x7 / stride 2) + Relu + pool1 in one launch that reads the f32 NCHW model input directly (the
// reference: convolution_op.rs:422-480, relu_op.rs, max_pool_op.rs:248-337).
//
// The path it replaces is two launches: nchw_to_nhwc_kernel<4> (f32 NCHW -> f16 NHWC4, 154 MB read,
// 103 MB written at B = 256) and conv_f16_kernel<..., F16_X_NHWC_PAIR, EP = 1>, whose per-stage
// register gather (two 8-B taps per lane, per-tap bounds checks) and VGPR -> LDS operand staging kept
// the MFMAs at ~15 % of the f16 peak.  Here:
//   * a persistent workgroup (two per CU) stages the whole packed weight matrix (K = kh x kwp x 4,
//     PAIR order (r, s', c'), 96 x 224 halves = 43 KB for conv1) in LDS once, rows permuted within
//     every 32-row block so accumulator element 8g + e of lane half h is channel 16 g + 8 h + e;
//   * per tile (the 13 x 19 conv patch feeding 6 x 9 pooled outputs, as the EP kernel) it stages the
//     patch's input window in LDS as f16 NHWC4 (rounding f32 -> f16 as nchw_to_nhwc_kernel does;
//     zeros outside the image) and reads every B fragment -- two horizontally adjacent taps x 4
//     channels, one 16-B aligned ds_read_b128 since the column stride is even -- from it;
//   * each wave computes 2 pixel fragments x MF channel fragments (MF = 3: 96 channels) over the
//     K / 16 k-steps, every A fragment from LDS;
//   * per channel fragment the conv values (bias, Relu, f16; 0 outside the conv plane) go to an LDS
//     tile [pixel][32 channels] and each (pooled output, 8 channels) takes its 3x3 max from -FLT_MAX
//     in f32 (the EP kernel's arithmetic) and leaves by one 16-B NHWC store.
// Same operands (the PAIR padding tap meets a zero weight; the gather path zeroes the operand too:
// zero products either way), same k order, same MFMA chain and epilogue as the two-launch path:
// bit-identical output (tests/test_f16_gpu.py).
#include <float.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>

#include "ore_kernels.h"

namespace ore {

namespace {

typedef _Float16 c1h8 __attribute__((ext_vector_type(8)));
typedef _Float16 c1h4 __attribute__((ext_vector_type(4)));
typedef float c1f16 __attribute__((ext_vector_type(16)));
constexpr int C1_PR = EPOOL_TILE_PR, C1_PC = EPOOL_TILE_PC;                // pooled outputs per tile
constexpr int C1_RC = 2 * C1_PR + 1, C1_CC = 2 * C1_PC + 1, C1_NPX = C1_RC * C1_CC;  // conv patch (13 x 19)
constexpr int C1_TS = 40;                                                  // conv tile pixel stride (halves)
static_assert(C1_NPX <= 256, "one 256-pixel patch per tile (8 fragments)");

typedef unsigned short c1u8 __attribute__((ext_vector_type(8)));

// 3x3 max of 8 channels of conv-tile pixels (row stride C1_CC pixels of C1_TS halves) from -FLT_MAX in
// f32 (the separate pool's arithmetic).  After the Relu every value is +0 or positive, so its f16 bits
// order like the value: the max is then 4 v_pk_max_u16 per tap on the raw bits (exact; the f32 route
// costs 8 conversions and 8 maxima per tap)
__device__ __forceinline__ c1h8 c1_pool8(const _Float16* base, bool relu) {
  if (relu) {
    c1u8 m = __builtin_bit_cast(c1u8, *reinterpret_cast<const c1h8*>(base));
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s = 0; s < 3; ++s)
        if (r || s)
          m = __builtin_elementwise_max(m, __builtin_bit_cast(c1u8, *reinterpret_cast<const c1h8*>(
                                                                   base + (r * C1_CC + s) * C1_TS)));
    return __builtin_bit_cast(c1h8, m);
  }
  float mx[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) mx[e] = -FLT_MAX;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const c1h8 v = *reinterpret_cast<const c1h8*>(base + (r * C1_CC + s) * C1_TS);
#pragma unroll
      for (int e = 0; e < 8; ++e) mx[e] = fmaxf(mx[e], (float)v[e]);
    }
  c1h8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (_Float16)mx[e];
  return o;
}


struct C1Geom {
  int KS;      // k-steps of 16
  int hr, hc;  // input window rows / columns of a tile
  int w_halves, halo_halves, lds_bytes;
};

// A fragments: staged in LDS once per persistent workgroup (read from L2 per k-step instead, three
// workgroups per CU fit by LDS but 158 VGPRs: measured 236 vs 179 us for conv1 + pool1 + squeeze at
// B = 256)
constexpr bool C1_WLDS = true;

__host__ __device__ inline C1Geom c1_geom(int MF, int kh, int kwp, int sh, int sw, bool sq = false) {
  C1Geom g;
  g.KS = kh * kwp * 4 / 16;
  g.hr = (C1_RC - 1) * sh + kh;
  g.hc = (C1_CC - 1) * sw + kwp;
  g.w_halves = C1_WLDS ? g.KS * MF * 32 * 16 : 0;
  g.halo_halves = (g.hr * g.hc * 4 + 7) / 8 * 8;
  g.lds_bytes = (g.w_halves + g.halo_halves + C1_NPX * C1_TS) * 2 + MF * 32 * 4 + (sq ? 64 * C1_TS * 2 + 32 * 4 : 0);
  return g;
}

template <int MF, int KH, int KW, int S, int SQ>
__global__ __launch_bounds__(256, 2) void conv_pair_pool_f16_kernel(ConvParams p, C1Squeeze sq) {
  constexpr int KWP = (KW + 1) & ~1, KS = KH * KWP * 4 / 16;
  constexpr int HR = (C1_RC - 1) * S + KH, HC = (C1_CC - 1) * S + KWP;  // input window of a tile
  constexpr int NQ = (HR * HC + 255) / 256;                              // window pixels per thread
  static_assert(KH * KWP % 4 == 0, "whole k-steps");
  extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
  constexpr int W_HALVES = C1_WLDS ? KS * MF * 32 * 16 : 0, HALO_HALVES = (HR * HC * 4 + 7) / 8 * 8;
  _Float16* Ws = smem;                      // [KS][MF * 32][16]
  _Float16* halo = smem + W_HALVES;         // [HR][HC][4]
  _Float16* ct = halo + HALO_HALVES;        // [C1_NPX][C1_TS]
  float* sbias = reinterpret_cast<float*>(ct + C1_NPX * C1_TS);  // [MF * 32]
  // SQ: the pooled values of one fragment [64 pixels][40] (all four waves pool, waves 0 and 1 run the
  // squeeze's MFMAs, its weights in registers) and the squeeze bias
  _Float16* pt = reinterpret_cast<_Float16*>(sbias + MF * 32);
  float* qbias = reinterpret_cast<float*>(pt + (SQ ? 64 * C1_TS : 0));
  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Kp = (p.K + 31) & ~31;
  const _Float16* __restrict__ wh = reinterpret_cast<const _Float16*>(p.wp);  // [Mp][Kp]

  // weights once: LDS row R of each 32-row block <- packed row (R & ~31) + 16 (i >> 1) + 8 hh +
  // 4 (i & 1) + j for R % 32 = 8 i + 4 hh + j (rows past M zero)
  for (int q = tid; C1_WLDS && q < KS * MF * 64; q += 256) {
    const int t = q / (MF * 64), rem = q - t * (MF * 64), R = rem >> 1, hh8 = rem & 1;
    const int r = R & 31, i = r >> 3, hq = (r >> 2) & 1, j = r & 3;
    const int m = (R & ~31) + 16 * (i >> 1) + 8 * hq + 4 * (i & 1) + j;
    c1h8 v = {};
    if (m < p.M) v = *reinterpret_cast<const c1h8*>(wh + m * Kp + 16 * t + 8 * hh8);
    *reinterpret_cast<c1h8*>(Ws + (t * MF * 32 + R) * 16 + 8 * hh8) = v;
  }

  for (int q = tid; q < MF * 32; q += 256) sbias[q] = (p.bias && q < p.M) ? p.bias[q] : 0.0f;
  if constexpr (SQ) {
    for (int q = tid; q < 32; q += 256) qbias[q] = q < sq.M ? sq.bias[q] : 0.0f;
  }
  const _Float16* __restrict__ wq = static_cast<const _Float16*>(sq.w);
  // the squeeze's A fragments (waves 0 and 1), loaded once per persistent workgroup: an L2 load per
  // fragment inside the epilogue sat between two barriers on every tile
  c1h8 aqr[SQ ? MF : 1][2];
  if constexpr (SQ) {
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int t = 0; t < 2; ++t) aqr[i][t] = *reinterpret_cast<const c1h8*>(wq + ((2 * i + t) * 32 + lr) * 16 + 8 * h);
  }

  // L2 weights: this lane's packed row of each fragment (the LDS permutation above, row lr of the
  // fragment), its 8 halves of a k-step at + 16 ks + 8 h; rows past M read a zero row (Mp >= 32 MF)
  const _Float16* arow_g[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    const int r = lr, ii = r >> 3, hq = (r >> 2) & 1, j = r & 3;
    const int m = 32 * i + 16 * (ii >> 1) + 8 * hq + 4 * (ii & 1) + j;
    arow_g[i] = wh + (long long)m * Kp + 8 * h;
  }
  // this lane's two patch pixels (fragments 2 wave, 2 wave + 1)
  int bofs[2], tpx[2];
  bool pin[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int px = (2 * wave + f) * 32 + lr;
    pin[f] = px < C1_NPX;
    const int pq = pin[f] ? px : 0;
    const int pr = pq / C1_CC, pc = pq - pr * C1_CC;
    bofs[f] = (pr * S * HC + pc * S) * 4;
    tpx[f] = pq * C1_TS + 8 * h;
  }
  // this thread's window pixels (fixed per thread: q = tid + 256 u)
  int qrow[NQ], qcol[NQ];
#pragma unroll
  for (int u = 0; u < NQ; ++u) {
    const int q = tid + 256 * u;
    qrow[u] = q < HR * HC ? q / HC : 1 << 20;  // past the window: never in the image
    qcol[u] = q - (q / HC) * HC;
  }
  const float* __restrict__ xf = p.x;
  _Float16* __restrict__ y = reinterpret_cast<_Float16*>(p.y);
  const int tpi = p.ep_tr * p.ep_tc, ntiles = p.N * tpi;
  const int ctile_tasks = C1_PR * C1_PC * 4;  // (pooled output, 8-channel group) of one fragment

  // the input window of a tile goes global -> registers (all NQ x C loads in flight) -> LDS, the
  // registers of tile t + 1 filled while tile t computes
  float xv[NQ][4];
  // raw buffer loads: an offset past the image's C planes reads 0 (the window's outside taps and the
  // channels >= C) with no branch, so the f16 conversion stays in store_window and the loads stay in flight (with
  // conditional loads the compiler converted each value right after its load, behind a vmcnt(0))
  auto load_window = [&](int tile) __attribute__((always_inline)) {
    const int tc = tile < ntiles ? tile : 0;
    const int img = tc / tpi, tt = tc - img * tpi;
    const int ph0 = (tt / p.ep_tc) * C1_PR, pw0 = (tt - (tt / p.ep_tc) * p.ep_tc) * C1_PC;
    const int ihb = (ph0 * 2 - p.ep_pt) * S - p.pt, iwb = (pw0 * 2 - p.ep_pl) * S - p.pl;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(xf + (long long)img * p.x_nstride), (short)0, p.C * p.x_ps * 4, 0x00020000);
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      const int ih = ihb + qrow[u], iw = iwb + qcol[u];
      const bool in = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      const int o = in ? (ih * p.W + iw) * 4 : (int)0x80000000;
#pragma unroll
      for (int ch = 0; ch < 4; ++ch)
        xv[u][ch] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, o, ch * p.x_ps * 4, 0));
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto store_window = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      const int q = tid + 256 * u;
      if (q < HR * HC) {
        c1h4 v;
#pragma unroll
        for (int ch = 0; ch < 4; ++ch) v[ch] = (_Float16)xv[u][ch];
        *reinterpret_cast<c1h4*>(halo + q * 4) = v;
      }
    }
  };
  const int wg0 = ORE_BAND_ID();
  load_window(wg0);
  store_window();

  for (int tile = wg0; tile < ntiles; tile += gridDim.x) {
    const int img = tile / tpi, tt = tile - img * tpi;
    const int ph0 = (tt / p.ep_tc) * C1_PR, pw0 = (tt - (tt / p.ep_tc) * p.ep_tc) * C1_PC;
    const int ohb = ph0 * 2 - p.ep_pt, owb = pw0 * 2 - p.ep_pl;  // conv coordinates of patch (0, 0)
    __syncthreads();  // this tile's window is in LDS; the previous tile's pool readers are done
    load_window(tile + gridDim.x);  // in flight during this tile's MFMAs

    c1f16 acc[MF][2];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][f][e] = 0.0f;
    c1h8 ag[2][MF];  // L2 weights: k-step ks + 1's fragments in flight during k-step ks
    if constexpr (!C1_WLDS) {
#pragma unroll
      for (int i = 0; i < MF; ++i) ag[0][i] = *reinterpret_cast<const c1h8*>(arow_g[i]);
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if constexpr (!C1_WLDS) {
        if (ks + 1 < KS) {
#pragma unroll
          for (int i = 0; i < MF; ++i) ag[(ks + 1) & 1][i] = *reinterpret_cast<const c1h8*>(arow_g[i] + 16 * (ks + 1));
        }
      }
      // the padding tap s + 1 = KW (odd KW) is read as it lies in the window (a finite value: image
      // data or an outside-the-image zero) and meets a zero weight (pack_weights_f16_kernel): its
      // products are zeros, as the gather path's zeroed operand gives
      const int pair = 2 * ks + h, tap = 2 * pair, r = tap / KWP, s = tap - r * KWP;
      c1h8 b[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) b[f] = *reinterpret_cast<const c1h8*>(halo + bofs[f] + (r * HC + s) * 4);
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        const c1h8 a = C1_WLDS ? *reinterpret_cast<const c1h8*>(Ws + ((ks * MF + i) * 32 + lr) * 16 + 8 * h) : ag[ks & 1][i];
#pragma unroll
        for (int f = 0; f < 2; ++f)
          acc[i][f] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b[f], acc[i][f], 0, 0, 0);
      }
    }

    // SQ: waves 0 and 1 own the tile's pooled pixels 32 w + lane (54 of 64 used) as the squeeze's B
    // columns; the squeeze accumulates over the channel fragments in order (k = channel)
    c1f16 sacc;
#pragma unroll
    for (int e = 0; e < 16; ++e) sacc[e] = 0.0f;
    const int kq = 32 * (wave & 1) + lr, kqc = kq < C1_PR * C1_PC ? kq : 0;
    const int qa = kqc / C1_PC, qb = kqc - qa * C1_PC;

    // per 32-channel fragment: conv tile, 3x3 max, 16-B NHWC stores (SQ: the squeeze's k-steps)
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      float bv[16];
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const float4 u0 = *reinterpret_cast<const float4*>(sbias + 32 * i + 16 * g + 8 * h);
        const float4 u1 = *reinterpret_cast<const float4*>(sbias + 32 * i + 16 * g + 8 * h + 4);
        bv[8 * g + 0] = u0.x; bv[8 * g + 1] = u0.y; bv[8 * g + 2] = u0.z; bv[8 * g + 3] = u0.w;
        bv[8 * g + 4] = u1.x; bv[8 * g + 5] = u1.y; bv[8 * g + 6] = u1.z; bv[8 * g + 7] = u1.w;
      }
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        if (!pin[f]) continue;
        const int px = (2 * wave + f) * 32 + lr, pr = px / C1_CC, pc = px - pr * C1_CC;
        const bool cok = (unsigned)(ohb + pr) < (unsigned)p.Ho && (unsigned)(owb + pc) < (unsigned)p.Wo;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          float av[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) av[e] = acc[i][f][8 * g + e];
          const c1h8 o = ore_f16_epilogue8(av, bv + 8 * g, p.relu != 0);
          const c1h8 zero = {};
          *reinterpret_cast<c1h8*>(ct + tpx[f] + 16 * g) = cok ? o : zero;  // 0 outside the conv plane
        }
      }
      __syncthreads();
      if (i == 0) store_window();  // every wave is past its k-loop: the window is free
      if constexpr (SQ) {
        {  // every thread: one (pooled pixel, 8 channels) of the 64 x 32 block (pixels >= 54: pixel 0)
          const int k = tid >> 2, cg = tid & 3, kc = k < C1_PR * C1_PC ? k : 0;
          const int a = kc / C1_PC, b = kc - a * C1_PC;
          *reinterpret_cast<c1h8*>(pt + k * C1_TS + cg * 8) =
              c1_pool8(ct + ((2 * a) * C1_CC + 2 * b) * C1_TS + cg * 8, p.relu != 0);
        }
        __syncthreads();
        // (waves 0 and 1 pooling their own squeeze operand from the conv tile, two 3x3 maxima per lane,
        // without this LDS block and barrier measured slower: 196-204 -> 203-212 us)
        if (wave < 2) {
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const c1h8 bq = *reinterpret_cast<const c1h8*>(pt + (32 * wave + lr) * C1_TS + 16 * t + 8 * h);
            sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(aqr[i][t], bq, sacc, 0, 0, 0);
          }
        }
      }
      if (!SQ && tid < ctile_tasks) {
        const int pp = tid >> 2, cg = tid & 3;
        const int a = pp / C1_PC, b = pp - a * C1_PC;
        const c1h8 o = c1_pool8(ct + ((2 * a) * C1_CC + 2 * b) * C1_TS + cg * 8, p.relu != 0);
        const int ph = ph0 + a, pw = pw0 + b, m = 32 * i + cg * 8;
        if (ph < p.ep_Ho && pw < p.ep_Wo && m < p.M)
          *reinterpret_cast<c1h8*>(y + (long long)img * p.y_nstride + (ph * p.ep_Wo + pw) * p.y_ps + m) = o;
      }
      if (i + 1 < MF) __syncthreads();  // the conv tile is rewritten by the next fragment
    }
    if constexpr (SQ) {
      // squeeze output: bias + Relu + one rounding; element 8 g + e of lane half h = channel 16 g + 8 h + e
      const int ph = ph0 + qa, pw = pw0 + qb;
      if (wave < 2 && kq < C1_PR * C1_PC && ph < p.ep_Ho && pw < p.ep_Wo) {
        _Float16* yq = static_cast<_Float16*>(sq.y) + (long long)img * sq.y_nstride + (ph * p.ep_Wo + pw) * sq.y_cs;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          const int ch = 16 * g + 8 * h;
          if (ch >= sq.M) continue;
          float av[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) av[e] = sacc[8 * g + e];
          *reinterpret_cast<c1h8*>(yq + ch) = ore_f16_epilogue8(av, qbias + ch, true);
        }
      }
    }
  }
}

template <int MF, int SQ>
static bool c1_dispatch(const ConvParams& p, const C1Squeeze& sq, unsigned grid, unsigned lds, hipStream_t s) {
  if (p.kh == 7 && p.kw == 7 && p.sh == 2) {
    hipLaunchKernelGGL((conv_pair_pool_f16_kernel<MF, 7, 7, 2, SQ>), dim3(grid), dim3(256), lds, s, p, sq);
    return true;
  }
  if (!SQ && p.kh == 3 && p.kw == 3 && p.sh == 2) {
    hipLaunchKernelGGL((conv_pair_pool_f16_kernel<MF, 3, 3, 2, 0>), dim3(grid), dim3(256), lds, s, p, sq);
    return true;
  }
  return false;
}

// ---------------------------------------------------------------------------------------------------
// Round 6: the f16 first conv + pool + squeeze as a band walker (the f32 kernel of the same
// name is ore_conv1_f32.hip's conv_band_pool_f32_kernel).  The patch kernel above computes 256 conv pixels per
// 13 x 19 patch for 220 used (the halo is recomputed by the neighbouring patch) and spends most of each tile in
// its pooled-epilogue chain (three barriers per 32-channel fragment).  Here one workgroup of 8 waves per CU owns
// an image and walks its conv rows in steps of four (SqueezeNet conv1: 28 steps of 4 x 109 conv columns):
//   * wave w computes conv row 4 s + w / 2 of the step, column pairs 31 (w & 1) + lr (two 32-pixel fragments of
//     v_mfma_f32_32x32x16_f16, the pair's two columns), all 96 channels; every conv output is computed once
//     (the pair shared by the two waves of a row aside: 1 of 63);
//   * A (the packed weights, the patch kernel's permuted rows) sits in LDS for the workgroup's life; B reads
//     the step's 13 input rows, staged in LDS as f16 NHWC4 (rounded as the patch kernel's window: the same
//     operands, k order and MFMA chain, so every conv output has the same bits);
//   * after the bias (the patch kernel's f32 add), the pair's pooled column takes max(col 2j, 2j + 1, 2j + 2) --
//     the two own columns in f32 before the f16 rounding (rounding is monotonic: the same bits as the max of the
//     patch kernel's rounded values), the third, rounded, by DPP wave_shl:1 from lane lr + 1 with every lane of
//     the wave enabled (tests/test_isa_guard.py) -- into a ring of horizontally pooled conv rows
//     [6 slots][56 columns][96 channels] (one writer per cell: no atomics);
//   * a step completes pooled rows 2 s - 1 and 2 s (conv rows 4 s - 2 .. 4 s + 2): waves 0-3 take their 3-row
//     maxima (the nine values of the patch kernel's max, exact) as the squeeze's B operands and run its six
//     MFMAs per fragment in the patch kernel's order; bias, Relu, one rounding, 16-B NHWC stores.
// Two barriers per step.  Bit-identical to the patch kernel (tests/test_f16_gpu.py::test_f16_conv1_band_*).
constexpr int FB_RW = 264;                                  // window row stride (pixels; reads reach col 257)
constexpr int FB_WR = 13;                                   // window rows: 4 conv rows per step (2 * 3 + 7)
constexpr int FB_SLOTS = 6;                                 // ring of conv rows 4 s - 2 .. 4 s + 3
constexpr int FB_HC = 56;                                   // ring columns (pooled columns <= 55)
constexpr int FB_CHS = 104;                                 // ring channel stride (halves): 96 + 8
constexpr int FB_KS = 14;                                   // k-steps: 7 rows x 8 taps x 4 channels / 16
constexpr int FB_W_HALVES = FB_KS * 96 * 16;                // 43008 B
constexpr int FB_WIN_HALVES = FB_WR * FB_RW * 4;            // 27456 B
constexpr int FB_RING_HALVES = FB_SLOTS * FB_HC * FB_CHS;   // 69888 B
constexpr int FB_NU = (FB_WR * 56 + 511) / 512;             // window units (row, 4 columns) per thread (2)
constexpr int FB_LDS = (FB_W_HALVES + FB_WIN_HALVES + FB_RING_HALVES) * 2 + (96 + 32) * 4;

__global__ __launch_bounds__(512, 1) void conv_band_pool_f16_kernel(ConvParams p, C1Squeeze sq) {
  constexpr int MF = 3;
  extern __shared__ __attribute__((aligned(16))) _Float16 fbs[];
  _Float16* Ws = fbs;                                                    // [KS][96][16]
  _Float16* win = Ws + FB_W_HALVES;                                      // [13][264][4]
  _Float16* ring = win + FB_WIN_HALVES;                                  // [6][56][104]
  float* sbias = reinterpret_cast<float*>(ring + FB_RING_HALVES);        // [96]
  float* qbias = sbias + 96;                                             // [32]
  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Kp = (p.K + 31) & ~31;
  const _Float16* __restrict__ wh = reinterpret_cast<const _Float16*>(p.wp);  // [Mp][Kp]
  // weights once, as the patch kernel stages them: LDS row R of each 32-row block <- packed row (R & ~31) +
  // 16 (i >> 1) + 8 hh + 4 (i & 1) + j for R % 32 = 8 i + 4 hh + j (rows past M zero)
  for (int q = tid; q < FB_KS * MF * 64; q += 512) {
    const int t = q / (MF * 64), rem = q - t * (MF * 64), R = rem >> 1, hh8 = rem & 1;
    const int r = R & 31, i = r >> 3, hq = (r >> 2) & 1, j = r & 3;
    const int m = (R & ~31) + 16 * (i >> 1) + 8 * hq + 4 * (i & 1) + j;
    c1h8 v = {};
    if (m < p.M) v = *reinterpret_cast<const c1h8*>(wh + m * Kp + 16 * t + 8 * hh8);
    *reinterpret_cast<c1h8*>(Ws + (t * MF * 32 + R) * 16 + 8 * hh8) = v;
  }
  for (int q = tid; q < 96; q += 512) sbias[q] = (p.bias && q < p.M) ? p.bias[q] : 0.0f;
  for (int q = tid; q < 32; q += 512) qbias[q] = q < sq.M ? sq.bias[q] : 0.0f;
  // the window's columns past the image (read by the last pairs' taps) stay zero: the staging writes < W
  for (int q = tid; q < FB_WIN_HALVES / 8; q += 512) reinterpret_cast<c1h8*>(win)[q] = c1h8{};
  // the squeeze's A fragments (waves 0-3), loaded once
  const _Float16* __restrict__ wq = static_cast<const _Float16*>(sq.w);
  c1h8 aqr[MF][2];
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int t = 0; t < 2; ++t) aqr[i][t] = *reinterpret_cast<const c1h8*>(wq + ((2 * i + t) * 32 + lr) * 16 + 8 * h);

  // this wave's conv row in a step and column pair (wave 2 r: pairs 0 .., wave 2 r + 1: pairs 31 ..)
  const int rr = wave >> 1, j = ((wave & 1) ? 31 : 0) + lr;
  // B: the lane's two pixels (conv columns 2 j + f) at window row 2 rr, k-step 0 (lane half h: taps 2 h, 2 h + 1)
  int bo[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) bo[f] = ((2 * rr) * FB_RW + 2 * (2 * j + f) + 2 * h) * 4;
  // the pooled column of the pair (wave 2 r's lane 31 is wave 2 r + 1's lane 0)
  const bool pok = lr < 31 && j < p.ep_Wo;
  const int aofs = lr * 16 + 8 * h;
  // window units of this thread: (row, 4 columns) u = tid + 512 k of FB_WR x 56
  int wgo[FB_NU], wlo[FB_NU], wrw[FB_NU];
#pragma unroll
  for (int k = 0; k < FB_NU; ++k) {
    const int u = tid + 512 * k, rw = u / 56, cg = u - rw * 56;
    const bool ok = u < FB_WR * 56 && 4 * cg < p.W;
    wgo[k] = ok ? (rw * p.W + 4 * cg) * 4 : (int)0x80000000;  // + the step's first row in the scalar offset
    wlo[k] = ok ? (rw * FB_RW + 4 * cg) * 4 : -1;
    wrw[k] = rw;
  }
  typedef float fbf4 __attribute__((ext_vector_type(4)));
  fbf4 xv[FB_NU][3];
  const int nsteps = (p.ep_Ho - 1 + 1) / 2 + 1;  // pooled row p completes at step ceil(p / 2)
  typedef unsigned short fbu8 __attribute__((ext_vector_type(8)));

  for (int img = blockIdx.x; img < p.N; img += gridDim.x) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(p.x + (long long)img * p.x_nstride), (short)0, p.C * p.x_ps * 4, 0x00020000);
    // the step's input rows [8 s, 8 s + 13) (rows past the image, channels >= C: past the records, 0)
    auto load_window = [&](int st) __attribute__((always_inline)) {
      const int so = 2 * (4 * st) * p.W * 4;
#pragma unroll
      for (int k = 0; k < FB_NU; ++k) {
        const int o = 8 * st + wrw[k] < p.H ? wgo[k] : (int)0x80000000;  // rows past the image: 0
#pragma unroll
        for (int c = 0; c < 3; ++c)
          xv[k][c] = __builtin_bit_cast(fbf4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  rs, c < p.C ? o : (int)0x80000000, so + c * p.x_ps * 4, 0));
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    auto store_window = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < FB_NU; ++k) {
        if (wlo[k] < 0) continue;
        c1h8 v0, v1;  // pixels 0, 1 and 2, 3 of the unit, channels 0 .. 3 (channel 3: 0)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            v0[4 * e + c] = (_Float16)xv[k][c][e];
            v1[4 * e + c] = (_Float16)xv[k][c][2 + e];
          }
          v0[4 * e + 3] = (_Float16)0.0f;
          v1[4 * e + 3] = (_Float16)0.0f;
        }
        *reinterpret_cast<c1h8*>(win + wlo[k]) = v0;
        *reinterpret_cast<c1h8*>(win + wlo[k] + 8) = v1;
      }
    };
    load_window(0);
    __syncthreads();  // (the previous image's last squeeze and the staging above are done)
    store_window();
    for (int st = 0; st < nsteps; ++st) {
      __syncthreads();  // window st is in LDS; the previous squeeze has read its ring rows
      if (st + 1 < nsteps) load_window(st + 1);
      const int cr = 4 * st + rr;  // this wave's conv row
      if (__builtin_amdgcn_readfirstlane(cr - p.Ho) < 0) {  // wave-uniform (the DPP below needs every lane)
        c1f16 acc[MF][2];
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
          for (int f = 0; f < 2; ++f)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][f][e] = 0.0f;
#pragma unroll
        for (int ks = 0; ks < FB_KS; ++ks) {
          // k-step ks: tap pair 2 ks + h = taps 4 ks + 2 h, + 1 (row (4 ks) / 8, column (4 ks) % 8 + 2 h)
          const int ko = ((4 * ks) / 8 * FB_RW + (4 * ks) % 8) * 4;
          c1h8 b[2];
#pragma unroll
          for (int f = 0; f < 2; ++f) b[f] = *reinterpret_cast<const c1h8*>(win + bo[f] + ko);
#pragma unroll
          for (int i = 0; i < MF; ++i) {
            const c1h8 a = *reinterpret_cast<const c1h8*>(Ws + (ks * MF + i) * 512 + aofs);
#pragma unroll
            for (int f = 0; f < 2; ++f) acc[i][f] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b[f], acc[i][f], 0, 0, 0);
          }
        }
        // the pair's pooled column: the bias (the patch kernel's f32 add); the two own columns' max in f32, then one
        // f16 rounding (rounding is monotonic: the rounded max is the max of the rounded values the patch kernel
        // pools) and the Relu on the bits; the third column (2 j + 2) as lane lr + 1's rounded first column by DPP
        // wave_shl:1, with every lane of the wave enabled (tests/test_isa_guard.py).  The DPP reads a 32-bit
        // v_cvt_pk_f16_f32 result: ROCm 7.2's compiler mis-lowers a DPP of either half of a packed f32 pair (it
        // shifts the low half and reuses it for the high one), the cause of round 5's
        // wrong-output band-walker variant.  A valid pooled column's three conv columns lie inside the plane
        // (2 ep_Wo <= Wo - 1), so no out-of-plane zero is needed
        const int slot = cr % FB_SLOTS;
        typedef float fbf2 __attribute__((ext_vector_type(2)));
        typedef _Float16 fbh2 __attribute__((ext_vector_type(2)));
        typedef short fbs2 __attribute__((ext_vector_type(2)));
        typedef unsigned short fbus2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
          for (int g = 0; g < 2; ++g) {
            unsigned o[4];
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
              const fbf2 b2 = {sbias[32 * i + 16 * g + 8 * h + e], sbias[32 * i + 16 * g + 8 * h + e + 1]};
              const fbf2 v0 = fbf2{acc[i][0][8 * g + e], acc[i][0][8 * g + e + 1]} + b2;
              const fbf2 v1 = fbf2{acc[i][1][8 * g + e], acc[i][1][8 * g + e + 1]} + b2;
              const fbf2 m01 = {fmaxf(v0[0], v1[0]), fmaxf(v0[1], v1[1])};
              const fbs2 r0 = __builtin_elementwise_max(__builtin_bit_cast(fbs2, __builtin_convertvector(v0, fbh2)), fbs2{0, 0});
              const fbs2 rm = __builtin_elementwise_max(__builtin_bit_cast(fbs2, __builtin_convertvector(m01, fbh2)), fbs2{0, 0});
              const int nb = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, r0), 0x130, 0xf, 0xf, true);
              // Relu outputs are >= +0: their f16 bits order like the values (unsigned max)
              o[e >> 1] = __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(fbus2, rm),
                                                                                 __builtin_bit_cast(fbus2, nb)));
            }
            if (pok) {
              typedef unsigned fbu4v __attribute__((ext_vector_type(4)));
              *reinterpret_cast<fbu4v*>(ring + (slot * FB_HC + j) * FB_CHS + 32 * i + 16 * g + 8 * h) =
                  fbu4v{o[0], o[1], o[2], o[3]};
            }
          }
      }
      __syncthreads();  // the step's ring rows are written; every K loop is done (the window is free)
      // the squeeze of pooled rows 2 st - 1 and 2 st: waves 0-3, 32 pooled pixels each
      if (wave < 4) {
        const int px = 32 * wave + lr, second = px >= p.ep_Wo ? 1 : 0;
        const int prow = 2 * st - 1 + second, pcol = px - second * p.ep_Wo;
        const bool qok = px < 2 * p.ep_Wo && prow >= 0 && prow < p.ep_Ho;
        const int pr = qok ? prow : 0, pc = qok ? pcol : 0;
        const _Float16* r0 = ring + (((2 * pr) % FB_SLOTS) * FB_HC + pc) * FB_CHS + 8 * h;
        const _Float16* r1 = ring + (((2 * pr + 1) % FB_SLOTS) * FB_HC + pc) * FB_CHS + 8 * h;
        const _Float16* r2 = ring + (((2 * pr + 2) % FB_SLOTS) * FB_HC + pc) * FB_CHS + 8 * h;
        c1f16 sacc;
#pragma unroll
        for (int e = 0; e < 16; ++e) sacc[e] = 0.0f;
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const int co = 32 * i + 16 * t;
            fbu8 m = __builtin_elementwise_max(*reinterpret_cast<const fbu8*>(r0 + co), *reinterpret_cast<const fbu8*>(r1 + co));
            m = __builtin_elementwise_max(m, *reinterpret_cast<const fbu8*>(r2 + co));
            sacc = __builtin_amdgcn_mfma_f32_32x32x16_f16(aqr[i][t], __builtin_bit_cast(c1h8, m), sacc, 0, 0, 0);
          }
        if (qok) {
          _Float16* yq = static_cast<_Float16*>(sq.y) + (long long)img * sq.y_nstride + (prow * p.ep_Wo + pcol) * sq.y_cs;
#pragma unroll
          for (int g = 0; g < 2; ++g) {
            const int ch = 16 * g + 8 * h;
            if (ch >= sq.M) continue;
            float av[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) av[e] = sacc[8 * g + e];
            *reinterpret_cast<c1h8*>(yq + ch) = ore_f16_epilogue8(av, qbias + ch, true);
          }
        }
      }
      if (st + 1 < nsteps) store_window();
    }
  }
}

}  // namespace

bool conv_pair_pool_f16_eligible(const ConvParams& p, const C1Squeeze* sq) {
  if (!((p.kh == 7 && p.kw == 7) || (p.kh == 3 && p.kw == 3))) return false;
  const int MF = (p.M + 31) / 32, kwp = (p.kw + 1) & ~1;
  if (MF < 1 || MF > 4 || p.M % 8 || p.C < 1 || p.C > 4 || p.sh != 2 || p.sw != 2 || p.pl % 2) return false;
  if (p.y_ps % 8 || p.y_nstride % 8 || (reinterpret_cast<uintptr_t>(p.y) & 15) || (reinterpret_cast<uintptr_t>(p.wp) & 15))
    return false;
  if (p.K != p.kh * kwp * 4 || p.Mp < MF * 32 - 31) return false;
  if (sq) {  // the fused squeeze: 7x7 only, whole 32-channel fragments in, <= 32 channels out
    auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    if (p.kh != 7 || (MF != 2 && MF != 3) || p.M != 32 * MF || sq->M < 8 || sq->M > 32 || sq->M % 8 || sq->y_cs % 8 ||
        sq->y_cs < sq->M || sq->y_nstride % 8 || !al16(sq->y) || !al16(sq->w) || !sq->bias)
      return false;
  }
  const C1Geom g = c1_geom(MF, p.kh, kwp, p.sh, p.sw, sq != nullptr);
  return g.lds_bytes <= 80 * 1024 && (long long)p.H * p.W < (1LL << 30) && p.ep_tr > 0 && p.ep_tc > 0;
}

bool conv_band_pool_f16_geometry(int C, int M, int kh, int kw, int sh, int sw, int pt, int pl, int W, int Wo, int ep_Ho,
                                 int ep_Wo, int ep_pt, int ep_pl, int sq_M) {
  return C >= 1 && C <= 3 && M == 96 && kh == 7 && kw == 7 && sh == 2 && sw == 2 && pt == 0 && pl == 0 && W <= 224 &&
         W % 4 == 0 && (Wo + 1) / 2 <= 63 && ep_Wo >= 1 && ep_Wo <= FB_HC - 1 && ep_Ho >= 1 &&
         ep_pt == 0 && ep_pl == 0 && 2 * (ep_Wo - 1) + 2 <= Wo - 1 && sq_M >= 8 && sq_M <= 32 && sq_M % 8 == 0;
}

bool conv_band_pool_f16_eligible(const ConvParams& p, const C1Squeeze* sq) {
  if (!sq || !p.relu || !conv_pair_pool_f16_eligible(p, sq)) return false;  // the patch kernel's layout rules
  return conv_band_pool_f16_geometry(p.C, p.M, p.kh, p.kw, p.sh, p.sw, p.pt, p.pl, p.W, p.Wo, p.ep_Ho, p.ep_Wo, p.ep_pt,
                                     p.ep_pl, sq->M) &&
         p.K == 7 * 8 * 4 && (long long)p.C * p.x_ps * 4 < (1LL << 31) && 2 * (p.ep_Ho - 1) + 2 < p.Ho;
}

void launch_conv_band_pool_f16(const ConvParams& p, const C1Squeeze& sq, hipStream_t s) {
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ncu = v;
  }
  static std::atomic<unsigned long long> raised{0};
  ore_raise_lds_once(raised, reinterpret_cast<const void*>(&conv_band_pool_f16_kernel), FB_LDS);
  const unsigned grid = (unsigned)std::max<long long>(1, std::min<long long>(p.N, ncu));  // one image per workgroup
  hipLaunchKernelGGL(conv_band_pool_f16_kernel, dim3(grid), dim3(512), FB_LDS, s, p, sq);
}

void launch_conv_pair_pool_f16(const ConvParams& p, const C1Squeeze* sq, hipStream_t s) {
  const int MF = (p.M + 31) / 32, kwp = (p.kw + 1) & ~1;
  const C1Geom g = c1_geom(MF, p.kh, kwp, p.sh, p.sw, sq != nullptr);
  long long tiles = (long long)p.N * p.ep_tr * p.ep_tc;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ncu = v;
  }
  // persistent: the workgroups resident at once (two per CU with the weights staged in LDS; registers
  // and LDS decide without), from the occupancy API
  int per_cu = 0;
  {
    const void* fn = sq ? (MF == 2 ? reinterpret_cast<const void*>(&conv_pair_pool_f16_kernel<2, 7, 7, 2, 1>)
                                   : reinterpret_cast<const void*>(&conv_pair_pool_f16_kernel<3, 7, 7, 2, 1>))
                        : reinterpret_cast<const void*>(&conv_pair_pool_f16_kernel<3, 7, 7, 2, 0>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, g.lds_bytes) != hipSuccess || per_cu < 1)
      per_cu = 2;
  }
  const unsigned grid = (unsigned)std::min<long long>(tiles, (long long)per_cu * ncu);
  const C1Squeeze none{};
  if (sq) {
    if (MF == 2) c1_dispatch<2, 1>(p, *sq, grid, g.lds_bytes, s);
    else c1_dispatch<3, 1>(p, *sq, grid, g.lds_bytes, s);
    return;
  }
  switch (MF) {
    case 1: c1_dispatch<1, 0>(p, none, grid, g.lds_bytes, s); break;
    case 2: c1_dispatch<2, 0>(p, none, grid, g.lds_bytes, s); break;
    case 3: c1_dispatch<3, 0>(p, none, grid, g.lds_bytes, s); break;
    default: c1_dispatch<4, 0>(p, none, grid, g.lds_bytes, s); break;
  }
}

}  // namespace ore
