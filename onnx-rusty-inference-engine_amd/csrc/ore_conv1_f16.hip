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
