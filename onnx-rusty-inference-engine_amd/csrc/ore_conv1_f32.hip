// First conv + Relu + its 3x3 / stride-2 MaxPool, f32 (the headline path's conv1 -> relu -> pool1;
// reference convolution_op.rs:94-517, relu_op.rs:31-33, max_pool_op.rs:157-360): pooled-epilogue
// variant 7 of launch_conv_epool, the f32 counterpart of conv_pair_pool_f16_kernel
// (ore_conv1_f16.hip).
//
// The row-walking kernel (ore_conv_pool.hip) streams each operand straight from L1 into the MFMA
// registers: ~58 VALU per k-step of tap state and addresses next to 24 MFMAs kept its main loop at
// ~75 % of the f32 MFMA peak.  Here the operand addressing is free:
//   * per tile (the 13 x 19 conv patch of 6 x 9 pooled outputs, the EP tile) the input window
//     [C][31][43] f32 sits in LDS, loaded one tile ahead by raw buffer loads (offsets outside the
//     image read 0: the conv's zero padding, no branch);
//   * v_mfma_f32_32x32x2_f32 in k = (c, r, s), the reference's order: lane half h takes k = 2j + h
//     of k-step j, whose window offset c*PLANE + r*43 + s is a compile-time immediate of one
//     ds_read_b32 -- the lane half's extra offset (+1, or a row / plane carry) is one of four
//     per-lane base registers, so the K loop is MFMAs, LDS reads and the A loads only;
//   * A (weights) from L2, packed by launch_pack_c1_f32 as [k/8][row][h][4]: one 16-B load per lane
//     covers four k-steps, a 1 KiB contiguous block per 32-row fragment;
//   * per 32-channel fragment: bias + Relu into an LDS conv tile [pixel][36], then each (pooled
//     output, 4 channels) takes its 3x3 max from -FLT_MAX and stores NCHW.
// Every conv output is the same k-ordered fma chain as the other pooled-conv kernels (the K tail
// k >= K multiplies a zero weight by a finite window value) and every pooled value the max of the
// same nine values: bit-identical to variants 1-6 (tests/test_model_gpu.py).
#include <float.h>
#include <hip/hip_runtime.h>

#include <algorithm>

#include "ore_kernels.h"

namespace ore {

namespace {

typedef float c3f4 __attribute__((ext_vector_type(4)));
typedef float c3f16 __attribute__((ext_vector_type(16)));

constexpr int C3_PR = EPOOL_TILE_PR, C3_PC = EPOOL_TILE_PC;  // pooled outputs per tile (6 x 9)
constexpr int C3_RC = 2 * C3_PR + 1, C3_CC = 2 * C3_PC + 1, C3_NPX = C3_RC * C3_CC;  // 13 x 19 conv patch
constexpr int C3_OOB = 0x40000000;  // a window byte offset past any image (C x_ps 4 < 2^30, eligibility)
constexpr int C3_TS = 36;  // conv tile pixel stride (floats): 144 B, 16-B aligned, an odd multiple of 16 B

template <int C, int KH, int KW, int S>
struct C3Geo {
  static constexpr int HR = (C3_RC - 1) * S + KH, HC = (C3_CC - 1) * S + KW, PLANE = HR * HC;
  static constexpr int K = C * KH * KW, KS = (K + 1) / 2, KQ = (K + 7) / 8;  // k-steps, 16-B A groups
  static constexpr int WIN = C * PLANE;                                     // window floats
  static constexpr int NQ = (WIN + 255) / 256;                              // window floats per thread
  static constexpr int LDS = (WIN + 3) / 4 * 16 + C3_NPX * C3_TS * 4;  // + the bias (launcher)
  // window offset of k (floats) and the kind of step from k to k + 1 (0: next column, 1: next row,
  // 2: next plane, 3: k + 1 >= K)
  static constexpr int koff(int k) { return (k / (KH * KW)) * PLANE + ((k / KW) % KH) * HC + k % KW; }
  static constexpr int kind(int k) {
    return k + 1 >= K ? 3 : (k % KW) < KW - 1 ? 0 : ((k / KW) % KH) < KH - 1 ? 1 : 2;
  }
};

template <int MF, int C, int KH, int KW, int S, int SQ, bool RELU, bool IN>  // IN: every tile's window inside the image
__global__ __launch_bounds__(256, 2) void conv_win_pool_f32_kernel(ConvParams p, const float* __restrict__ wc,
                                                                   C1SqueezeF32 sq) {
  using G = C3Geo<C, KH, KW, S>;
  extern __shared__ __attribute__((aligned(16))) float c3s[];
  float* win = c3s;                          // [C][HR][HC]
  float* ct = c3s + (G::WIN + 3) / 4 * 4;    // [C3_NPX][C3_TS]
  float* sbias = ct + C3_NPX * C3_TS;        // [MF * 32]
  // SQ: one fragment's pooled values [64 pixels][C3_TS] (the squeeze's B operand) and its bias
  float* pt = sbias + MF * 32;
  float* qbias = pt + (SQ ? 64 * C3_TS : 0);
  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Mp32 = MF * 32;
  for (int q = tid; q < Mp32; q += 256) sbias[q] = (p.bias && q < p.M) ? p.bias[q] : 0.0f;
  if constexpr (SQ) {
    for (int q = tid; q < 16; q += 256) qbias[q] = q < sq.M ? sq.bias[q] : 0.0f;
  }

  // SQ: the squeeze's A values of this lane for every fragment, once per workgroup (the weights do
  // not change across tiles; loaded at their use each would expose an L2 round trip)
  float aqv[SQ ? MF : 1][8];
  if constexpr (SQ) {
    const int lj = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int t = 0; t < 8; ++t) {  // channels past M (M < 96): a zero weight, not the next row's
        const int k = 32 * i + 4 * t + lk;
        aqv[i][t] = k < p.M ? sq.w[(lj < sq.M ? lj : 0) * p.M + k] : 0.0f;
      }
  }
  // the lane's two patch pixels: window base (bytes) per step kind (plain scalars, not an array: an
  // array indexed by the unrolled step's kind stayed in scratch), conv-tile offset
  int bk0[2], bk1[2], bk2[2], bk3[2], tpx[2];
  bool pin[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int px = (2 * wave + f) * 32 + lr;
    pin[f] = px < C3_NPX;
    const int pq = pin[f] ? px : 0;
    const int pr = pq / C3_CC, pc = pq - pr * C3_CC;
    const int base = pr * S * G::HC + pc * S;
    constexpr int d0 = 1, d1 = G::HC - (KW - 1), d2 = G::PLANE - (KH - 1) * G::HC - (KW - 1);
    bk0[f] = (base + (h ? d0 : 0)) * 4;
    bk1[f] = (base + (h ? d1 : 0)) * 4;
    bk2[f] = (base + (h ? d2 : 0)) * 4;
    bk3[f] = base * 4;
    tpx[f] = pq * C3_TS;
  }
  // this thread's window elements q = tid + 256 u, (plane c, row r, column cc).  IN: the byte offset
  // (c x_ps + r W + cc) 4 from the window's origin in the image (past the window: C3_OOB, which reads
  // 0); else the packed (c, r, cc) for the per-element bounds
  int wq[G::NQ];
#pragma unroll
  for (int u = 0; u < G::NQ; ++u) {
    const int q = tid + 256 * u;
    const int c = q / G::PLANE, rc = q - c * G::PLANE, r = rc / G::HC, cc = rc - r * G::HC;
    if constexpr (IN)
      wq[u] = q < G::WIN ? (c * p.x_ps + r * p.W + cc) * 4 : C3_OOB;
    else
      wq[u] = q < G::WIN ? (c << 24) | (r << 12) | cc : -1;
  }
  const int tpi = p.ep_tr * p.ep_tc, ntiles = p.N * tpi;
  float xv[G::NQ];
  auto load_window = [&](int tile) __attribute__((always_inline)) {
    const int tc = tile < ntiles ? tile : 0;
    const int img = tc / tpi, tt = tc - img * tpi;
    const int ph0 = (tt / p.ep_tc) * C3_PR, pw0 = (tt - (tt / p.ep_tc) * p.ep_tc) * C3_PC;
    const int ihb = (ph0 * 2 - p.ep_pt) * S - p.pt, iwb = (pw0 * 2 - p.ep_pl) * S - p.pl;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(p.x + (long long)img * p.x_nstride), (short)0, C * p.x_ps * 4, 0x00020000);
    if constexpr (IN) {
      // every window lies inside the image (conv1 of a 224 x 224 SqueezeNet input): the tile's origin
      // is the scalar offset of each load, no per-element VALU (f32 MFMAs hold the SIMD's VALU,
      // DESIGN.md section 3.7)
      const int so = (ihb * p.W + iwb) * 4;
#pragma unroll
      for (int u = 0; u < G::NQ; ++u)
        xv[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, wq[u], so, 0));
    } else {  // per-element bounds (offsets outside the image read 0: the conv's zero padding)
#pragma unroll
      for (int u = 0; u < G::NQ; ++u) {
        const int e = wq[u], c = e >> 24, ih = ihb + ((e >> 12) & 0xfff), iw = iwb + (e & 0xfff);
        const bool in = e >= 0 && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        xv[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                              rs, in ? (c * p.x_ps + ih * p.W + iw) * 4 : (int)0x80000000, 0, 0));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto store_window = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < G::NQ; ++u)
      if (tid + 256 * u < G::WIN) win[tid + 256 * u] = xv[u];
  };
  const char* winb = reinterpret_cast<const char*>(win);
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(wc), (short)0, G::KQ * Mp32 * 32, 0x00020000);
  const int aoff = (lr * 2 + h) * 16;  // + ((q * Mp32 + 32 i) * 2) * 16

  // the workgroups of XCD x (blockIdx % 8; the grid is a multiple of 8) walk a contiguous eighth of
  // the tiles, neighbouring patches at the same time: their shared window rows and columns meet in
  // one L2
  const bool grouped = (gridDim.x & 7) == 0;
  const int xg = grouped ? (int)(blockIdx.x & 7) : 0;
  const int nslot = grouped ? (int)(gridDim.x >> 3) : (int)gridDim.x;
  const int tlo = (int)((long long)ntiles * xg / (grouped ? 8 : 1));
  const int thi = grouped ? (int)((long long)ntiles * (xg + 1) / 8) : ntiles;
  const int tfirst = tlo + (grouped ? (int)(blockIdx.x >> 3) : (int)blockIdx.x);
  load_window(tfirst < thi ? tfirst : ntiles);
  store_window();
  for (int tile = tfirst; tile < thi; tile += nslot) {
    const int img = tile / tpi, tt = tile - img * tpi;
    const int ph0 = (tt / p.ep_tc) * C3_PR, pw0 = (tt - (tt / p.ep_tc) * p.ep_tc) * C3_PC;
    const int ohb = ph0 * 2 - p.ep_pt, owb = pw0 * 2 - p.ep_pl;
    __syncthreads();  // this tile's window is in LDS; the previous tile's pool readers are done
    load_window(tile + nslot < thi ? tile + nslot : ntiles);

    c3f16 acc[MF][2];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][f][e] = 0.0f;
    // A: 16-B groups of four k-steps, two groups ahead
    c3f4 a[2][MF];
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int i = 0; i < MF; ++i)
        if (g < G::KQ)
          a[g][i] = __builtin_bit_cast(c3f4, __builtin_amdgcn_raw_buffer_load_b128(wr, aoff, ((g * Mp32 + 32 * i) * 2) * 16, 0));
    // B one k-step ahead; A groups two ahead, refilled right after the MFMAs of a group's last
    // step; the scheduling barrier keeps each step's loads in it (unpinned, the scheduler sank the
    // A loads next to their first use, behind a vmcnt(0))
    auto bread = [&](int f, int j) __attribute__((always_inline)) {
      const int k0 = 2 * j, kd = G::kind(k0), ko = G::koff(k0) * 4;
      const int bb = kd == 0 ? bk0[f] : kd == 1 ? bk1[f] : kd == 2 ? bk2[f] : bk3[f];
      return *reinterpret_cast<const float*>(winb + bb + ko);
    };
    float bn[2] = {bread(0, 0), bread(1, 0)};
#pragma unroll
    for (int j = 0; j < G::KS; ++j) {
      const int q = j >> 2, ii = j & 3;
      const float b[2] = {bn[0], bn[1]};
      if (j + 1 < G::KS) {
        bn[0] = bread(0, j + 1);
        bn[1] = bread(1, j + 1);
      }
#pragma unroll
      for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int f = 0; f < 2; ++f)
          acc[i][f] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q & 1][i][ii], b[f], acc[i][f], 0, 0, 0);
      if (ii == 3 && q + 2 < G::KQ) {
#pragma unroll
        for (int i = 0; i < MF; ++i)
          a[q & 1][i] = __builtin_bit_cast(
              c3f4, __builtin_amdgcn_raw_buffer_load_b128(wr, aoff, (((q + 2) * Mp32 + 32 * i) * 2) * 16, 0));
      }
      __builtin_amdgcn_sched_barrier(0);
    }

    // SQ: the squeeze (<= 16 channels, v_mfma_f32_16x16x4_f32) over the tile's 54 pooled pixels, 16 per
    // wave: lane (lk, lj) accumulates rows 4 lk + 0..3 of pixel 16 wave + lj, k = channel ascending
    c3f4 sacc = {0.0f, 0.0f, 0.0f, 0.0f};
    const int sk = 16 * wave + (lane & 15), slk = lane >> 4;

    // SQ: the squeeze's 8 k-steps of fragment i: B = pooled (pixel sk, channel 4 t + lk) from pt, A = W[lj][32 i + 4 t + lk]
    const int lj = lane & 15;
    auto squeeze = [&](int i) __attribute__((always_inline)) {
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const float bq = pt[sk * C3_TS + 4 * t + slk];
        const float aq = lj < sq.M ? aqv[i][t] : 0.0f;
        sacc = __builtin_amdgcn_mfma_f32_16x16x4f32(aq, bq, sacc, 0, 0, 0);
      }
    };
    // per 32-channel fragment: conv tile (bias, Relu, 0 outside the conv plane), 3x3 max, NCHW stores.  SQ:
    // fragment i's squeeze k-steps run after fragment i + 1's conv-tile writes, before the barrier both
    // need (ct's pool readers of fragment i and pt's squeeze readers are done at the barriers around
    // them): two barriers per fragment instead of three (the squeeze's k order is unchanged)
#pragma unroll
    for (int i = 0; i < MF; ++i) {
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        if (!pin[f]) continue;
        const int px = (2 * wave + f) * 32 + lr, pr = px / C3_CC, pc = px - pr * C3_CC;
        const bool cok = (unsigned)(ohb + pr) < (unsigned)p.Ho && (unsigned)(owb + pc) < (unsigned)p.Wo;
        // Relu and the zero outside the conv plane in one v_med3_f32: median(v, 0, +inf) = max(v, 0),
        // median(v, 0, 0) = 0; the bias adds on packed f32 (f32 MFMAs hold the SIMD's VALU, so every
        // epilogue instruction is paid in full)
        const float top = cok ? __builtin_inff() : 0.0f;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int ch = 8 * g + 4 * h;  // accumulator rows 8 g + 4 h + 0..3
          const c3f4 sb = *reinterpret_cast<const c3f4*>(sbias + 32 * i + ch);
          c3f4 o = c3f4{acc[i][f][4 * g], acc[i][f][4 * g + 1], acc[i][f][4 * g + 2], acc[i][f][4 * g + 3]} + sb;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if constexpr (RELU)
              o[e] = __builtin_amdgcn_fmed3f(o[e], 0.0f, top);
            else
              o[e] = cok ? o[e] : 0.0f;
          }
          *reinterpret_cast<c3f4*>(ct + tpx[f] + ch) = o;
        }
      }
      if constexpr (SQ) {
        if (i > 0) squeeze(i - 1);
      }
      __syncthreads();
      if (i == 0) store_window();  // every wave is past its K loop: the window is free
      // (pooled output, 4 channels) per task, 432 tasks (a one-round 8-channel variant with all 18
      // reads in flight measured slower: 923 vs 891 us)
      if constexpr (SQ) {
        // every thread: two (pooled pixel, 4 channels) of the 64 x 32 block (pixels >= 54: pixel 0)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int t = tid + 256 * u, k = t >> 3, cg = t & 7, kc = k < C3_PR * C3_PC ? k : 0;
          const int aa = kc / C3_PC, bb = kc - aa * C3_PC;
          c3f4 mx = {-FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
#pragma unroll
          for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int s = 0; s < 3; ++s) {
              const c3f4 v = *reinterpret_cast<const c3f4*>(ct + ((2 * aa + r) * C3_CC + 2 * bb + s) * C3_TS + 4 * cg);
#pragma unroll
              for (int e = 0; e < 4; ++e) mx[e] = fmaxf(mx[e], v[e]);
            }
          *reinterpret_cast<c3f4*>(pt + k * C3_TS + 4 * cg) = mx;
        }
        __syncthreads();
        if (i + 1 == MF) squeeze(i);
      }
      for (int t = tid; !SQ && t < C3_PR * C3_PC * 8; t += 256) {
        const int cg = t / (C3_PR * C3_PC), pp = t - cg * (C3_PR * C3_PC);
        const int aa = pp / C3_PC, bb = pp - aa * C3_PC;
        c3f4 mx = {-FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int s = 0; s < 3; ++s) {
            const c3f4 v = *reinterpret_cast<const c3f4*>(ct + ((2 * aa + r) * C3_CC + 2 * bb + s) * C3_TS + 4 * cg);
#pragma unroll
            for (int e = 0; e < 4; ++e) mx[e] = fmaxf(mx[e], v[e]);
          }
        const int ph = ph0 + aa, pw = pw0 + bb;
        if (ph < p.ep_Ho && pw < p.ep_Wo) {
          float* yo = p.y + (long long)img * p.y_nstride + ph * p.ep_Wo + pw;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int m = 32 * i + 4 * cg + e;
            if (m < p.M) yo[(long long)m * p.y_ps] = mx[e];
          }
        }
      }
      if (!SQ && i + 1 < MF) __syncthreads();  // the conv tile is rewritten by the next fragment
    }
    if constexpr (SQ) {  // squeeze output: bias + Relu, NCHW (rows 4 lk + e of pixel sk)
      const int aa = sk / C3_PC, bb = sk - aa * C3_PC, ph = ph0 + aa, pw = pw0 + bb;
      if (sk < C3_PR * C3_PC && ph < p.ep_Ho && pw < p.ep_Wo) {
        float* yq = sq.y + (long long)img * sq.y_nstride + ph * p.ep_Wo + pw;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = 4 * slk + e;
          if (m < sq.M) yq[(long long)m * sq.y_ps] = fmaxf(sacc[e] + qbias[m], 0.0f);
        }
      }
    }
  }
}

// W [M][C][KH][KW] f32 -> [ceil(K / 8)][Mp32][2][4]: entry (q, row, h, t) = W[row][8 q + 2 t + h]
// (zero past M or K)
__global__ __launch_bounds__(256) void pack_c1_f32_kernel(const float* __restrict__ w, int M, int K, int Mp32,
                                                          float* __restrict__ out) {
  const long long total = (long long)((K + 7) / 8) * Mp32 * 8;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int t = (int)(i & 3), hh = (int)((i >> 2) & 1);
    const long long rq = i >> 3;
    const int row = (int)(rq % Mp32), q = (int)(rq / Mp32);
    const int k = 8 * q + 2 * t + hh;
    out[i] = (row < M && k < K) ? w[(long long)row * K + k] : 0.0f;
  }
}

template <int MF, int C, int SQ, bool RELU, bool IN>
static bool c3_launch(const ConvParams& p, const float* wc, const C1SqueezeF32& sq, hipStream_t s) {
  using G = C3Geo<C, 7, 7, 2>;
  const long long tiles = (long long)p.N * p.ep_tr * p.ep_tc;
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ncu = v;
  }
  // persistent: as many workgroups as fit on the chip at once (registers and LDS; 3 per CU for
  // conv1's 96 channels), each taking every grid-th tile
  const unsigned lds = G::LDS + MF * 32 * 4 + (SQ ? 64 * C3_TS * 4 + 16 * 4 : 0);
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, conv_win_pool_f32_kernel<MF, C, 7, 7, 2, SQ, RELU, IN>, 256, lds) !=
          hipSuccess || per_cu < 1)
    per_cu = 2;
  long long grid = std::min<long long>(tiles, (long long)per_cu * ncu);
  if (grid >= 8) grid &= ~7LL;  // a multiple of 8: XCD-grouped tile ranges
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL((conv_win_pool_f32_kernel<MF, C, 7, 7, 2, SQ, RELU, IN>), dim3((unsigned)grid), dim3(256), lds, s, p, wc, sq);
  return true;
}

template <int MF, int C, int SQ>
static bool c3_launch_r(const ConvParams& p, const float* wc, const C1SqueezeF32& sq, hipStream_t s) {
  // every tile's input window [ihb, ihb + HR) x [iwb, iwb + HC) inside the image?
  using G = C3Geo<C, 7, 7, 2>;
  const long long ih0 = -(long long)p.ep_pt * 2 - p.pt, iw0 = -(long long)p.ep_pl * 2 - p.pl;
  const long long ih1 = ((long long)(p.ep_tr - 1) * C3_PR * 2 - p.ep_pt) * 2 - p.pt + G::HR;
  const long long iw1 = ((long long)(p.ep_tc - 1) * C3_PC * 2 - p.ep_pl) * 2 - p.pl + G::HC;
  const bool in = ih0 >= 0 && iw0 >= 0 && ih1 <= p.H && iw1 <= p.W;
  if (p.relu)
    return in ? c3_launch<MF, C, SQ, true, true>(p, wc, sq, s) : c3_launch<MF, C, SQ, true, false>(p, wc, sq, s);
  return in ? c3_launch<MF, C, SQ, false, true>(p, wc, sq, s) : c3_launch<MF, C, SQ, false, false>(p, wc, sq, s);
}

// ---- variant 8: the band walker (conv1 + pool1 + the fused squeeze, no conv output computed twice) ----
//
// The window kernel above recomputes the 13 x 19 patch's halo: 256 MFMA columns per 54 pooled outputs,
// 16 % above the 220 conv outputs they need.  Here a workgroup (8 waves, one per CU: 153 KB of LDS)
// owns a band of pooled rows of one image and walks its conv rows row-major in steps of 256 column
// PAIRS (each conv row padded to an even number of columns, 55 pairs for conv1's 109): lane lr of wave
// w computes the pair's two columns as its two 32-pixel MFMA fragments, so
//   * the step's input rows [2 r_lo, 2 r_lo + 17) x 224 x 3 sit in LDS (float4 loads one step ahead,
//     stored after the step's MFMAs) and the K loop is the window kernel's (per-lane base registers,
//     compile-time k offsets, A from L2);
//   * pooling: after bias + Relu (one v_med3_i32 on the bits: negatives and out-of-plane columns -> +0),
//     the lane's pooled column j takes max(col 2j, 2j + 1, 2j + 2) -- the third from lane lr + 1 by DPP
//     wave_shl:1 -- into the pooled cells (row (cr + pt) / 2, and the one above for even rows) by
//     ds_max_u32 (Relu outputs are >= +0: their bits order like the values, and a max is exact in any
//     order); lane 0 hands its first column to the previous pair by ds_max (the previous lane sits in
//     another wave).  Invalid targets go to a per-lane dummy cell (ring slot 4);
//   * pooled rows live in a 4-slot LDS ring [96][5][56] (at most 4 are open while a step touches <= 6
//     conv rows); after each step the completed rows are squeezed (16x16x4 f32 MFMA, channel-ascending,
//     the window kernel's chain), stored NCHW and their cells cleared by the lane that read them.
// Conv outputs are the same k-ordered chains and pooled values the max of the same nine values as the
// window kernel: bit-identical to it (tests/test_model_gpu.py::test_conv1_band_bit_identical).
constexpr int CB_RW = 224;                 // LDS window row stride (floats): inputs up to 224 wide
constexpr int CB_WR = 17;                  // window rows: <= 6 conv rows per step (2 * 5 + 7)
constexpr int CB_PLANE = CB_WR * CB_RW;    // one channel of the window
constexpr int CB_C = 3, CB_NV = CB_C * CB_WR * (CB_RW / 4);  // float4s of the window (2856)
constexpr int CB_NU = (CB_NV + 511) / 512;                   // per thread (6)
constexpr int CB_RPW = 56;                 // ring row (pooled columns)
constexpr int CB_CS = 5 * CB_RPW;          // ring channel stride: 4 row slots + the dummy slot (= 8 mod 16:
                                           // the lane halves' channels 4 apart fall on other banks)
constexpr int CB_LDS = (3 * CB_PLANE + 96 * CB_CS + 96 + 16) * 4;
constexpr int CB_OOB = 0x40000000;

struct CBGeo {
  static constexpr int KH = 7, KW = 7, K = CB_C * 49, KS = (K + 1) / 2, KQ = (K + 7) / 8;
  static constexpr int koff(int k) { return (k / 49) * CB_PLANE + ((k / 7) % 7) * CB_RW + k % 7; }
  static constexpr int kind(int k) {
    return k + 1 >= K ? 3 : (k % KW) < KW - 1 ? 0 : ((k / KW) % KH) < KH - 1 ? 1 : 2;
  }
};

// median(b, 0, top) on ints (a min and a max: no inline asm here, whose VALU writes the hazard recognizer
// does not see ahead of the DPP reads that follow)
__device__ __forceinline__ int cb_med3(int b, int top) { return max(0, min(b, top)); }
__device__ __forceinline__ void cb_maxp(unsigned* a, unsigned v) {
  __hip_atomic_fetch_max(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__global__ __launch_bounds__(512, 1) void conv_band_pool_f32_kernel(ConvParams p, const float* __restrict__ wc,
                                                                    C1SqueezeF32 sq, int nb) {
  using G = CBGeo;
  constexpr int MF = 3;
  extern __shared__ __attribute__((aligned(16))) float cbs[];
  float* win = cbs;                        // [3][17][224]
  float* ring = cbs + 3 * CB_PLANE;        // [96][5][56]
  float* sbias = ring + 96 * CB_CS;        // [96]
  float* qbias = sbias + 96;               // [16]
  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int q = tid; q < 96; q += 512) sbias[q] = (p.bias && q < p.M) ? p.bias[q] : 0.0f;
  for (int q = tid; q < 16; q += 512) qbias[q] = q < sq.M ? sq.bias[q] : 0.0f;
  for (int q = tid; q < 96 * CB_CS; q += 512) ring[q] = 0.0f;
  float aqv[MF][8];  // the squeeze's A values of this lane (W[lj][32 i + 4 t + lk])
  {
    const int lj = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int t = 0; t < 8; ++t) {  // channels past M (M < 96): a zero weight, not the next row's
        const int k = 32 * i + 4 * t + lk;
        aqv[i][t] = lj < sq.M && k < p.M ? sq.w[lj * p.M + k] : 0.0f;
      }
  }
  // this thread's window float4s e = tid + 512 u: (channel c, row r, float4 j4); global byte offset from
  // the step's first input row (past the row's width: CB_OOB, which reads 0), LDS float index
  int wg[CB_NU], wl[CB_NU];
#pragma unroll
  for (int u = 0; u < CB_NU; ++u) {
    const int e = tid + 512 * u, c = e / (CB_WR * 56), rem = e - c * (CB_WR * 56), r = rem / 56, j4 = rem - r * 56;
    const bool ok = e < CB_NV && 4 * j4 < p.W;
    wg[u] = ok ? (c * p.x_ps + r * p.W + 4 * j4) * 4 : CB_OOB;
    wl[u] = e < CB_NV ? c * CB_PLANE + r * CB_RW + 4 * j4 : -1;
  }
  c3f4 xv[CB_NU];
  const char* winb = reinterpret_cast<const char*>(win);
  char* ringb = reinterpret_cast<char*>(ring);
  const int Mp32 = MF * 32;
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(wc), (short)0, G::KQ * Mp32 * 32, 0x00020000);
  const int aoff = (lr * 2 + h) * 16;
  const int HP = (p.Wo + p.ep_pl + 1) >> 1;  // column pairs per conv row
  const int units = p.N * nb;
  const int hb = h * 4 * CB_CS * 4;          // the lane half's first channel (rows 4 h + 0..3 of each 8)
  const int dummy = hb + (4 * CB_RPW + lr) * 4;

  for (int unit = blockIdx.x; unit < units; unit += gridDim.x) {
    const int img = unit / nb, band = unit - img * nb;
    const int pb0 = band * p.ep_Ho / nb, pb1 = (band + 1) * p.ep_Ho / nb;
    const int cr0 = max(0, 2 * pb0 - p.ep_pt), cr1 = min(p.Ho, 2 * pb1 - p.ep_pt + 1);
    const int npairs = (cr1 - cr0) * HP, nsteps = (npairs + 255) >> 8;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(p.x + (long long)img * p.x_nstride), (short)0, CB_C * p.x_ps * 4, 0x00020000);
    auto load_window = [&](int s) __attribute__((always_inline)) {
      const int so = 2 * (cr0 + (s << 8) / HP) * p.W * 4;
#pragma unroll
      for (int u = 0; u < CB_NU; ++u)
        xv[u] = __builtin_bit_cast(c3f4, __builtin_amdgcn_raw_buffer_load_b128(rs, wg[u], so, 0));
      __builtin_amdgcn_sched_barrier(0);
    };
    auto store_window = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < CB_NU - 1; ++u) *reinterpret_cast<c3f4*>(win + wl[u]) = xv[u];  // 512 u + tid < CB_NV
      if (wl[CB_NU - 1] >= 0) *reinterpret_cast<c3f4*>(win + wl[CB_NU - 1]) = xv[CB_NU - 1];
    };
    load_window(0);
    store_window();
    // A: 16-B groups of four k-steps (group u = i KQ + q of the step's 3 KQ: fragment i, k-steps 4 q ..),
    // two groups ahead, across fragments and steps
    constexpr int NG = MF * G::KQ;
    c3f4 a[2];
    auto load_a = [&](int u) __attribute__((always_inline)) {
      const int i = u / G::KQ, q = u - i * G::KQ;
      a[u & 1] = __builtin_bit_cast(c3f4, __builtin_amdgcn_raw_buffer_load_b128(wr, aoff, ((q * Mp32 + 32 * i) * 2) * 16, 0));
    };
    load_a(0);
    load_a(1);
    // the pooled rows [q_lo, q_hi) completed by a step: squeezed after it, between its two barriers
    int sq_lo = pb0;
    const int ng = (p.ep_Wo + 15) >> 4, lj = lane & 15, slk = lane >> 4;
    auto squeeze_rows = [&](int q_lo, int q_hi) __attribute__((always_inline)) {
      const int ntask = (q_hi - q_lo) * ng;
      for (int t = wave; t < ntask; t += 8) {
        const int pr = q_lo + t / ng, pc = 16 * (t - (t / ng) * ng) + lj;
        const bool pok = pc < p.ep_Wo;
        float* cell = ring + slk * CB_CS + (pok ? (pr & 3) * CB_RPW + pc : 4 * CB_RPW + 32 + lj);
        // all 24 B values in flight at once (one LDS round trip, not one per MFMA), then the chain
        float bq[MF][8];
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
          for (int tt = 0; tt < 8; ++tt) bq[i][tt] = cell[(32 * i + 4 * tt) * CB_CS];
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
          for (int tt = 0; tt < 8; ++tt) cell[(32 * i + 4 * tt) * CB_CS] = 0.0f;
        __builtin_amdgcn_sched_barrier(0);
        c3f4 sacc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
          for (int tt = 0; tt < 8; ++tt) sacc = __builtin_amdgcn_mfma_f32_16x16x4f32(aqv[i][tt], bq[i][tt], sacc, 0, 0, 0);
        if (pok) {
          float* yq = sq.y + (long long)img * sq.y_nstride + pr * p.ep_Wo + pc;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int m = 4 * slk + e;
            if (m < sq.M) yq[(long long)m * sq.y_ps] = fmaxf(sacc[e] + qbias[m], 0.0f);
          }
        }
      }
    };
    for (int s = 0; s < nsteps; ++s) {
      const int r_lo = cr0 + (s << 8) / HP;
      __syncthreads();  // window s is in LDS; the previous squeeze's reads and clears are done
      if (s + 1 < nsteps) load_window(s + 1);

      // the lane's pair: conv row cr, columns 2 j - pl + f
      const int P = (s << 8) + 32 * wave + lr;
      const bool pv = P < npairs;
      const int prow = P / HP, j = P - prow * HP, cr = cr0 + prow;
      int bk0[2], bk1[2], bk2[2], bk3[2], top[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const int col = 2 * j - p.ep_pl + f;
        const bool ok = pv && col >= 0 && col < p.Wo;
        const int base = ok ? 2 * (cr - r_lo) * CB_RW + 2 * col : 0;
        constexpr int d0 = 1, d1 = CB_RW - (G::KW - 1), d2 = CB_PLANE - (G::KH - 1) * CB_RW - (G::KW - 1);
        bk0[f] = (base + (h ? d0 : 0)) * 4;
        bk1[f] = (base + (h ? d1 : 0)) * 4;
        bk2[f] = (base + (h ? d2 : 0)) * 4;
        bk3[f] = base * 4;
        top[f] = ok ? 0x7fffffff : 0;
      }
      // pooled cells of the pair (row pa = (cr + pt) / 2 and, for even cr + pt, pa - 1; column j), and
      // of lane 0's first column (column j - 1)
      const int ap = cr + p.ep_pt, pa = ap >> 1;
      const bool rA = pv && pa >= pb0 && pa < pb1, rB = pv && !(ap & 1) && pa - 1 >= pb0 && pa - 1 < pb1;
      const int cA = ((pa & 3) * CB_RPW) * 4 + hb, cB = (((pa - 1) & 3) * CB_RPW) * 4 + hb;
      const bool jok = j < p.ep_Wo, bok = lr == 0 && j > 0 && j - 1 < p.ep_Wo;
      const int oA = rA && jok ? cA + j * 4 : dummy, oB = rB && jok ? cB + j * 4 : dummy;
      const int qA = rA && bok ? cA + (j - 1) * 4 : dummy, qB = rB && bok ? cB + (j - 1) * 4 : dummy;
      const bool nbok = lr < 31 && j + 1 < HP;  // the next column pair: this wave's lane lr + 1, same row
      // wave-uniform skips of LDS max operations that would all go to dummy cells: a wave on one odd row
      // has no second pooled row, and lane 0's first column rarely has nowhere to go
      const bool anyB = __builtin_amdgcn_ballot_w64(rB && jok) != 0;
      const bool anyQ = __builtin_amdgcn_ballot_w64(bok && (rA || rB)) != 0;
      auto bread = [&](int f, int jj) __attribute__((always_inline)) {
        const int k0 = 2 * jj, kd = G::kind(k0), ko = G::koff(k0) * 4;
        const int bb = kd == 0 ? bk0[f] : kd == 1 ? bk1[f] : kd == 2 ? bk2[f] : bk3[f];
        return *reinterpret_cast<const float*>(winb + bb + ko);
      };
      // per 32-channel fragment i: its K loop (both pixels), then its pooled contributions, whose LDS
      // max operations drain under the next fragment's MFMAs.  A wave whose pairs all lie past the band
      // (the band's last, partial step) skips both: its SIMD partner runs alone (its A ring already holds
      // the next step's first groups).  The condition is wave-uniform by construction (readfirstlane): the
      // DPP neighbour exchange below must run with every lane of the wave enabled -- a DPP read from a lane
      // that EXEC disables returns 0 (bound_ctrl) -- and tests/test_isa_guard.py checks the compiled kernel
      // for an EXEC-masked exchange
      if (__builtin_amdgcn_readfirstlane((s << 8) + 32 * wave - npairs) < 0) {
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        c3f16 acc[2];
#pragma unroll
        for (int f = 0; f < 2; ++f)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[f][e] = 0.0f;
        float bn[2] = {bread(0, 0), bread(1, 0)};
#pragma unroll
        for (int jj = 0; jj < G::KS; ++jj) {
          const int q = jj >> 2, ii = jj & 3, u = i * G::KQ + q;
          const float b[2] = {bn[0], bn[1]};
          if (jj + 1 < G::KS) {
            bn[0] = bread(0, jj + 1);
            bn[1] = bread(1, jj + 1);
          }
#pragma unroll
          for (int f = 0; f < 2; ++f)
            acc[f] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u & 1][ii], b[f], acc[f], 0, 0, 0);
          if (ii == 3 || jj + 1 == G::KS) {  // group u is done: its slot takes group u + 2
            if (u + 2 < NG) {
              load_a(u + 2);
            } else if (u + 1 == NG) {  // NG is odd: the next step's groups 0 and 1 after the last one
              load_a(0);
              load_a(1);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        // the fragment's cell pointers (channel 32 i + 4 h of each target): the 16 channel rows are
        // compile-time offsets of one pointer each
        unsigned* pA = reinterpret_cast<unsigned*>(ringb + 32 * i * CB_CS * 4 + oA);
        unsigned* pB = reinterpret_cast<unsigned*>(ringb + 32 * i * CB_CS * 4 + oB);
        unsigned first[16], mv[16];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const c3f4 sb = *reinterpret_cast<const c3f4*>(sbias + 32 * i + 8 * g + 4 * h);
          // the bias on packed f32 (two channels per v_pk_add_f32)
          const c3f4 o0 = c3f4{acc[0][4 * g], acc[0][4 * g + 1], acc[0][4 * g + 2], acc[0][4 * g + 3]} + sb;
          const c3f4 o1 = c3f4{acc[1][4 * g], acc[1][4 * g + 1], acc[1][4 * g + 2], acc[1][4 * g + 3]} + sb;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float f0 = o0[e], f1 = o1[e];
            // Relu and the out-of-plane zero on the bits: median(b, 0, top) (negative floats are
            // negative ints -> +0; top = 0 for a column outside the conv plane)
            const int b0 = cb_med3(__builtin_bit_cast(int, f0), top[0]);
            const int b1 = cb_med3(__builtin_bit_cast(int, f1), top[1]);
            int nbv = __builtin_amdgcn_update_dpp(0, b0, 0x130, 0xf, 0xf, true);  // wave_shl:1: lane l + 1's b0
            nbv = nbok ? nbv : 0;
            mv[4 * g + e] = (unsigned)max(max(b0, b1), nbv);
            first[4 * g + e] = (unsigned)b0;
          }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) cb_maxp(pA + ((r >> 2) * 8 + (r & 3)) * CB_CS, mv[r]);
        if (anyB) {
#pragma unroll
          for (int r = 0; r < 16; ++r) cb_maxp(pB + ((r >> 2) * 8 + (r & 3)) * CB_CS, mv[r]);
        }
        if (anyQ && lr == 0) {
          unsigned* qpA = reinterpret_cast<unsigned*>(ringb + 32 * i * CB_CS * 4 + qA);
          unsigned* qpB = reinterpret_cast<unsigned*>(ringb + 32 * i * CB_CS * 4 + qB);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            cb_maxp(qpA + ((r >> 2) * 8 + (r & 3)) * CB_CS, first[r]);
            cb_maxp(qpB + ((r >> 2) * 8 + (r & 3)) * CB_CS, first[r]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      }
      // the pooled rows completed by step s
      const int rdone = s + 1 == nsteps ? p.Ho : cr0 + ((s + 1) << 8) / HP;
      int sq_hi = sq_lo;
      while (sq_hi < pb1 && min(2 * sq_hi - p.ep_pt + 2, p.Ho - 1) < rdone) ++sq_hi;
      __syncthreads();  // every pooled contribution of step s is in the ring; every K loop is done
      squeeze_rows(sq_lo, sq_hi);
      sq_lo = sq_hi;
      if (s + 1 < nsteps) store_window();
    }
    __syncthreads();  // the unit's last squeeze is done before the next unit's window and ring writes
  }
}

}  // namespace

bool conv_band_pool_f32_geometry(int C, int M, int kh, int kw, int sh, int sw, int pt, int pl, int W, int Wo, int ep_Ho,
                                 int ep_Wo, int ep_pt, int ep_pl, int sq_M, bool relu) {
  const int HP = (Wo + ep_pl + 1) / 2;
  return sq_M >= 1 && sq_M <= 16 && relu && C == 3 && M > 64 && M <= 96 && kh == 7 && kw == 7 && sh == 2 && sw == 2 &&
         pt == 0 && pl == 0 && W <= CB_RW && W % 4 == 0 && HP >= 52 && ep_Wo <= CB_RPW && ep_Ho >= 1 && ep_pl <= 1 &&
         ep_pt <= 1;
}

bool conv_band_pool_f32_eligible(const ConvParams& p, const C1SqueezeF32* sq) {
  return sq && sq->w && sq->bias && sq->y && sq->y_ps >= p.ep_Ho * p.ep_Wo &&
         conv_band_pool_f32_geometry(p.C, p.M, p.kh, p.kw, p.sh, p.sw, p.pt, p.pl, p.W, p.Wo, p.ep_Ho, p.ep_Wo, p.ep_pt,
                                     p.ep_pl, sq->M, p.relu != 0) &&
         p.x_ps % 4 == 0 && p.x_nstride % 4 == 0 && p.x_ps >= p.H * p.W && (long long)3 * p.x_ps * 4 < (1LL << 30);
}

void launch_conv_band_pool_f32(const ConvParams& p, const float* wc, const C1SqueezeF32& sq, hipStream_t s) {
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ncu = v;
  }
  static std::atomic<unsigned long long> raised{0};
  ore_raise_lds_once(raised, reinterpret_cast<const void*>(&conv_band_pool_f32_kernel), CB_LDS);
  // bands of pooled rows per image: enough workgroups for one per CU (>= 4 pooled rows per band)
  int nb = 1;
  if ((long long)p.N < ncu) nb = std::max(1, std::min<int>((ncu + p.N - 1) / p.N, p.ep_Ho / 4));
  const long long units = (long long)p.N * nb;
  const long long grid = std::max<long long>(1, std::min<long long>(units, ncu));
  hipLaunchKernelGGL(conv_band_pool_f32_kernel, dim3((unsigned)grid), dim3(512), CB_LDS, s, p, wc, sq, nb);
}

size_t c1_f32_pack_bytes(int M, int K) { return size_t((K + 7) / 8) * size_t((M + 31) / 32 * 32) * 32; }

void launch_pack_c1_f32(const float* w, int M, int K, float* out, hipStream_t s) {
  const int Mp32 = (M + 31) / 32 * 32;
  const long long total = (long long)((K + 7) / 8) * Mp32 * 8;
  long long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pack_c1_f32_kernel, dim3((unsigned)blocks), dim3(256), 0, s, w, M, K, Mp32, out);
}

bool conv_win_pool_f32_eligible(const ConvParams& p, const C1SqueezeF32* sq) {
  const int MF = (p.M + 31) / 32;
  if (sq && (sq->M < 1 || sq->M > 16 || !sq->w || !sq->bias || !sq->y || sq->y_ps < p.ep_Ho * p.ep_Wo || MF != 3 ||
             p.C != 3))
    return false;
  return p.kh == 7 && p.kw == 7 && p.sh == 2 && p.sw == 2 && (p.C == 1 || p.C == 3 || p.C == 4) && MF >= 2 &&
         MF <= 4 && p.ep_tr > 0 && p.ep_tc > 0 && p.x_ps >= p.H * p.W && (long long)p.C * p.x_ps * 4 < (1LL << 30) &&
         p.H < 4096 && p.W < 4096;
}

void launch_conv_win_pool_f32(const ConvParams& p, const float* wc, const C1SqueezeF32* sq, hipStream_t s) {
  const int MF = (p.M + 31) / 32;
  const C1SqueezeF32 none{};
  if (sq) {  // the fused squeeze: conv1's geometry (96 channels, 3 inputs)
    c3_launch_r<3, 3, 1>(p, wc, *sq, s);
    return;
  }
  switch (MF * 8 + p.C) {
    case 2 * 8 + 1: c3_launch_r<2, 1, 0>(p, wc, none, s); break;
    case 2 * 8 + 3: c3_launch_r<2, 3, 0>(p, wc, none, s); break;
    case 2 * 8 + 4: c3_launch_r<2, 4, 0>(p, wc, none, s); break;
    case 3 * 8 + 1: c3_launch_r<3, 1, 0>(p, wc, none, s); break;
    case 3 * 8 + 3: c3_launch_r<3, 3, 0>(p, wc, none, s); break;
    case 3 * 8 + 4: c3_launch_r<3, 4, 0>(p, wc, none, s); break;
    case 4 * 8 + 1: c3_launch_r<4, 1, 0>(p, wc, none, s); break;
    case 4 * 8 + 3: c3_launch_r<4, 3, 0>(p, wc, none, s); break;
    default: c3_launch_r<4, 4, 0>(p, wc, none, s); break;
  }
}

}  // namespace ore
