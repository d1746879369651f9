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
      for (int t = 0; t < 8; ++t) aqv[i][t] = sq.w[(lj < sq.M ? lj : 0) * p.M + 32 * i + 4 * t + lk];
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

}  // namespace

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
