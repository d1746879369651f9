// 3x3 / stride-1 / pad-1 Conv (convolution_op.rs:94-517 at SqueezeNet's expand3x3 geometry) by
// Winograd F(2x2, 3x3) in f32 on the f32-input MFMA (v_mfma_f32_32x32x2_f32; 16x16x4 variants).
//
// Every 2x2 block ("tile") of output pixels of one channel m is
//   Y = A^T [ sum_c (G g_mc G^T) .* (B^T d_c B) ] A
// with d_c the 4x4 input window of channel c (rows 2ty-1 .. 2ty+2, columns 2tx-1 .. 2tx+2, zero
// outside the image: the reference's zero padding) and g_mc the 3x3 kernel.  The 16 element-wise
// products over c are 16 independent GEMMs ("positions" xi = 4 i + j):
//   M_xi[m][t] = sum_c U_xi[m][c] V_xi[c][t],   U = G g G^T (packed once), V = B^T d B (per k-step)
// so the MFMA work is 16 C M per tile against 36 C M for the direct conv (2.25x fewer MFMAs).  All
// arithmetic is f32; each position sums C products (the direct conv sums 9C), and the measured error
// against a float64 reference is at or below the direct f32 conv's (DESIGN.md section 3.3,
// tests/test_wino_gpu.py).  The results are NOT bit-identical to the direct kernels; they do not
// depend on the tile (every position is one c-ordered chain, the transforms a fixed add order).
//
// Operands go straight from global memory (L1/L2) into the MFMA registers, as in the streaming conv
// (no LDS, no barrier; each wave runs independently):
//   * B: in the 32x32x2 kernel lane l of MFMA xi supplies V_xi[c = 2 s + (l >> 5)][tile l & 31]: it
//     loads the 4x4 window of its tile for that channel (four 16-B row loads, 4-B aligned; rows
//     outside the image get an out-of-range buffer offset and read as 0; the image's first tile
//     column loads from column 0 and shifts right in registers, so no offset is negative), zeroes the
//     columns outside the image and transforms it in registers (32 adds): one window feeds 16 MFMAs.
//   * A: U is packed [c][xi / 4][m][xi % 4]: a lane's 16 positions of its channel row are four 16-B
//     loads, each wave-instruction two contiguous 512-B runs.
//   * the K loop is unrolled, with the weights DA and the windows DB k-steps ahead in register rings.
// Wave tile: 32 channels x 32 tiles (128 output pixels, 16 x 16 accumulators of 16 floats in the
// AccVGPRs); 4 waves per block share a tile group when M >= 128 (their windows hit the CU's L1).
// Epilogue: each lane holds all 16 positions of 16 (channel, tile) pairs -> A^T M A (24 adds) + bias
// (+ Relu) -> 4 pixels each, no cross-lane traffic.
// The 16x16x4 kernel (16 MF channels x 16 NT tiles per wave) is the same scheme at other tile shapes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <type_traits>

#include "ore_kernels.h"

namespace ore {

typedef float wg_floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16_t __attribute__((ext_vector_type(16)));
typedef int int4d_t __attribute__((ext_vector_type(4)));
typedef float wg_f2 __attribute__((ext_vector_type(2)));

// U[((c * 4 + xi / 4) * Mp + m) * 4 + xi % 4] = (G g_mc G^T)[xi / 4][xi % 4] (f64, rounded once): for a
// fixed (channel, position quad) the channels' 16-B quads are contiguous, so the A loads of a wave
// (one quad per lane, consecutive channels in consecutive lanes) are 512-B runs;
// G = [[1, 0, 0], [1/2, 1/2, 1/2], [1/2, -1/2, 1/2], [0, 0, 1]]; rows m >= M are zero
__global__ __launch_bounds__(256) void wino_pack_kernel(const float* __restrict__ w, float* __restrict__ u, int M,
                                                        int C, int Mp) {
  const long long total = (long long)C * Mp * 16;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long r = i >> 2;  // (c * 4 + q) * Mp + m
    const int m = (int)(r % Mp);
    const long long cq = r / Mp;
    const int c = (int)(cq >> 2);
    const int xi = (int)(((cq & 3) << 2) | (i & 3));
    float v = 0.0f;
    if (m < M) {
      const double G[4][3] = {{1.0, 0.0, 0.0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0.0, 0.0, 1.0}};
      const float* g = w + ((long long)m * C + c) * 9;
      const int a = xi >> 2, b = xi & 3;
      double s = 0.0;
      for (int p = 0; p < 3; ++p)
        for (int q = 0; q < 3; ++q) s += G[a][p] * (double)g[p * 3 + q] * G[b][q];
      v = (float)s;
    }
    u[i] = v;
  }
}

int wino_packed_mp(int M) { return (M + 63) / 64 * 64; }

void launch_pack_wino(const float* w, int M, int C, int Mp, float* u, hipStream_t s) {
  long long blocks = ((long long)C * Mp * 16 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(wino_pack_kernel, dim3((unsigned)blocks), dim3(256), 0, s, w, u, M, C, Mp);
}

// V = B^T d B of a 4x4 window (rows i, columns j), B^T = [[1,0,-1,0],[0,1,1,0],[0,-1,1,0],[0,1,0,-1]];
// v[4 i + j]
__device__ __forceinline__ void wg_input_transform(const float (&d)[4][4], float (&v)[16]) {
  float t[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    t[0][j] = d[0][j] - d[2][j];
    t[1][j] = d[1][j] + d[2][j];
    t[2][j] = d[2][j] - d[1][j];
    t[3][j] = d[1][j] - d[3][j];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[4 * i + 0] = t[i][0] - t[i][2];
    v[4 * i + 1] = t[i][1] + t[i][2];
    v[4 * i + 2] = t[i][2] - t[i][1];
    v[4 * i + 3] = t[i][1] - t[i][3];
  }
}

// Y = A^T M A, A^T = [[1,1,1,0],[0,1,-1,-1]]: y[2 i + j] (i = row, j = column of the 2x2 tile)
__device__ __forceinline__ void wg_output_transform(const float (&mx)[16], float (&y)[4]) {
  float t0[4], t1[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    t0[j] = mx[j] + mx[4 + j] + mx[8 + j];
    t1[j] = mx[4 + j] - mx[8 + j] - mx[12 + j];
  }
  y[0] = t0[0] + t0[1] + t0[2];
  y[1] = t0[1] - t0[2] - t0[3];
  y[2] = t1[0] + t1[1] + t1[2];
  y[3] = t1[1] - t1[2] - t1[3];
}

constexpr int WG_OOB = 0x7FFFFF00;  // a buffer offset past any resource (x_bytes < 2^31 - 2^21)

// the tile and window geometry of one lane: tile t (flattened over images), its window's row byte
// offsets for input channel `csub` (out-of-range rows -> WG_OOB), the column shift of the image's
// first tile column, the column-validity masks of the loaded elements and the output position
struct WgTile {
  int roff[4];
  int ybase;         // output element offset of the tile's top-left pixel (channel 0)
  unsigned cmask;    // bit k: loaded element k lies inside the row
  bool sh1, tok, c1ok, r1ok;
};

template <class P>
__device__ __forceinline__ WgTile wg_tile(const P& p, int t, int csub, int T, int TW, int TPI) {
  WgTile w;
  w.tok = t < T;
  if (!w.tok) t = T - 1;
  const int img = t / TPI;
  const int rem = t - img * TPI;
  const int ty = rem / TW, tx = rem - ty * TW;
  const int iy0 = 2 * ty - 1;
  w.sh1 = tx == 0;
  const int cs = w.sh1 ? 0 : 2 * tx - 1;  // first loaded column
  unsigned cm = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) cm |= (cs + k < p.W ? 1u : 0u) << k;
  w.cmask = cm;
  const int base = (img * (int)p.x_nstride + csub * p.x_ps + cs) * 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) w.roff[r] = (unsigned)(iy0 + r) < (unsigned)p.H ? base + (iy0 + r) * p.W * 4 : WG_OOB;
  w.ybase = img * (int)p.y_nstride + (2 * ty) * p.W + 2 * tx;
  w.c1ok = 2 * tx + 1 < p.W;
  w.r1ok = 2 * ty + 1 < p.H;
  return w;
}

// the 4 loaded rows of a window -> V = B^T d B (column masks, first-column shift)
__device__ __forceinline__ void wg_window(const wg_floatx4 (&rows)[4], const WgTile& w, float (&v)[16]) {
  float d[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int4 q = __builtin_bit_cast(int4, rows[r]);
    const int e0 = q.x, e1 = q.y & __builtin_amdgcn_sbfe((int)w.cmask, 1, 1);
    const int e2 = q.z & __builtin_amdgcn_sbfe((int)w.cmask, 2, 1);
    const int e3 = q.w & __builtin_amdgcn_sbfe((int)w.cmask, 3, 1);
    d[r][0] = w.sh1 ? 0.0f : __builtin_bit_cast(float, e0);
    d[r][1] = __builtin_bit_cast(float, w.sh1 ? e0 : e1);
    d[r][2] = __builtin_bit_cast(float, w.sh1 ? e1 : e2);
    d[r][3] = __builtin_bit_cast(float, w.sh1 ? e2 : e3);
  }
  wg_input_transform(d, v);
}

// the window's centre values d[1 + q / 2][1 + q % 2] (as wg_window builds d), i.e. the input at the
// tile's output pixel q: the B operand of a 1x1 conv on the same input
__device__ __forceinline__ void wg_centres(const wg_floatx4 (&rows)[4], const WgTile& w, float (&c)[4]) {
#pragma unroll
  for (int r = 1; r < 3; ++r) {
    const int4 q = __builtin_bit_cast(int4, rows[r]);
    const int e0 = q.x, e1 = q.y & __builtin_amdgcn_sbfe((int)w.cmask, 1, 1);
    const int e2 = q.z & __builtin_amdgcn_sbfe((int)w.cmask, 2, 1);
    c[2 * (r - 1) + 0] = __builtin_bit_cast(float, w.sh1 ? e0 : e1);
    c[2 * (r - 1) + 1] = __builtin_bit_cast(float, w.sh1 ? e1 : e2);
  }
}

// a tile's (up to) 4 output pixels o[2 i + j] of channel m -> yb (p.y's plane and image strides)
__device__ __forceinline__ void wg_store_px(const ConvParams& p, const WgTile& w, float* yb, int m, const float (&o)[4]) {
  if (!w.tok) return;
#ifdef ORE_EXP_WG_NOSTORE  // timing experiment only: stores skipped (kept live by a never-true test)
  if (o[0] != 1.2345e-30f) return;
#endif
  // a tile row's two pixels as one 8-B store (4-B aligned on odd planes; buffer stores take that),
  // so a wave-instruction writes whole lines: two 4-B stores per row wrote every line twice
  // (PMC WRITE_SIZE 1.5x the output, profiles/r02e_pmc_layers.txt)
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(yb, (short)0, 0x7FFFFFF0, 0x00020000);
  const int yo = (w.ybase + m * p.y_ps) * 4;
  typedef int wg_i2 __attribute__((ext_vector_type(2)));
  if (w.c1ok) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(wg_i2, (wg_f2){o[0], o[1]}), yr, yo, 0, 0);
    if (w.r1ok)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(wg_i2, (wg_f2){o[2], o[3]}), yr, yo + p.W * 4, 0, 0);
  } else {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, o[0]), yr, yo, 0, 0);
    if (w.r1ok) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, o[2]), yr, yo + p.W * 4, 0, 0);
  }
}

// the 16 position sums of one (channel m, tile) -> bias b (+ Relu) -> the tile's (up to) 4 pixels
__device__ __forceinline__ void wg_store(const ConvParams& p, const WgTile& w, int m, float b, const float (&mx)[16]) {
  float o[4];
  wg_output_transform(mx, o);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    o[q] += b;
    if (p.relu) o[q] = fmaxf(o[q], 0.0f);
  }
  wg_store_px(p, w, p.y, m, o);
}

// The K loop of both kernels over WG_LOAD_A(slot, step), WG_LOAD_B(slot, step), WG_MFMA(a slot, b slot)
#define WG_KLOOP(NKS_RT)                                                                               \
  if constexpr (NKS > 0) {                                                                             \
    /* step s: its MFMAs (operands A slot s % DA, windows transformed during step s - 1) interleaved  \
       with the refill loads and the transform of step s + 1's windows, so the loads' and VALU's     \
       issue cycles hide behind the MFMA pipe (one wave per SIMD: nothing else would cover them) */   \
    _Pragma("unroll") for (int s_ = 0; s_ < (DB < NKS ? DB : NKS); ++s_) { WG_LOAD_B(s_, s_) }          \
    _Pragma("unroll") for (int s_ = 0; s_ < (DA < NKS ? DA : NKS); ++s_) { WG_LOAD_A(s_, s_) }          \
    WG_WINDOWS(0, vc_)                                                                                 \
    _Pragma("unroll") for (int s_ = 0; s_ < NKS; ++s_) {                                              \
      __builtin_amdgcn_sched_barrier(0);                                                               \
      WG_MFMAS(s_ % DA, vc_);                                                                          \
      WG_EXTRA(s_ % DA, s_ % DB)                                                                       \
      if (s_ + 1 < NKS) { WG_WINDOWS((s_ + 1) % DB, vn_) }                                             \
      if (s_ + DA < NKS) { WG_LOAD_A(s_ % DA, s_ + DA) }                                               \
      if (s_ + DB < NKS) { WG_LOAD_B(s_ % DB, s_ + DB) }                                               \
      _Pragma("unroll") for (int i_ = 0; i_ < WG_NMFMA; ++i_) {                                        \
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0); /* one MFMA */                              \
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0); /* one VMEM read */                         \
        __builtin_amdgcn_sched_group_barrier(0x002, WG_VALU_PER_MFMA, 0);                              \
      }                                                                                                \
      __builtin_amdgcn_sched_barrier(0);                                                               \
      WG_COPYV(vc_, vn_)                                                                               \
    }                                                                                                  \
  } else { /* rolled: 2-deep rings (host: the k-step count is even) */                                \
    const int nks_ = (NKS_RT);                                                                         \
    _Pragma("unroll") for (int d_ = 0; d_ < 2; ++d_) { WG_LOAD_A(d_, d_) WG_LOAD_B(d_, d_) }           \
    for (int s0_ = 0; s0_ < nks_ - 2; s0_ += 2) {                                                      \
      _Pragma("unroll") for (int d_ = 0; d_ < 2; ++d_) {                                               \
        WG_MFMA(d_, d_);                                                                               \
        __builtin_amdgcn_sched_barrier(0);                                                             \
        WG_LOAD_A(d_, s0_ + 2 + d_)                                                                    \
        WG_LOAD_B(d_, s0_ + 2 + d_)                                                                    \
        __builtin_amdgcn_sched_barrier(0);                                                             \
      }                                                                                                \
    }                                                                                                  \
    _Pragma("unroll") for (int d_ = 0; d_ < 2; ++d_) { WG_MFMA(d_, d_); }                              \
  }

#define WG_EXTRA(SA, SB)  // per-kernel hook after a k-step's MFMAs (conv_wino16_kernel E1)

__device__ __forceinline__ int wg_block_wave(int* gw) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-aware bijective block remap, as in the other conv kernels
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, rr8 = nwg & 7;
  const int wgid = (xcd < rr8 ? xcd * (q8 + 1) : rr8 * (q8 + 1) + (xcd - rr8) * q8) + (bid >> 3);
  *gw = wgid * 4 + wave;
  return wave;
}

// 32x32x2 kernel: 32 channels x 32 tiles per wave.  NKS > 0: the K loop has exactly NKS k-steps (2
// channels each) and is unrolled completely, the A operands (weights, L2-resident) DA k-steps ahead
// and the B windows (activations, first touch from HBM / the Infinity Cache) DB k-steps ahead, and
// the compiler's wait-count pass waits for each step's own loads (in a rolled loop it drains every
// load at the loop head, exposing a full memory latency per ring turn); NKS = 0: any C, a rolled
// loop with 2-deep rings.
template <int DA, int DB, int NKS>
__global__ __launch_bounds__(256, 1) void conv_wino32_kernel(ConvParams p) {
  const int lane = threadIdx.x & 63;
  int gw;
  wg_block_wave(&gw);
  const int mt = gw % p.mtiles, tg = gw / p.mtiles;
  if (tg >= p.ntiles) return;  // wave-uniform; no barrier in this kernel
  const int m0 = mt * 32;
  const int lr = lane >> 5, lc = lane & 31;
  const int TW = (p.W + 1) >> 1, TPI = TW * ((p.H + 1) >> 1);
  const WgTile w = wg_tile(p, tg * 32 + lc, lr, p.N * TPI, TW, TPI);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.x), (short)0,
                                                                      (int)p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.wp), (short)0,
                                                                      p.C * p.Mp * 16 * 4, 0x00020000);
  const int aoff = (lr * 4 * p.Mp + m0 + lc) * 16;  // bytes: U[c = lr][quad 0][m0 + lc]; + Mp 16 per quad
  const int aq = p.Mp * 16, astep = 2 * 4 * p.Mp * 16, xstep = 8 * p.x_ps;
  // the wave's 32 biases by scalar loads before the K loop (a vector load in the epilogue would wait
  // on the stores issued before it; SGPRs keep the VGPRs for the ring)
  float bs[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) bs[j] = p.bias ? p.bias[min(m0 + j, p.M - 1)] : 0.0f;

  floatx16_t acc[16];
#pragma unroll
  for (int xi = 0; xi < 16; ++xi)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[xi][e] = 0.0f;
  wg_floatx4 ra[DA][4], rb[DB][4];
#ifndef ORE_EXP_WG_NOA
#define WG_LOAD_A(SLOT, S_)                                                                            \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) ra[SLOT][i] = __builtin_bit_cast(                    \
        wg_floatx4, __builtin_amdgcn_raw_buffer_load_b128(ur, aoff + aq * i, (S_) * astep, 0));
#else  // timing experiment only (tools/build_exp.sh): no A loads
#define WG_LOAD_A(SLOT, S_)                                                                            \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) ra[SLOT][i] = wg_floatx4{(float)(S_), 1.f, 2.f, 3.f};
#endif
#if !defined(ORE_EXP_WG_NOB) && !defined(ORE_EXP_WG_ALIGNB)
#define WG_LOAD_B(SLOT, S_)                                                                            \
    _Pragma("unroll") for (int r = 0; r < 4; ++r) rb[SLOT][r] = __builtin_bit_cast(                    \
        wg_floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, w.roff[r], (S_) * xstep, 0));
#elif defined(ORE_EXP_WG_ALIGNB)  // timing experiment only: the B rows loaded from 16-B aligned offsets
#define WG_LOAD_B(SLOT, S_)                                                                            \
    _Pragma("unroll") for (int r = 0; r < 4; ++r) rb[SLOT][r] = __builtin_bit_cast(                    \
        wg_floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, w.roff[r] & ~15, (S_) * xstep, 0));
#else  // timing experiment only: no B loads
#define WG_LOAD_B(SLOT, S_)                                                                            \
    _Pragma("unroll") for (int r = 0; r < 4; ++r) rb[SLOT][r] = wg_floatx4{(float)(S_), (float)lane, 2.f, 3.f};
#endif
#define WG_MFMA(SA, SB)                                                                                \
  {                                                                                                    \
    float v_[16];                                                                                      \
    wg_window(rb[SB], w, v_);                                                                          \
    WG_MFMAS(SA, v_)                                                                                   \
  }
#ifndef ORE_EXP_WG_NOMFMA
#define WG_MFMAS(SA, V)                                                                                \
    _Pragma("unroll") for (int xi = 0; xi < 16; ++xi)                                                  \
        acc[xi] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[SA][xi >> 2][xi & 3], V[xi], acc[xi], 0, 0, 0);
#else  // timing experiment only: operands consumed by one VALU op each instead of the MFMAs
#define WG_MFMAS(SA, V)                                                                                \
    _Pragma("unroll") for (int xi = 0; xi < 16; ++xi) acc[xi][xi] += ra[SA][xi >> 2][xi & 3] * V[xi];
#endif
#define WG_WINDOWS(SB, V) wg_window(rb[SB], w, V);
#define WG_COPYV(D_, S_) _Pragma("unroll") for (int i = 0; i < 16; ++i) D_[i] = S_[i];
#define WG_NMFMA 16
#define WG_VALU_PER_MFMA 4
  float vc_[16], vn_[16];
  WG_KLOOP(p.C >> 1)
#undef WG_MFMAS
#undef WG_WINDOWS
#undef WG_COPYV
#undef WG_NMFMA
#undef WG_VALU_PER_MFMA
#undef WG_LOAD_A
#undef WG_LOAD_B
#undef WG_MFMA
  // accumulator element e of a lane is row (e & 3) + 8 (e >> 2) + 4 lr (channel), column lc (tile)
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int m = m0 + (e & 3) + 8 * (e >> 2) + 4 * lr;
    if (m >= p.M) continue;
    float mx[16];
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) mx[xi] = acc[xi][e];
    const int r = (e & 3) + 8 * (e >> 2);
    wg_store(p, w, m, lr ? bs[r + 4] : bs[r], mx);
  }
}

// 16x16x4 kernel: MF 16-channel fragments x NT 16-tile groups per wave (row slot j of fragment f is
// channel m0 + MF j + f); k-steps of 4 channels; DA, DB, NKS as in conv_wino32_kernel.
// E1 (NKS > 0 only): the 1x1 conv (+ bias, Relu) on the same input with the same output channels
// (SqueezeNet's expand1x1 beside this expand3x3, ConvParams::e1_*) in the same K loop: its B operand at
// tile pixel q is the window's centre value (already in registers, wg_centres), its A the MF
// consecutive floats of its K-major packed weights (conv_stream_kernel's operand, one 4/8-B load per
// k-step), 4 MF NT more 16x16x4 MFMAs per k-step in k order -- the standalone 1x1 kernels' fma chain,
// so bit-identical -- and its pixels stored like the Winograd outputs.  The expand1x1 kernel and its
// HBM read of the input disappear (fire8: 75 us per B = 256 step).
template <int MF, int NT, int DA, int DB, int NKS, bool E1>
__global__ __launch_bounds__(256, 1) void conv_wino16_kernel(ConvParams p) {
  static_assert(!E1 || NKS > 0, "the fused 1x1 conv needs the unrolled K loop");
  const int lane = threadIdx.x & 63;
  int gw;
  wg_block_wave(&gw);
  const int mt = gw % p.mtiles, tg = gw / p.mtiles;
  if (tg >= p.ntiles) return;
  const int m0 = mt * (16 * MF);
  const int lk = lane >> 4, lj = lane & 15;
  const int TW = (p.W + 1) >> 1, TPI = TW * ((p.H + 1) >> 1);
  WgTile w[NT];
#pragma unroll
  for (int g = 0; g < NT; ++g) w[g] = wg_tile(p, (tg * NT + g) * 16 + lj, lk, p.N * TPI, TW, TPI);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.x), (short)0,
                                                                      (int)p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.wp), (short)0,
                                                                      p.C * p.Mp * 16 * 4, 0x00020000);
  const int aoff = (lk * 4 * p.Mp + m0 + MF * lj) * 16;  // U[c = lk][quad 0][MF consecutive channels]
  const int aq = p.Mp * 16, astep = 4 * 4 * p.Mp * 16, xstep = 16 * p.x_ps;
  float bias[MF][4];
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + MF * (4 * lk + e) + f;
      bias[f][e] = p.bias && m < p.M ? p.bias[m] : 0.0f;
    }

  wg_floatx4 acc[16][MF][NT];
#pragma unroll
  for (int xi = 0; xi < 16; ++xi)
#pragma unroll
    for (int f = 0; f < MF; ++f)
#pragma unroll
      for (int g = 0; g < NT; ++g) acc[xi][f][g] = wg_floatx4{0.f, 0.f, 0.f, 0.f};
  wg_floatx4 ra[DA][MF][4], rb[DB][NT][4];
  // E1: accumulators [pixel q][f][g], biases, A ring (W1[m0 + MF lj + f][4 s + lk] at k-step s)
  wg_floatx4 acc1[E1 ? 4 : 1][MF][NT];
  float bias1[E1 ? MF : 1][4];
  float ra1[E1 ? DA : 1][MF];
  if constexpr (E1) {
#pragma unroll
    for (int f = 0; f < MF; ++f)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + MF * (4 * lk + e) + f;
        bias1[f][e] = p.e1_bias && m < p.M ? p.e1_bias[m] : 0.0f;
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int g = 0; g < NT; ++g) acc1[q][f][g][e] = 0.0f;
      }
  }
  const __amdgpu_buffer_rsrc_t e1r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(E1 ? p.e1_wp : p.wp), (short)0, E1 ? p.C * p.e1_Mp * 4 : 0, 0x00020000);
  const int a1off = (lk * p.e1_Mp + m0 + MF * lj) * 4, a1step = 4 * p.e1_Mp * 4;
#define WG_LOAD_A(SLOT, S)                                                                             \
  {                                                                                                    \
    const int st_ = (S);                                                                               \
    _Pragma("unroll") for (int f = 0; f < MF; ++f)                                                     \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) ra[SLOT][f][i] = __builtin_bit_cast(                 \
        wg_floatx4, __builtin_amdgcn_raw_buffer_load_b128(ur, aoff + 16 * f + aq * i, st_ * astep, 0)); \
    if constexpr (E1) {                                                                                \
      static_assert(MF == 2, "E1: MF = 2 (one 8-B A load)");                                           \
      typedef float wg_f2_ __attribute__((ext_vector_type(2)));                                        \
      const wg_f2_ v_ = __builtin_bit_cast(wg_f2_, __builtin_amdgcn_raw_buffer_load_b64(e1r, a1off, st_ * a1step, 0)); \
      ra1[SLOT][0] = v_[0];                                                                            \
      ra1[SLOT][1] = v_[1];                                                                            \
    }                                                                                                  \
  }
#define WG_LOAD_B(SLOT, S)                                                                             \
  {                                                                                                    \
    const int st_ = (S);                                                                               \
    _Pragma("unroll") for (int g = 0; g < NT; ++g)                                                     \
    _Pragma("unroll") for (int r = 0; r < 4; ++r) rb[SLOT][g][r] = __builtin_bit_cast(                 \
        wg_floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, w[g].roff[r], st_ * xstep, 0));          \
  }
#define WG_MFMA(SA, SB)                                                                                \
  {                                                                                                    \
    float v_[NT][16];                                                                                  \
    WG_WINDOWS(SB, v_)                                                                                 \
    WG_MFMAS(SA, v_)                                                                                   \
  }
#define WG_MFMAS(SA, V)                                                                                \
    _Pragma("unroll") for (int xi = 0; xi < 16; ++xi)                                                  \
    _Pragma("unroll") for (int f = 0; f < MF; ++f)                                                     \
    _Pragma("unroll") for (int g = 0; g < NT; ++g)                                                     \
        acc[xi][f][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[SA][f][xi >> 2][xi & 3], V[g][xi], acc[xi][f][g], 0, 0, 0);
#define WG_WINDOWS(SB, V) _Pragma("unroll") for (int g = 0; g < NT; ++g) wg_window(rb[SB][g], w[g], V[g]);
#define WG_COPYV(D_, S_) \
    _Pragma("unroll") for (int g = 0; g < NT; ++g) _Pragma("unroll") for (int i = 0; i < 16; ++i) D_[g][i] = S_[g][i];
#define WG_NMFMA (16 * MF * NT)
#define WG_VALU_PER_MFMA 2
#undef WG_EXTRA
#define WG_EXTRA(SA, SB)                                                                               \
    if constexpr (E1) {                                                                                \
      _Pragma("unroll") for (int g = 0; g < NT; ++g) {                                                 \
        float c_[4];                                                                                   \
        wg_centres(rb[SB][g], w[g], c_);                                                               \
        _Pragma("unroll") for (int q = 0; q < 4; ++q)                                                  \
        _Pragma("unroll") for (int f = 0; f < MF; ++f)                                                 \
            acc1[q][f][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra1[SA][f], c_[q], acc1[q][f][g], 0, 0, 0); \
      }                                                                                                \
    }
  float vc_[NT][16], vn_[NT][16];
  WG_KLOOP(p.C >> 2)
#undef WG_EXTRA
#define WG_EXTRA(SA, SB)
#undef WG_MFMAS
#undef WG_WINDOWS
#undef WG_COPYV
#undef WG_NMFMA
#undef WG_VALU_PER_MFMA
#undef WG_LOAD_A
#undef WG_LOAD_B
#undef WG_MFMA
  // lane (lk, lj) of fragment f holds rows 4 lk + e = channel m0 + MF (4 lk + e) + f of tile lj
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + MF * (4 * lk + e) + f;
      if (m >= p.M) continue;
#pragma unroll
      for (int g = 0; g < NT; ++g) {
        float mx[16];
#pragma unroll
        for (int xi = 0; xi < 16; ++xi) mx[xi] = acc[xi][f][g][e];
        wg_store(p, w[g], m, bias[f][e], mx);
        if constexpr (E1) {  // the 1x1 conv's channel m at tile lj's 4 pixels: + bias (+ Relu)
          float o[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            o[q] = acc1[q][f][g][e] + bias1[f][e];
            if (p.e1_relu) o[q] = fmaxf(o[q], 0.0f);
          }
          wg_store_px(p, w[g], p.e1_y, m, o);
        }
      }
    }
}

// ---------------------------------------------------------------------------------------------------
// The fused fire module (ore_fire.hip's fire_kernel: expand1x1 + expand3x3 + Concat + the next
// squeeze in one launch) with the expand3x3 by Winograd F(2x2, 3x3): FireParams::wino.  A wave owns
// 16 2x2 tiles (64 output pixels, the direct kernel's column tile); MFMA column slot lj of MFMA q is
// pixel q (row-major in the tile) of tile lj, for e1, e3 and the squeeze alike.
//   * e1: 64-channel chunks, the direct kernel's 1x1 K loop and row-permuted weights (launch_fire_pack)
//     with the B operand of tile lj's 4 pixels loaded as two 8-B row pairs;
//   * e3: 32-channel chunks on conv_wino16_kernel's scheme (MF = 2); U packed [c][q][E3][4] with the
//     rows of each 32-channel chunk permuted (launch_fire_pack_wino) so that accumulator row 4 lk + e of
//     fragment f is channel c0 + 16 f + 4 e + lk: after the output transform, lane group lk holds
//     concat channel c0 + 4 t + lk at t = 4 f + e, the operand the squeeze takes at its k-step t;
//   * squeeze: unchanged (ascending concat channels, one fmaf chain).
// Bit-identical to the unfused graph with Winograd expand3x3 (every e3 output is the same c-ordered
// position sums and the same transform; the row permutation only moves outputs between lanes).
__global__ __launch_bounds__(256) void fire_wino_pack_kernel(const float* __restrict__ w, float* __restrict__ u,
                                                             int M, int C) {
  const long long total = (long long)C * M * 16;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long r = i >> 2;  // (c * 4 + q) * M + m'
    const int mq = (int)(r % M);
    const long long cq = r / M;
    const int c = (int)(cq >> 2);
    const int xi = (int)(((cq & 3) << 2) | (i & 3));
    const int c0 = mq & ~31, j = mq & 31, lj = j >> 1, f = j & 1;
    const int m = c0 + 16 * f + 4 * (lj & 3) + (lj >> 2);
    const double G[4][3] = {{1.0, 0.0, 0.0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0.0, 0.0, 1.0}};
    const float* g = w + ((long long)m * C + c) * 9;
    const int a = xi >> 2, b = xi & 3;
    double sacc = 0.0;
    for (int pp = 0; pp < 3; ++pp)
      for (int q = 0; q < 3; ++q) sacc += G[a][pp] * (double)g[pp * 3 + q] * G[b][q];
    u[i] = (float)sacc;
  }
}

void launch_fire_pack_wino(const float* w, int M, int C, float* u, hipStream_t s) {
  long long blocks = ((long long)C * M * 16 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(fire_wino_pack_kernel, dim3((unsigned)blocks), dim3(256), 0, s, w, u, M, C);
}

// MFS: 16-row fragments of the squeeze output; NKS: e3 k-steps (C / 4); DA / DB: e3 ring depths
template <int MFS, int NKS, int DA, int DB>
__global__ __launch_bounds__(256, 1) void fire_wino_kernel(FireParams p) {
  const int lane = threadIdx.x & 63;
  int gw;
  wg_block_wave(&gw);
  if (gw >= p.ntiles) return;  // wave-uniform; no barrier in this kernel
  const int lk = lane >> 4, lj = lane & 15;
  const int TW = (p.W + 1) >> 1, TPI = TW * ((p.H + 1) >> 1);
  const int T = p.N * TPI;
  const WgTile w = wg_tile(p, gw * 16 + lj, lk, T, TW, TPI);  // e3 window rows (channel lk of a k-step)
  // e1 / squeeze pixels of tile lj: element offsets of its top-left pixel (input plane / output)
  int t_ = gw * 16 + lj;
  if (t_ >= T) t_ = T - 1;
  const int img = t_ / TPI, rem = t_ - img * TPI, ty = rem / TW, tx = rem - ty * TW;
  const int xpix = img * (int)p.x_nstride + (2 * ty) * p.W + 2 * tx;  // channel 0
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.x), (short)0,
                                                                      (int)p.x_bytes, 0x00020000);
  const int C = p.C;
  const __amdgpu_buffer_rsrc_t w1r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.w1), (short)0, ((C + 31) & ~31) * p.E1 * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.w3), (short)0,
                                                                      C * p.E3 * 16 * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t wsr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.ws), (short)0, (((p.E1 + p.E3) + 31) & ~31) * p.Msp * 4, 0x00020000);

  wg_floatx4 accs[MFS][4];  // squeeze: row 4 lk + e of fragment fs, pixel q of tile lj
#pragma unroll
  for (int fs = 0; fs < MFS; ++fs)
#pragma unroll
    for (int q = 0; q < 4; ++q) accs[fs][q] = wg_floatx4{0.f, 0.f, 0.f, 0.f};

  // squeeze k-steps over T_ chunk values val[t][q] = concat channel cat0 + 4 t + lk at pixel q
  auto squeeze = [&](auto nt_tag, const float (*val)[4], int cat0) __attribute__((always_inline)) {
    constexpr int NTT = decltype(nt_tag)::value;
    const int saoff = ((cat0 + lk) * p.Msp + MFS * lj) * 4;
#pragma unroll
    for (int t = 0; t < NTT; ++t) {
      float as[MFS];
      const int so = saoff + t * 16 * p.Msp;
      if constexpr (MFS == 4) {
        const wg_floatx4 v = __builtin_bit_cast(wg_floatx4, __builtin_amdgcn_raw_buffer_load_b128(wsr, so, 0, 0));
        as[0] = v[0]; as[1] = v[1]; as[2] = v[2]; as[3] = v[3];
      } else if constexpr (MFS == 3) {
        typedef float f3 __attribute__((ext_vector_type(3)));
        const f3 v = __builtin_bit_cast(f3, __builtin_amdgcn_raw_buffer_load_b96(wsr, so, 0, 0));
        as[0] = v[0]; as[1] = v[1]; as[2] = v[2];
      } else if constexpr (MFS == 2) {
        typedef float f2 __attribute__((ext_vector_type(2)));
        const f2 v = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(wsr, so, 0, 0));
        as[0] = v[0]; as[1] = v[1];
      } else {
        as[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wsr, so, 0, 0));
      }
#pragma unroll
      for (int fs = 0; fs < MFS; ++fs)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          accs[fs][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(as[fs], val[t][q], accs[fs][q], 0, 0, 0);
    }
  };

  // ---- e1: 64-channel chunks (the direct fire kernel's K loop over C, 4 channels per k-step)
  typedef float f2v __attribute__((ext_vector_type(2)));
  for (int c0 = 0; c0 < p.E1; c0 += 64) {
    const int aoff = (lk * p.E1 + c0 + 4 * lj) * 4, astep = 16 * p.E1;
    const int xo = (xpix + lk * p.x_ps) * 4, xstep = 16 * p.x_ps, xrow = p.W * 4;
    wg_floatx4 acc[4][4];
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[f][q] = wg_floatx4{0.f, 0.f, 0.f, 0.f};
    constexpr int D1 = 4;
    wg_floatx4 ra[D1];
    f2v rb0[D1], rb1[D1];
#define FW_LOAD1(SLOT, S)                                                                              \
    {                                                                                                  \
      const int s_ = (S);                                                                              \
      ra[SLOT] = __builtin_bit_cast(wg_floatx4, __builtin_amdgcn_raw_buffer_load_b128(w1r, aoff, s_ * astep, 0)); \
      rb0[SLOT] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(xr, xo, s_ * xstep, 0));  \
      rb1[SLOT] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(xr, xo + xrow, s_ * xstep, 0)); \
    }
#define FW_MFMA1(SLOT)                                                                                 \
    {                                                                                                  \
      const float bq_[4] = {rb0[SLOT][0], rb0[SLOT][1], rb1[SLOT][0], rb1[SLOT][1]};                   \
      __builtin_amdgcn_s_setprio(1);                                                                   \
      _Pragma("unroll") for (int f = 0; f < 4; ++f)                                                    \
      _Pragma("unroll") for (int q = 0; q < 4; ++q)                                                    \
        acc[f][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[SLOT][f], bq_[q], acc[f][q], 0, 0, 0);     \
      __builtin_amdgcn_s_setprio(0);                                                                   \
    }
    constexpr int nks1 = NKS;  // C / 4 k-steps (host: NKS % D1 == 0)
#pragma unroll
    for (int d = 0; d < D1; ++d) FW_LOAD1(d, d);
#pragma unroll
    for (int s0 = 0; s0 < nks1 - D1; s0 += D1) {
#pragma unroll
      for (int d = 0; d < D1; ++d) {
        FW_MFMA1(d);
        __builtin_amdgcn_sched_barrier(0);
        FW_LOAD1(d, s0 + D1 + d);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int d = 0; d < D1; ++d) FW_MFMA1(d);
#undef FW_LOAD1
#undef FW_MFMA1
    // bias + Relu: accumulator row 4 lk + e of fragment f is channel c0 + 16 f + 4 e + lk (t = 4 f + e)
    float val[16][4];
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float b = p.b1[c0 + 16 * f + 4 * e + lk];
#pragma unroll
        for (int q = 0; q < 4; ++q) val[4 * f + e][q] = fmaxf(acc[f][q][e] + b, 0.0f);
      }
    squeeze(std::integral_constant<int, 16>{}, val, c0);
  }

  // ---- e3: 32-channel Winograd chunks
  for (int c0 = 0; c0 < p.E3; c0 += 32) {
    const int aoff = (lk * 4 * p.E3 + c0 + 2 * lj) * 16;  // U[c = lk][quad 0][c0 + 2 lj]
    const int aq = p.E3 * 16, astep = 4 * 4 * p.E3 * 16, xstep = 16 * p.x_ps;
    wg_floatx4 acc[16][2][1];
#pragma unroll
    for (int xi = 0; xi < 16; ++xi)
#pragma unroll
      for (int f = 0; f < 2; ++f) acc[xi][f][0] = wg_floatx4{0.f, 0.f, 0.f, 0.f};
    wg_floatx4 ra[DA][2][4], rb[DB][1][4];
    constexpr int MF = 2, NT = 1;
    const WgTile* wp_ = &w;
#define WG_LOAD_A(SLOT, S)                                                                             \
  {                                                                                                    \
    const int st_ = (S);                                                                               \
    _Pragma("unroll") for (int f = 0; f < MF; ++f)                                                     \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) ra[SLOT][f][i] = __builtin_bit_cast(                 \
        wg_floatx4, __builtin_amdgcn_raw_buffer_load_b128(ur, aoff + 16 * f + aq * i, st_ * astep, 0)); \
  }
#define WG_LOAD_B(SLOT, S)                                                                             \
  {                                                                                                    \
    const int st_ = (S);                                                                               \
    _Pragma("unroll") for (int r = 0; r < 4; ++r) rb[SLOT][0][r] = __builtin_bit_cast(                 \
        wg_floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, wp_->roff[r], st_ * xstep, 0));          \
  }
#define WG_MFMA(SA, SB)                                                                                \
  {                                                                                                    \
    float v_[NT][16];                                                                                  \
    WG_WINDOWS(SB, v_)                                                                                 \
    WG_MFMAS(SA, v_)                                                                                   \
  }
#define WG_MFMAS(SA, V)                                                                                \
    _Pragma("unroll") for (int xi = 0; xi < 16; ++xi)                                                  \
    _Pragma("unroll") for (int f = 0; f < MF; ++f)                                                     \
        acc[xi][f][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[SA][f][xi >> 2][xi & 3], V[0][xi], acc[xi][f][0], 0, 0, 0);
#define WG_WINDOWS(SB, V) wg_window(rb[SB][0], *wp_, V[0]);
#define WG_COPYV(D_, S_) _Pragma("unroll") for (int i = 0; i < 16; ++i) D_[0][i] = S_[0][i];
#define WG_NMFMA (16 * MF * NT)
#define WG_VALU_PER_MFMA 2
    float vc_[NT][16], vn_[NT][16];
    WG_KLOOP(NKS)
#undef WG_MFMAS
#undef WG_WINDOWS
#undef WG_COPYV
#undef WG_NMFMA
#undef WG_VALU_PER_MFMA
#undef WG_LOAD_A
#undef WG_LOAD_B
#undef WG_MFMA
    // output transform + bias + Relu: row 4 lk + e of fragment f = channel c0 + 16 f + 4 e + lk (t = 4 f + e)
    float val[8][4];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float mx[16], o[4];
#pragma unroll
        for (int xi = 0; xi < 16; ++xi) mx[xi] = acc[xi][f][0][e];
        wg_output_transform(mx, o);
        const float b = p.b3[c0 + 16 * f + 4 * e + lk];
#pragma unroll
        for (int q = 0; q < 4; ++q) val[4 * f + e][q] = fmaxf(o[q] + b, 0.0f);
      }
    squeeze(std::integral_constant<int, 8>{}, val, p.E1 + c0);
  }

  // S' = Relu(squeeze + bs): squeeze channel MFS (4 lk + e) + fs at pixel q of tile lj
  if (!w.tok) return;
  float* __restrict__ y = p.y;
  const int ybase = img * (int)p.y_nstride + (2 * ty) * p.W + 2 * tx;
#pragma unroll
  for (int fs = 0; fs < MFS; ++fs)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = MFS * (4 * lk + e) + fs;
      if (m >= p.Ms) continue;
      const float b = p.bs[m];
      float o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = fmaxf(accs[fs][q][e] + b, 0.0f);
      float* yp = y + (unsigned)(ybase + m * p.y_ps);
      yp[0] = o[0];
      if (w.c1ok) yp[1] = o[1];
      if (w.r1ok) {
        yp[p.W] = o[2];
        if (w.c1ok) yp[p.W + 1] = o[3];
      }
    }
}

bool fire_wino_eligible(const FireParams& p) {
  const uintptr_t xa = reinterpret_cast<uintptr_t>(p.x);
  return p.E1 % 64 == 0 && p.E3 % 32 == 0 && p.E1 > 0 && p.E3 > 0 && p.Ms >= 1 && p.Ms <= 64 && p.C % 16 == 0 &&
         p.C <= 64 && p.C > 0 && (xa & 3) == 0 && p.x_bytes > 0 && p.x_bytes < (1LL << 31) - (1LL << 21) &&
         (long long)p.C * p.E3 * 64 < (1LL << 31) && p.Msp % 4 == 0 &&
         (long long)p.N * ((p.H + 1) / 2) * ((p.W + 1) / 2) < (1LL << 30);
}

template <int MFS, int NKS>
static void launch_fw(const FireParams& p0, hipStream_t s) {
  FireParams p = p0;
  const long long T = (long long)p.N * ((p.H + 1) / 2) * ((p.W + 1) / 2);
  p.ntiles = (int)((T + 15) / 16);
  hipLaunchKernelGGL((fire_wino_kernel<MFS, NKS, 2, 4>), dim3((unsigned)((p.ntiles + 3) / 4)), dim3(256), 0, s, p);
}

template <int MFS>
static void launch_fw_c(const FireParams& p, hipStream_t s) {
  switch (p.C / 16) {
    case 1: launch_fw<MFS, 4>(p, s); break;
    case 2: launch_fw<MFS, 8>(p, s); break;
    case 3: launch_fw<MFS, 12>(p, s); break;
    default: launch_fw<MFS, 16>(p, s); break;
  }
}

void launch_fire_wino(const FireParams& p, hipStream_t s) {
  switch ((p.Ms + 15) / 16) {
    case 1: launch_fw_c<1>(p, s); break;
    case 2: launch_fw_c<2>(p, s); break;
    case 3: launch_fw_c<3>(p, s); break;
    default: launch_fw_c<4>(p, s); break;
  }
}

// ---------------------------------------------------------------------------------------------------
// LDS-staged Winograd kernel (tile 4).  The register-streaming kernels above move 16 window floats and
// 16 U floats per (channel, tile) and lane through the vector-memory path, which caps them near 15 B
// per clock per CU of VGPR-bound loads (profiles/r02b_pmc_wino32_vs_gemm_f8e3.txt: TD 79 % busy at
// 41 % MFMA).  Here
//   * U of the block's 32 output channels (C x 16 x 32 floats, 32-128 KB) is loaded into LDS once
//     and stays there: blocks are persistent over a range of tile groups of one 32-channel tile;
//   * each wave stages, per k-step, the input rows its tile group reads (2 channels x (2R + 2) rows,
//     zero-padded by one column each side) into its own LDS ring by LDS-DMA: each input element
//     crosses the memory path once per wave instead of ~4 times, and rows / columns outside the
//     image arrive as zeros (out-of-range buffer offsets), so the windows need no masks;
//   * windows (16 x ds_read_b32) and U (4 x ds_read_b128) come from LDS, one k-step ahead of the MFMAs.
// A tile group is R whole tile rows of one image (R = floor(32 / TW)); lane l & 31 is tile
// (l & 31) / TW, (l & 31) % TW of the group (lanes past the group idle), l >> 5 the channel.
struct WlGeom {
  int TW, TH, R, Wp;  // tiles per row / column, tile rows per group, padded staging row width
  int gpi, G;         // groups per image, groups in the batch
  int bpm;            // blocks in the grid (split evenly over the 32-channel tiles)
  int ubytes, ringb;  // LDS bytes of U and of one wave's ring
};

__device__ __forceinline__ void wl_dma(int4d_t rsrc, unsigned lds_addr, int voffset, int soffset) {
  int m0save;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dword %2, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(m0save)
      : "s"(__builtin_amdgcn_readfirstlane(lds_addr)), "v"(voffset), "s"(rsrc), "s"(soffset)
      : "memory");
}

#define WL_VMCNT(n) (((n) & 15) | (((n) >> 4) << 14) | (7 << 4) | (15 << 8))

// NKS: k-steps (C / 2), NI: 64-float DMA pieces per staged channel, DR: ring slots (k-steps ahead,
// at most 4: the counted waits below assume at most 2 later steps in flight)
template <int NKS, int NI, int DR>
__global__ __launch_bounds__(256, 1) void conv_winol_kernel(ConvParams p, WlGeom g) {
  extern __shared__ __attribute__((aligned(16))) float wl_lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // block b -> (32-channel tile mt, its bi-th of bpm(mt) group ranges): the m-tiles split the grid
  // evenly (g.bpm = blocks in the grid)
  const int b = blockIdx.x;
  const int mt = (int)(((long long)b * p.mtiles) / g.bpm);
  const int b0 = (int)(((long long)mt * g.bpm + p.mtiles - 1) / p.mtiles);
  const int b1 = (int)(((long long)(mt + 1) * g.bpm + p.mtiles - 1) / p.mtiles);
  const int bi = b - b0, nbm = b1 - b0;
  const int m0 = mt * 32;
  constexpr int C = 2 * NKS;
  // ---- U of channels m0 .. m0 + 31 into LDS: [c][q][32][4] floats (from the global [c][q][Mp][4])
  {
    const wg_floatx4* __restrict__ ug = reinterpret_cast<const wg_floatx4*>(p.wp);
    wg_floatx4* ul = reinterpret_cast<wg_floatx4*>(wl_lds);
    for (int i = tid; i < C * 4 * 32; i += 256) {
      const int m = i & 31, cq = i >> 5;
      ul[i] = ug[(long long)cq * p.Mp + m0 + m];
    }
  }
  __syncthreads();  // the only barrier: from here each wave runs on its own
  const int g0 = (int)((long long)bi * g.G / nbm), g1 = (int)((long long)(bi + 1) * g.G / nbm);
  const int ringf = (g.ubytes + wave * g.ringb) / 4;  // this wave's ring (float index)
  const unsigned ring = (unsigned)(size_t)(__attribute__((address_space(3))) float*)wl_lds + ringf * 4;  // LDS address
  constexpr int CHUNK = NI * 64 + 1;  // floats per staged channel (+1: the two channels on other banks)
  const int lr = lane >> 5, lc = lane & 31;
  const unsigned long long xb = reinterpret_cast<unsigned long long>(p.x);
  const int4d_t xdesc = {(int)(unsigned)xb, (int)((xb >> 32) & 0xffff), (int)p.x_bytes, 0x00020000};
  const int cstep = p.x_ps * 4;  // bytes between input channel planes
  const wg_floatx4* ul = reinterpret_cast<const wg_floatx4*>(wl_lds);

  for (int gi = g0 + wave; gi < g1; gi += 4) {
    const int img = gi / g.gpi, ty0 = (gi - img * g.gpi) * g.R;
    // opaque per group: the per-step DMA offsets below are computed at their use, not hoisted out of
    // the group loop into ~100 live SGPRs
    int cst = cstep;
    unsigned rg = ring;
    asm volatile("" : "+s"(cst), "+s"(rg));
    // this lane's DMA sources: staged element e = i 64 + lane of a channel = padded row e / Wp,
    // column e % Wp (column 0 and W + 1 .. Wp - 1 are padding) -> input row 2 ty0 - 1 + row
    int voff[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int e = i * 64 + lane;
      const int rr = e / g.Wp, cc = e - rr * g.Wp;
      const int row = 2 * ty0 - 1 + rr, col = cc - 1;
      voff[i] = (rr < 2 * g.R + 2 && (unsigned)row < (unsigned)p.H && (unsigned)col < (unsigned)p.W)
                    ? (int)((img * p.x_nstride + (long long)row * p.W + col) * 4)
                    : WG_OOB;
    }
    // this lane's tile and its window's base in a staged channel (floats)
    const int tyl = lc / g.TW, tx = lc - tyl * g.TW;
    const bool tok = lc < g.R * g.TW && ty0 + tyl < g.TH;
    const int wbase = (2 * tyl) * g.Wp + 2 * tx + lr * CHUNK;
    const float* rowp[4];  // the window's rows in ring slot 0 (other slots: + a constant offset)
#pragma unroll
    for (int r = 0; r < 4; ++r) rowp[r] = wl_lds + ringf + wbase + r * g.Wp;
    WgTile w;
    w.tok = tok;
    w.ybase = img * (int)p.y_nstride + (2 * (ty0 + tyl)) * p.W + 2 * tx;
    w.c1ok = 2 * tx + 1 < p.W;
    w.r1ok = 2 * (ty0 + tyl) + 1 < p.H;

#define WL_STAGE(SLOT, S)                                                                              \
    _Pragma("unroll") for (int ch = 0; ch < 2; ++ch)                                                   \
    _Pragma("unroll") for (int i = 0; i < NI; ++i)                                                     \
      wl_dma(xdesc, rg + (((SLOT) * 2 + ch) * CHUNK + i * 64) * 4, voff[i], (2 * (S) + ch) * cst);
#define WL_READ(SLOT, S, RA, V)                                                                        \
    {                                                                                                  \
      float d_[4][4];                                                                                  \
      _Pragma("unroll") for (int r = 0; r < 4; ++r)                                                    \
      _Pragma("unroll") for (int j = 0; j < 4; ++j) d_[r][j] = rowp[r][(SLOT) * 2 * CHUNK + j];        \
      _Pragma("unroll") for (int q = 0; q < 4; ++q) RA[q] = ul[((2 * (S) + lr) * 4 + q) * 32 + lc];    \
      wg_input_transform(d_, V);                                                                       \
    }
    floatx16_t acc[16];
#pragma unroll
    for (int xi = 0; xi < 16; ++xi)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[xi][e] = 0.0f;
#pragma unroll
    for (int s = 0; s < DR && s < NKS; ++s) { WL_STAGE(s, s) }
    wg_floatx4 ra[2][4];
    float v[2][16];
    __builtin_amdgcn_s_waitcnt(WL_VMCNT(2 * NI * ((DR < NKS ? DR : NKS) - 1)));
    WL_READ(0, 0, ra[0], v[0])
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      const int cur = s & 1, nxt = cur ^ 1;
      __builtin_amdgcn_sched_barrier(0);  // keep each step's LDS reads in their step (register pressure)
      if (s + 1 < NKS) {
        // step s + 1's staged rows have landed (the DMAs of the `later` steps after it may still be in
        // flight; every older VMEM operation, epilogue stores included, has completed)
        const int later = (DR - 2 < NKS - 2 - s ? DR - 2 : NKS - 2 - s);
        if (later >= 2) __builtin_amdgcn_s_waitcnt(WL_VMCNT(2 * 2 * NI));
        else if (later == 1) __builtin_amdgcn_s_waitcnt(WL_VMCNT(2 * NI));
        else __builtin_amdgcn_s_waitcnt(WL_VMCNT(0));
        WL_READ((s + 1) % DR, s + 1, ra[nxt], v[nxt])
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int xi = 0; xi < 16; ++xi)
        acc[xi] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[cur][xi >> 2][xi & 3], v[cur][xi], acc[xi], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if (s + DR < NKS) {
        // slot s % DR was read (step s's window, before the previous MFMAs): refill it for step s + DR
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this lane's reads of the slot are done
        WL_STAGE(s % DR, s + DR)
      }
    }
#undef WL_STAGE
#undef WL_READ
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int rw = (e & 3) + 8 * (e >> 2);
      const int m = m0 + rw + 4 * lr;
      // the two lane halves' biases by scalar loads (lgkmcnt: no wait on the stores issued before)
      const float b0 = p.bias ? p.bias[min(m0 + rw, p.M - 1)] : 0.0f;
      const float b1 = p.bias ? p.bias[min(m0 + rw + 4, p.M - 1)] : 0.0f;
      if (m < p.M) {
        float mx[16];
#pragma unroll
        for (int xi = 0; xi < 16; ++xi) mx[xi] = acc[xi][e];
        wg_store(p, w, m, lr ? b1 : b0, mx);
      }
      __builtin_amdgcn_sched_barrier(0);  // one accumulator row at a time (register pressure)
    }
  }
}

// Winograd tiles (ConvPlan cfg = WINO_TILE_BASE + t): shape (32: 32x32x2, 16: 16x16x4), channels and
// 2x2 tiles per wave, A / B ring depths of the unrolled K loop
struct WinoTile { int shape, ch, tiles, da, db; };
static const WinoTile WINO_TILES[WINO_TILES_N] = {{32, 32, 32, 2, 8}, {32, 32, 32, 2, 4}, {16, 32, 16, 2, 8},
                                                  {16, 16, 32, 2, 4}, {0, 32, 32, 0, 4}};  // 4: conv_winol_kernel
constexpr int WL_DR = 4;

// the LDS kernel's geometry; false when the layer does not fit it
static bool wl_geom(const ConvParams& p, WlGeom* g, int* ni, size_t* lds) {
  if (p.C % 16 != 0 || p.C > 64 || p.C <= 0) return false;
  g->TW = (p.W + 1) / 2;
  g->TH = (p.H + 1) / 2;
  if (g->TW > 32) return false;
  g->R = std::min(32 / g->TW, g->TH);
  g->Wp = 2 * g->TW + 2;
  const int floats = (2 * g->R + 2) * g->Wp;
  if (floats > 256) return false;
  *ni = floats > 192 ? 4 : 3;
  g->gpi = (g->TH + g->R - 1) / g->R;
  g->G = p.N * g->gpi;
  g->ubytes = p.C * 4 * 32 * 16;
  g->ringb = (WL_DR * 2 * ((*ni) * 64 + 1) * 4 + 15) / 16 * 16;
  *lds = (size_t)g->ubytes + 4 * (size_t)g->ringb;
  return *lds <= 160 * 1024;
}

// the fused 1x1 conv (ConvParams::e1_*) runs in the unrolled 16x16 kernel of tile 2 (32 channels x
// 16 tiles per wave: room for its accumulators beside the Winograd ones)
bool conv_wino_e1_eligible(const ConvParams& p, int tile) {
  return tile == 2 && p.C % 16 == 0 && p.C >= 16 && p.C <= 64 && p.e1_wp && p.e1_y && p.e1_Mp >= (p.M + 31) / 32 * 32 &&
         (long long)p.C * p.e1_Mp * 4 < (1LL << 31) && conv_wino_eligible(p, tile);
}

bool conv_wino_geometry(int C, int kh, int kw, int sh, int sw, int pt, int pl, int H, int W, int Ho, int Wo) {
  return kh == 3 && kw == 3 && sh == 1 && sw == 1 && pt == 1 && pl == 1 && Ho == H && Wo == W && C % 16 == 0 && C > 0;
}

bool conv_wino_eligible(const ConvParams& p, int tile) {
  if (tile < 0 || tile >= WINO_TILES_N) return false;
  if (tile == 4) {
    WlGeom g;
    int ni;
    size_t lds;
    return conv_wino_geometry(p.C, p.kh, p.kw, p.sh, p.sw, p.pt, p.pl, p.H, p.W, p.Ho, p.Wo) && wl_geom(p, &g, &ni, &lds) &&
           p.x_bytes > 0 && p.x_bytes < (1LL << 31) - (1LL << 21) && p.Mp % 64 == 0;
  }
  const WinoTile& wt = WINO_TILES[tile];
  const int nks = p.C / (wt.shape == 32 ? 2 : 4);
  return conv_wino_geometry(p.C, p.kh, p.kw, p.sh, p.sw, p.pt, p.pl, p.H, p.W, p.Ho, p.Wo) && nks % 2 == 0 &&
         p.x_bytes > 0 && p.x_bytes < (1LL << 31) - (1LL << 21) && (reinterpret_cast<uintptr_t>(p.x) & 3) == 0 &&
         p.Mp % 64 == 0 && (long long)p.C * p.Mp * 64 < (1LL << 31) &&
         (long long)p.N * ((p.H + 1) / 2) * ((p.W + 1) / 2) < (1LL << 30);
}

static void wg_grid(ConvParams& p, int ch, int tiles, dim3* grid) {
  const long long T = (long long)p.N * ((p.H + 1) / 2) * ((p.W + 1) / 2);
  p.mtiles = (p.M + ch - 1) / ch;
  p.ntiles = (int)((T + tiles - 1) / tiles);
  const long long waves = (long long)p.mtiles * p.ntiles;
  *grid = dim3((unsigned)((waves + 3) / 4));
}

template <int NKS, int NI>
static void launch_wl(const ConvParams& p, const WlGeom& g, size_t lds, dim3 grid, hipStream_t s) {
  if (lds > 64 * 1024) {  // above the default dynamic-LDS limit: raise it once per device and instantiation
    static std::atomic<unsigned long long> raised{0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    const unsigned long long bit = 1ull << (dev & 63);
    if (!(raised.load(std::memory_order_acquire) & bit)) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_winol_kernel<NKS, NI, WL_DR>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      raised.fetch_or(bit, std::memory_order_acq_rel);
    }
  }
  hipLaunchKernelGGL((conv_winol_kernel<NKS, NI, WL_DR>), grid, dim3(256), lds, s, p, g);
}

static void launch_winol(const ConvParams& p0, hipStream_t s) {
  ConvParams p = p0;
  WlGeom g;
  int ni = 3;
  size_t lds = 0;
  if (!wl_geom(p, &g, &ni, &lds)) return;  // the caller checked conv_wino_eligible
  p.mtiles = (p.M + 31) / 32;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    hipDeviceProp_t prop;
    ncu = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) ? prop.multiProcessorCount
                                                                                                   : 256;
  }
  const int bpc = lds <= 80 * 1024 ? 2 : 1;  // blocks per CU the LDS allows
  // one round of blocks over the chip, at least 4 groups (one per wave) per block and one block per m-tile
  g.bpm = std::max(p.mtiles, std::min(ncu * bpc, p.mtiles * ((g.G + 3) / 4)));
  const dim3 grid((unsigned)g.bpm);
  switch (p.C / 16 * 10 + ni) {
    case 13: launch_wl<8, 3>(p, g, lds, grid, s); break;
    case 14: launch_wl<8, 4>(p, g, lds, grid, s); break;
    case 23: launch_wl<16, 3>(p, g, lds, grid, s); break;
    case 24: launch_wl<16, 4>(p, g, lds, grid, s); break;
    case 33: launch_wl<24, 3>(p, g, lds, grid, s); break;
    case 34: launch_wl<24, 4>(p, g, lds, grid, s); break;
    case 43: launch_wl<32, 3>(p, g, lds, grid, s); break;
    default: launch_wl<32, 4>(p, g, lds, grid, s); break;
  }
}

void launch_conv_wino(const ConvParams& p0, int tile, hipStream_t s) {
  if (tile == 4) {
    launch_winol(p0, s);
    return;
  }
  ConvParams p = p0;
  const WinoTile& wt = WINO_TILES[tile < 0 || tile >= WINO_TILES_N ? 0 : tile];
  dim3 grid;
  wg_grid(p, wt.ch, wt.tiles, &grid);
  // C = 16, 32, 48, 64 (SqueezeNet's expand3x3 inputs): K loop fully unrolled
  const int cq = p.C % 16 == 0 && p.C <= 64 ? p.C / 16 : 0;
#define WG_L32(DA_, DB_, CQ) hipLaunchKernelGGL((conv_wino32_kernel<DA_, DB_, 8 * CQ>), grid, dim3(256), 0, s, p)
#define WG_L16(MF_, NT_, DA_, DB_, CQ) \
  hipLaunchKernelGGL((conv_wino16_kernel<MF_, NT_, DA_, DB_, 4 * CQ, false>), grid, dim3(256), 0, s, p)
#define WG_L16E(CQ) hipLaunchKernelGGL((conv_wino16_kernel<2, 1, 2, 8, 4 * CQ, true>), grid, dim3(256), 0, s, p)
  if (p.e1_y) {  // the fused 1x1 conv: tile 2, C in 16..64 by 16 (conv_wino_e1_eligible)
    switch (cq) {
      case 1: WG_L16E(1); break;
      case 2: WG_L16E(2); break;
      case 3: WG_L16E(3); break;
      default: WG_L16E(4); break;
    }
    return;
  }
#define WG_BY_C(L, ...)                         \
  switch (cq) {                                 \
    case 1: L(__VA_ARGS__, 1); break;           \
    case 2: L(__VA_ARGS__, 2); break;           \
    case 3: L(__VA_ARGS__, 3); break;           \
    case 4: L(__VA_ARGS__, 4); break;           \
    default: L(__VA_ARGS__, 0); break;          \
  }
  switch (tile) {
    case 0: WG_BY_C(WG_L32, 2, 8); break;
    case 1: WG_BY_C(WG_L32, 2, 4); break;
    case 2: WG_BY_C(WG_L16, 2, 1, 2, 8); break;
    default: WG_BY_C(WG_L16, 1, 2, 2, 4); break;
  }
#undef WG_BY_C
#undef WG_L16
#undef WG_L16E
#undef WG_L32
}

}  // namespace ore
