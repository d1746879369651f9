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
typedef float wg_f2 __attribute__((ext_vector_type(2)));

// U[((c * 4 + xi / 4) * Mp + m) * 4 + xi % 4] = s_xi (G g_mc G^T)[xi / 4][xi % 4] (f64, rounded once; the
// sign s_xi = -1 for xi % 4 == 3, +1 otherwise, and V is stored with the same signs, so every product
// U_xi V_xi is the unsigned one exactly; the packed input transform needs it, wg_input_transform_pk): for a
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
      if ((i & 3) == 3) v = -v;  // positions 4 i + 3 carry the sign (V likewise, wg_input_transform)
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
// v[4 i + j] = s_(4 i + j) V[i][j] (the packing's signs: column 3 negated)
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
    v[4 * i + 3] = t[i][3] - t[i][1];  // -(t1 - t3), exactly
  }
}

// wg_input_transform on packed f32 (v_pk_add_f32 / v_pk_fma_f32: two lanes' worth of adds per VALU
// instruction; the same adds on the same operands, so bit-identical): d[i][h] = (d[i][2h], d[i][2h + 1]),
// v[2 i + h] = (v[4 i + 2h], v[4 i + 2h + 1]).  The row pass pairs two columns.  The column pass takes
// (t0 - t2, t1 + t2) = t2 * (-1, 1) + (t0, t1) (a product by +-1 is exact, one rounding: the sum) and,
// thanks to the negated position 3, (t2 - t1, t3 - t1) = (t2, t3) - t1: two instructions per row.
// (Inline-asm packed adds with op_sel would do the same, but the compiler's hazard recognizer does not
// see inline asm as VALU, and MFMA operands read beside them came out wrong on gfx950.)
__device__ __forceinline__ void wg_input_transform_pk(const wg_f2 (&d)[4][2], wg_f2 (&v)[8]) {
  wg_f2 tr[4][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    tr[0][h] = d[0][h] - d[2][h];
    tr[1][h] = d[1][h] + d[2][h];
    tr[2][h] = d[2][h] - d[1][h];
    tr[3][h] = d[1][h] - d[3][h];
  }
  const wg_f2 pm = {-1.0f, 1.0f};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const wg_f2 a = tr[i][0], b = tr[i][1];  // (t0, t1), (t2, t3)
    v[2 * i] = __builtin_elementwise_fma(__builtin_shufflevector(b, b, 0, 0), pm, a);
    v[2 * i + 1] = b - __builtin_shufflevector(a, a, 1, 1);
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

// wg_output_transform of two (channel, tile) pairs at once (packed f32, the same adds in the same order)
__device__ __forceinline__ void wg_output_transform_pk(const wg_f2 (&mx)[16], wg_f2 (&y)[4]) {
  wg_f2 t0[4], t1[4];
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

// a tile's (up to) 4 output pixels o[2 i + j] of channel m -> yb (p.y's plane and image strides)
__device__ __forceinline__ void wg_store_px(const ConvParams& p, const WgTile& w, float* yb, int m, const float (&o)[4]) {
  if (!w.tok) return;
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

// wg_store with the Relu a compile-time choice (a runtime one costs a select per pixel)
template <bool RELU>
__device__ __forceinline__ void wg_store_t(const ConvParams& p, const WgTile& w, int m, float b, const float (&mx)[16]) {
  float o[4];
  wg_output_transform(mx, o);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    o[q] += b;
    if constexpr (RELU) o[q] = fmaxf(o[q], 0.0f);
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
#define WG_LOAD_A(SLOT, S_)                                                                            \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) ra[SLOT][i] = __builtin_bit_cast(                    \
        wg_floatx4, __builtin_amdgcn_raw_buffer_load_b128(ur, aoff + aq * i, (S_) * astep, 0));
#define WG_LOAD_B(SLOT, S_)                                                                            \
    _Pragma("unroll") for (int r = 0; r < 4; ++r) rb[SLOT][r] = __builtin_bit_cast(                    \
        wg_floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, w.roff[r], (S_) * xstep, 0));
#define WG_MFMA(SA, SB)                                                                                \
  {                                                                                                    \
    float v_[16];                                                                                      \
    wg_window(rb[SB], w, v_);                                                                          \
    WG_MFMAS(SA, v_)                                                                                   \
  }
#define WG_MFMAS(SA, V)                                                                                \
    _Pragma("unroll") for (int xi = 0; xi < 16; ++xi)                                                  \
        acc[xi] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[SA][xi >> 2][xi & 3], V[xi], acc[xi], 0, 0, 0);
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
template <int MF, int NT, int DA, int DB, int NKS>
__global__ __launch_bounds__(256, 1) void conv_wino16_kernel(ConvParams p) {
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
  float vc_[NT][16], vn_[NT][16];
  WG_KLOOP(p.C >> 2)
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
      }
    }
}

// ---------------------------------------------------------------------------------------------------
// LDS-staged Winograd kernel (tile 4, "wino lds").  The register-streaming kernels above move each
// lane's own window and U values through the vector-memory path every k-step (the texture path ran
// ~80 % busy at ~41-45 % MFMA, profiles/r02b_pmc_wino32_vs_gemm_f8e3.txt, profiles/r03_pmc_wino_tiles.txt);
// a first LDS kernel with 32x32x2 tiles (512 registers, one wave per SIMD) lost to them: its
// per-workgroup prologue and epilogue were never overlapped (profiles/r03_wino_lds_ablation.txt).
// This one runs two waves per SIMD (<= 256 registers) and two workgroups per CU:
//   * a workgroup of 4 waves owns 64 consecutive 2x2 tiles (16 per wave, flattened over the batch) x 32
//     output channels; lane (lk, lj) of the 16x16x4 MFMAs supplies channel k = lk and tile / output row
//     lj, the wave's two 16-channel fragments are channels m0 + lj and m0 + 16 + lj;
//   * K in chunks of WM_KC = 8 input channels, double-buffered in LDS.  Per chunk and channel the input
//     rows the 64 tiles read are copied as contiguous runs (one per image the group touches, rows clamped
//     to the image) global -> LDS by 16-B LDS-DMA; U of the 32 channels likewise.  The next chunk's DMAs
//     are in flight during this chunk's MFMAs; one barrier per chunk.  Window rows outside the image
//     read a zero block at the start of the channel's area; window columns outside the image are
//     zeroed by per-lane selects (exact zeros: the other tiles' zero padding);
//   * per k-step (4 channels) a lane reads its 4x4 window (ds_read2_b32) and 8 U quads (ds_read_b128),
//     transforms the window (32 adds) and issues 32 v_mfma_f32_16x16x4_f32 (1024 cycles per wave); the
//     next k-step's U quads are read as the MFMAs that used the current ones issue.
// Each position is the same c-ordered fma chain and the transforms the same add order as tiles 0-3:
// bit-identical to them.
constexpr int WM_KC = 8;      // input channels per K chunk (2 k-steps of 4)
constexpr int WM_TILES = 64;  // 2x2 tiles per workgroup (16 per wave)
constexpr int WM_CH = 32;     // output channels per workgroup
constexpr int WM_ZL = 8;      // zero floats at the start of a staged channel (rows outside the image)

__device__ __forceinline__ void wm_dma16(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_addr, int voffset, int soffset) {
  ore_lds_dma16(rsrc, lds_addr, voffset, soffset);
}

// geometry of the LDS kernel (host-computed)
struct WmGeom {
  int TW, TPI;            // tiles per row / per image
  float rTW, rTPI, rNMG;  // 1 / TW, 1 / TPI, 1 / nmg (wm_div)
  int CS;                 // LDS floats per staged channel: zero block + the longest run set + slack (= 32 mod 64)
  int ntg;                // tile groups of WM_TILES
  int mbs;                // 32-channel m-blocks per workgroup (its m-group)
  int nmg;                // m-groups per tile group = ceil(mtiles / mbs)
};

// n / d for 0 <= n < 2^22 (wm_geom checks the workgroup and tile counts) from a float reciprocal rd = 1 / d:
// the float quotient is within (n / d) 2^-23 < 1 / (2 d) of n / d, so the truncation is the quotient or one
// below, fixed by the remainder
__device__ __forceinline__ int wm_div(int n, int d, float rd) {
  int q = (int)((float)n * rd);
  q += n - q * d >= d ? 1 : 0;
  return q;
}

// rows of image `img` staged for the tile group [t0, t1]: [rs, re], clamped to the image
__host__ __device__ __forceinline__ void wm_rows(int img, int img0, int ty0, int img1, int ty1, int H, int* rs, int* re) {
  *rs = img == img0 ? max(0, 2 * ty0 - 1) : 0;
  *re = img == img1 ? min(H - 1, 2 * ty1 + 2) : H - 1;
}

// floats staged per channel for the tile group starting at t0 (each image's run + 1, rounded up to 4)
static int wm_group_floats(long long t0, long long T, int TPI, int TW, int H, int W, int tiles) {
  const long long t1 = std::min(T, t0 + tiles) - 1;
  const int img0 = (int)(t0 / TPI), ty0 = (int)(t0 % TPI) / TW;
  const int img1 = (int)(t1 / TPI), ty1 = (int)(t1 % TPI) / TW;
  int total = 0;
  for (int i = img0; i <= img1; ++i) {
    int rs, re;
    wm_rows(i, img0, ty0, img1, ty1, H, &rs, &re);
    total += ((re - rs + 1) * W + 4) & ~3;  // one spare float: odd channels' shifted last element
  }
  return total;
}

// Round 6: a workgroup owns a tile group x an m-group of mbs 32-channel blocks and walks the blocks in turn
// (each of the 4-8 channel blocks of a tile group re-ran the whole prologue -- the index
// arithmetic, the run layout, the first stage's latency -- for only C / 8 chunks of MFMAs).  The chunk
// pipeline runs on across the blocks: the last chunk of block b stages chunk 0 of block b + 1 (the same
// windows, the next block's U), so only the workgroup's first stage is exposed, and block b's epilogue
// (output transform, stores) runs while that stage lands.  The per-block arithmetic is unchanged (each
// position one c-ordered chain, the same transforms): bit-identical to one block per workgroup.
// (Measured and rejected, round 6: 8-wave workgroups of 128 tiles, one per CU, whose two waves per SIMD share one
// staged copy of each chunk -- half the DMA pieces per wave, but both partners of a SIMD then meet at every
// barrier: fire8 297 -> 342 us, profiles/r06_wino_ablations.txt.)
template <int NDMA, bool RELU>  // NDMA: 256-float DMA pieces per staged channel (ceil(longest run set / 256))
__global__ __launch_bounds__(256, 2) void conv_winol_kernel(ConvParams p, WmGeom g) {
  constexpr int NW = 4, TILES = WM_TILES;
  extern __shared__ __attribute__((aligned(16))) float wm_lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // block -> (tile group, m-group), the m-groups of a tile group consecutive (one XCD: they share the staged
  // rows in L2)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, rr8 = nwg & 7;
  const int wgid = (xcd < rr8 ? xcd * (q8 + 1) : rr8 * (q8 + 1) + (xcd - rr8) * q8) + (bid >> 3);
  // (integer divisions by reciprocals: the wave-uniform ones back to scalars by readfirstlane)
  const int tgi = __builtin_amdgcn_readfirstlane(wm_div(wgid, g.nmg, g.rNMG)), mg = wgid - tgi * g.nmg;
  const int mb0 = mg * g.mbs, mb1 = min(p.mtiles, mb0 + g.mbs);
  const int mw0 = mb0 * WM_CH, nch = (mb1 - mb0) * WM_CH;  // the workgroup's channels [mw0, mw0 + nch)
  const int T = p.N * g.TPI;
  const int t0 = tgi * TILES, t1 = min(T, t0 + TILES) - 1;
  const int img0 = __builtin_amdgcn_readfirstlane(wm_div(t0, g.TPI, g.rTPI));
  const int ty0 = __builtin_amdgcn_readfirstlane(wm_div(t0 - img0 * g.TPI, g.TW, g.rTW));
  const int img1 = __builtin_amdgcn_readfirstlane(wm_div(t1, g.TPI, g.rTPI));
  const int ty1 = __builtin_amdgcn_readfirstlane(wm_div(t1 - img1 * g.TPI, g.TW, g.rTW));
  const int SS = WM_KC * (g.CS + 512);  // floats per stage: [channel][CS] windows, then [channel][4 quads][32 m][4] U

  // the workgroup's biases (0 past M), read by the epilogues: loaded to a register here and written to LDS
  // after the first stage's DMAs have issued, so the prologue's wait for the first chunk covers their latency
  const bool bias_lane = (int)threadIdx.x < nch;
  float bias_v = 0.0f;
  if (bias_lane) {
    const int m = mw0 + (int)threadIdx.x;
    bias_v = p.bias && m < p.M ? p.bias[m] : 0.0f;
  }

  // ---- this lane's tile (lj of the wave's 16) and the run layout of the group
  const int lk = lane >> 4, lj = lane & 15;
  int t = t0 + 16 * wave + lj;
  WgTile w;
  w.tok = t < T;
  if (!w.tok) t = T - 1;
  const int img = wm_div(t, g.TPI, g.rTPI), rem = t - img * g.TPI, ty = wm_div(rem, g.TW, g.rTW), tx = rem - ty * g.TW;
  // DMA piece gi of a channel: floats [4 (64 gi + lane), +4) of the run set
  int voff[NDMA];
#pragma unroll
  for (int gi = 0; gi < NDMA; ++gi) voff[gi] = -1;
  int my_lb = 0, my_rs = 0;
  int lb = 0;
  for (int i = img0; i <= img1; ++i) {
    int rs, re;
    wm_rows(i, img0, ty0, img1, ty1, p.H, &rs, &re);
    const int len = (re - rs + 1) * p.W;
#pragma unroll
    for (int gi = 0; gi < NDMA; ++gi) {
      const int k4 = 4 * (64 * gi + lane);
      if (k4 >= lb && k4 <= lb + len) voff[gi] = (int)((i * p.x_nstride + (long long)rs * p.W + (k4 - lb)) * 4);
    }
    if (i == img) {
      my_lb = lb;
      my_rs = rs;
    }
    lb += (len + 4) & ~3;  // runs of len + 1 floats (odd channels land one float later), rounded to 4
  }
  // window rows (floats from the channel's area; rows outside the image -> the zero block)
  int aw[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int gr = 2 * ty - 1 + r;
    // odd channels are staged one float later (their DMA source starts one float early), so the two
    // channels of a ds_read_b32 lane group (lk = 0, 1: CS = 0 mod 32 apart) use opposite bank parities
    const int rel = ((unsigned)gr < (unsigned)p.H ? WM_ZL + my_lb + (gr - my_rs) * p.W + 2 * tx - 1 : 0) + (lk & 1);
    aw[r] = (lk * g.CS + rel) * 4;  // bytes, channel lk of a k-step
  }
  const bool c0ok = tx > 0, c2ok = 2 * tx + 1 < p.W, c3ok = 2 * tx + 2 < p.W;
  w.ybase = img * (int)p.y_nstride + (2 * ty) * p.W + 2 * tx;
  w.c1ok = 2 * tx + 1 < p.W;
  w.r1ok = 2 * ty + 1 < p.H;
  const int au = (WM_KC * g.CS + lk * 512 + lj * 4) * 4;  // bytes: U[c = lk][quad 0][m = lj] of a k-step

  // ---- DMA sources: wave w stages channels w and w + 4 of a chunk, and U pieces d = w + 4 v
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.x), (short)0, (int)p.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ur =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.wp), (short)0, p.C * p.Mp * 16 * 4, 0x00020000);
  const int uq = 2 * (wave & 1) + (lane >> 5);
  const int uoff = (uq * p.Mp + (lane & 31)) * 16;  // the block's first channel goes in the scalar offset
  const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) float*)wm_lds;
  const int nchunks = p.C / WM_KC;  // even (C % 16 == 0): chunk 0 of every block uses stage 0
  // chunk kc's windows and U of channels [m0, m0 + 32) -> stage st
  auto stage = [&](int kc, int m0, int st) __attribute__((always_inline)) {
    const unsigned sb = lds0 + (unsigned)(st * SS) * 4;
#pragma unroll
    for (int h = 0; h < 8 / NW; ++h) {
      const int cc = wave + NW * h;
      const int so = (kc * WM_KC + cc) * p.x_ps * 4 - 4 * (cc & 1);  // odd channels: one float early (>= 0)
#pragma unroll
      for (int gi = 0; gi < NDMA; ++gi)
        if (voff[gi] >= 0) wm_dma16(xr, sb + (cc * g.CS + WM_ZL + 256 * gi) * 4, voff[gi], so);
    }
#pragma unroll
    for (int v = 0; v < 16 / NW; ++v) {
      const int d = wave + NW * v, cc = d >> 1;
      wm_dma16(ur, sb + (WM_KC * g.CS + (cc * 4 + 2 * (d & 1)) * 128) * 4, uoff,
               ((kc * WM_KC + cc) * 4 * p.Mp + m0) * 16);
    }
  };

  // accumulators: no zeroing -- each block's first k-step takes C = 0 (an inline operand of the MFMA; 128
  // v_mov per wave otherwise, and f32 MFMAs and VALU share the SIMD's issue, nothing overlaps them)
  wg_floatx4 acc[16][2];
  const wg_floatx4 zero4 = {0.f, 0.f, 0.f, 0.f};

  const char* lds_b = reinterpret_cast<const char*>(wm_lds);
  auto load_win = [&](int sto, wg_f2 (&d)[4][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        d[r][j >> 1][j & 1] = *reinterpret_cast<const float*>(lds_b + aw[r] + sto + 4 * j);
  };
  auto load_u = [&](int sto, int f, int q) __attribute__((always_inline)) {
    return *reinterpret_cast<const wg_floatx4*>(lds_b + au + sto + q * 512 + f * 256);  // m = 16 f + lj
  };
  auto xform = [&](wg_f2 (&d)[4][2], wg_f2 (&v)[8]) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      d[r][0][0] = c0ok ? d[r][0][0] : 0.0f;
      d[r][1][0] = c2ok ? d[r][1][0] : 0.0f;
      d[r][1][1] = c3ok ? d[r][1][1] : 0.0f;
    }
    wg_input_transform_pk(d, v);
  };
  // one chunk (two k-steps of 4 channels) of the block at m0; FIRST: chunk 0, its first k-step starts the
  // accumulators.  It first stages the next job: chunk kc + 1 of this block, or chunk 0 of the next block
  // (more), or nothing
  // PRE: chunk 0 of a block after the first, whose next job (chunk 1) was staged before the previous block's
  // epilogue (see the block loop)
  auto chunk = [&](int kc, int m0, bool more, auto first, auto stc, auto prec) __attribute__((always_inline)) {
    constexpr bool FIRST = decltype(first)::value;
    constexpr int st = decltype(stc)::value;  // kc & 1, a constant: the stage's LDS bases are loop-invariant
    constexpr bool PRE = decltype(prec)::value;
    if constexpr (!PRE) {
      if (kc + 1 < nchunks)
        stage(kc + 1, m0, st ^ 1);
      else if (more)
        stage(0, m0 + WM_CH, st ^ 1);
    }
    const int sto0 = st * SS * 4, sto1 = sto0 + 4 * g.CS * 4;  // k-step 1: channels 4 .. 7 of the chunk
    wg_floatx4 ua[2][4];
    wg_f2 d0[4][2], d1[4][2], v[8];  // v[2 i + h][e]: position 4 i + 2 h + e
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int f = 0; f < 2; ++f) ua[f][q] = load_u(sto0, f, q);
    load_win(sto0, d0);
    xform(d0, v);
    load_win(sto1, d1);
    __builtin_amdgcn_sched_barrier(0);
    // k-step 0; U of k-step 1 (its channels' quads at +4 * 512 floats) replaces each quad once used
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int f = 0; f < 2; ++f)
          acc[4 * q + j][f] =
              __builtin_amdgcn_mfma_f32_16x16x4f32(ua[f][q][j], v[2 * q + (j >> 1)][j & 1], FIRST ? zero4 : acc[4 * q + j][f], 0, 0, 0);
#pragma unroll
      for (int f = 0; f < 2; ++f) ua[f][q] = load_u(sto0 + 4 * 512 * 4, f, q);
    }
    __builtin_amdgcn_sched_barrier(0);
    xform(d1, v);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int f = 0; f < 2; ++f)
          acc[4 * q + j][f] = __builtin_amdgcn_mfma_f32_16x16x4f32(ua[f][q][j], v[2 * q + (j >> 1)][j & 1], acc[4 * q + j][f], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    // this wave's DMAs of the next job have landed (vmcnt counts DMAs and stores in issue order: after an
    // epilogue, whose >= 16 stores followed them, the stores need not have completed)
    if constexpr (PRE)
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // ... every wave's, and every wave is done reading stage st
  };

  stage(0, mw0, 0);
  // the zero blocks (never written by the DMAs) and the biases after the two stages
  if (threadIdx.x < 2 * WM_KC * WM_ZL)
    wm_lds[(threadIdx.x >> 6) * SS + ((threadIdx.x >> 3) & 7) * g.CS + (threadIdx.x & 7)] = 0.0f;
  if (bias_lane) wm_lds[2 * SS + (int)threadIdx.x] = bias_v;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // stores without branches: 8-B row stores at per-lane byte offsets fixed for the kernel (the tile, channel
  // 4 lk), with the block's channel as the scalar offset; a missing tile, row or second column (the right
  // edge of an odd-width plane) has its offset past the output (the buffer range check drops the store), and
  // a wave with such right-edge tiles (fast = false) also issues their 4-B first-column stores.  Channels
  // past M (a partial last block) take the per-lane check
  const int oob = 0x7FFFFFF0;
  const int ylane = (w.ybase + 4 * lk * p.y_ps) * 4;
  const int so0 = w.tok && w.c1ok ? ylane : oob, so1 = w.tok && w.c1ok && w.r1ok ? ylane + p.W * 4 : oob;
  const int se0 = w.tok && !w.c1ok ? ylane : oob, se1 = w.tok && !w.c1ok && w.r1ok ? ylane + p.W * 4 : oob;
  const bool fast = __builtin_amdgcn_ballot_w64(w.tok && !w.c1ok) == 0;
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(p.y, (short)0, 0x7FFFFFF0, 0x00020000);
  typedef int wg_i2 __attribute__((ext_vector_type(2)));
  // (an epilogue issues 16 8-B stores per wave, 32 stores with the right-edge ones: the vmcnt(16) of the
  // next chunk relies on >= 16)
  // the output transform and bias of channels (e, e + 1) on packed f32 (acc[xi][f] holds e = 0 .. 3 in
  // consecutive registers), the same adds in the same order as wg_store_t, then the stores; MOK: channel
  // checks (a partial last block)
  auto epilogue = [&](int m0, auto mokc) __attribute__((always_inline)) {
    constexpr bool MOK = decltype(mokc)::value;
    // lane (lk, lj) of fragment f holds rows 4 lk + e = channel m0 + 16 f + 4 lk + e of tile lj
    wg_floatx4 bv[2];
#pragma unroll
    for (int f = 0; f < 2; ++f)
      bv[f] = *reinterpret_cast<const wg_floatx4*>(wm_lds + 2 * SS + (m0 - mw0) + 16 * f + 4 * lk);
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int ep = 0; ep < 4; ep += 2) {
        wg_f2 mx[16], y[4];
#pragma unroll
        for (int xi = 0; xi < 16; ++xi) mx[xi] = ep == 0 ? acc[xi][f].xy : acc[xi][f].zw;
        wg_output_transform_pk(mx, y);
        const wg_f2 b2 = {bv[f][ep], bv[f][ep + 1]};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float o[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            o[q] = (y[q] + b2)[h];
            if constexpr (RELU) o[q] = fmaxf(o[q], 0.0f);
          }
          const int c = m0 + 16 * f + ep + h;  // the channel of lane group lk = 0
          const int soff = c * p.y_ps * 4;
          int a0 = so0, a1 = so1, e0 = se0, e1 = se1;
          if constexpr (MOK) {
            const bool mok = c + 4 * lk < p.M;
            a0 = mok ? a0 : oob; a1 = mok ? a1 : oob; e0 = mok ? e0 : oob; e1 = mok ? e1 : oob;
          }
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(wg_i2, (wg_f2){o[0], o[1]}), yr, a0, soff, 0);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(wg_i2, (wg_f2){o[2], o[3]}), yr, a1, soff, 0);
          if (!fast) {  // tiles at the right edge of an odd-width plane: their first column only
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, o[0]), yr, e0, soff, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, o[2]), yr, e1, soff, 0);
          }
        }
      }
  };
  using st0 = std::integral_constant<int, 0>;
  using st1 = std::integral_constant<int, 1>;
  // the blocks in turn.  At a block boundary the next block's chunk 1 is staged (stage 1 is free once the
  // last chunk's barrier has passed) BEFORE the epilogue's stores: vmcnt counts loads, stores and LDS-DMA
  // in issue order, so chunk 0's wait for those DMAs then does not wait for the stores
  using pre0 = std::false_type;
  using pre1 = std::true_type;
  for (int mb = mb0; mb < mb1; ++mb) {
    const int m0 = mb * WM_CH;
    const bool more = mb + 1 < mb1;
    if (mb == mb0)
      chunk(0, m0, more, std::true_type{}, st0{}, pre0{});
    else
      chunk(0, m0, more, std::true_type{}, st0{}, pre1{});
    int kc = 1;
    for (; kc + 1 < nchunks; kc += 2) {  // chunk pairs: odd, even
      chunk(kc, m0, more, std::false_type{}, st1{}, pre0{});
      chunk(kc + 1, m0, more, std::false_type{}, st0{}, pre0{});
    }
    chunk(kc, m0, more, std::false_type{}, st1{}, pre0{});  // the last, odd chunk (nchunks is even)
    if (more) stage(1, m0 + WM_CH, 1);  // the next block's chunk 1
    if (m0 + WM_CH <= p.M)
      epilogue(m0, std::false_type{});
    else
      epilogue(m0, std::true_type{});
  }
}

// workgroups the m-grouping keeps at least (4 per resident slot of a 256-CU part at two per CU): the blocks of
// a tile group are shared out only as far as the launch stays this wide
constexpr long long WM_MIN_WG = 2048;
constexpr int WM_MAX_MBS = 8;

// the LDS kernel's geometry; false when the layer does not fit it
static bool wm_geom(const ConvParams& p, WmGeom* g, size_t* lds, int* ndma) {
  const int tiles = WM_TILES;
  if (p.C % 16 != 0 || p.C <= 0 || p.H <= 0 || p.W <= 0 || p.M <= 0) return false;
  g->TW = (p.W + 1) / 2;
  const int TH = (p.H + 1) / 2;
  g->TPI = g->TW * TH;
  g->rTW = 1.0f / (float)g->TW;
  g->rTPI = 1.0f / (float)g->TPI;
  const long long T = (long long)p.N * g->TPI;
  if (T >= (1LL << 22)) return false;  // wm_div's range (4M tiles: 5,700 images at 54 x 54)
  g->ntg = (int)((T + tiles - 1) / tiles);
  // m-blocks per workgroup: the largest divisor of the block count that keeps >= WM_MIN_WG workgroups
  const int mtiles = (p.M + WM_CH - 1) / WM_CH;
  g->mbs = 1;
  for (int b = 2; b <= std::min(mtiles, WM_MAX_MBS); ++b)
    if (mtiles % b == 0 && (long long)g->ntg * (mtiles / b) >= WM_MIN_WG) g->mbs = b;
  g->nmg = (mtiles + g->mbs - 1) / g->mbs;
  g->rNMG = 1.0f / (float)g->nmg;
  if ((long long)g->ntg * g->nmg >= (1LL << 22)) return false;  // wm_div's range for the workgroup id
  // group starts repeat modulo TPI (period TPI / gcd(tiles, TPI)): every case is among the first TPI
  int tmax = 0;
  const long long ng = std::min<long long>(g->ntg, g->TPI);
  for (long long gi = 0; gi < ng; ++gi)
    tmax = std::max(tmax, wm_group_floats(gi * tiles, T, g->TPI, g->TW, p.H, p.W, tiles));
  *ndma = (tmax + 255) / 256;
  g->CS = (WM_ZL + tmax + 5 + 31) / 64 * 64 + 32;  // + 1: odd channels' shift, + 4: the last window's overrun
  *lds = (size_t)2 * WM_KC * (g->CS + 512) * 4 + (size_t)g->mbs * WM_CH * 4;  // two stages + the biases
  return *ndma <= 8 && *lds <= 160 * 1024;
}

template <int NDMA, bool RELU>
static void launch_wm_r(const ConvParams& p0, const WmGeom& g, size_t lds, hipStream_t s) {
  ConvParams p = p0;
  p.mtiles = (p.M + WM_CH - 1) / WM_CH;
  if (lds > 64 * 1024) {  // above the default dynamic-LDS limit: raise it once per device
    static std::atomic<unsigned long long> raised{0};
    ore_raise_lds_once(raised, reinterpret_cast<const void*>(&conv_winol_kernel<NDMA, RELU>), 160 * 1024);
  }
  hipLaunchKernelGGL((conv_winol_kernel<NDMA, RELU>), dim3((unsigned)(g.ntg * g.nmg)), dim3(256), lds, s, p, g);
}

template <int NDMA>
static void launch_wm(const ConvParams& p, const WmGeom& g, size_t lds, hipStream_t s) {
  if (p.relu)
    launch_wm_r<NDMA, true>(p, g, lds, s);
  else
    launch_wm_r<NDMA, false>(p, g, lds, s);
}

static void launch_winol(const ConvParams& p, hipStream_t s) {
  WmGeom g;
  size_t lds = 0;
  int ndma = 0;
  if (!wm_geom(p, &g, &lds, &ndma)) return;  // the caller checked conv_wino_eligible
  switch (ndma) {
    case 1: launch_wm<1>(p, g, lds, s); break;
    case 2: launch_wm<2>(p, g, lds, s); break;
    case 3: launch_wm<3>(p, g, lds, s); break;
    case 4: launch_wm<4>(p, g, lds, s); break;
    case 5: launch_wm<5>(p, g, lds, s); break;
    case 6: launch_wm<6>(p, g, lds, s); break;
    case 7: launch_wm<7>(p, g, lds, s); break;
    default: launch_wm<8>(p, g, lds, s); break;
  }
}

// Winograd tiles (ConvPlan cfg = WINO_TILE_BASE + t): shape (32: 32x32x2, 16: 16x16x4), channels and
// 2x2 tiles per wave, A / B ring depths of the unrolled K loop
struct WinoTile { int shape, ch, tiles, da, db; };
static const WinoTile WINO_TILES[WINO_TILES_N] = {{32, 32, 32, 2, 8}, {32, 32, 32, 2, 4}, {16, 32, 16, 2, 8},
                                                  {16, 16, 32, 2, 4}, {0, WM_CH, WM_TILES, 0, 0}};  // 4: conv_winol_kernel

bool conv_wino_geometry(int C, int kh, int kw, int sh, int sw, int pt, int pl, int H, int W, int Ho, int Wo) {
  return kh == 3 && kw == 3 && sh == 1 && sw == 1 && pt == 1 && pl == 1 && Ho == H && Wo == W && C % 16 == 0 && C > 0;
}

bool conv_wino_eligible(const ConvParams& p, int tile) {
  if (tile < 0 || tile >= WINO_TILES_N) return false;
  if (tile == 4) {
    WmGeom g;
    size_t lds;
    int ndma;
    return conv_wino_geometry(p.C, p.kh, p.kw, p.sh, p.sw, p.pt, p.pl, p.H, p.W, p.Ho, p.Wo) && wm_geom(p, &g, &lds, &ndma) &&
           p.x_bytes > 0 && p.x_bytes < (1LL << 31) - (1LL << 21) && (reinterpret_cast<uintptr_t>(p.x) & 3) == 0 &&
           p.Mp % 64 == 0 && (long long)p.C * p.Mp * 64 < (1LL << 31) &&
           (long long)p.N * ((p.H + 1) / 2) * ((p.W + 1) / 2) < (1LL << 30) &&
           (long long)p.N * p.y_nstride < (1LL << 31);
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
  hipLaunchKernelGGL((conv_wino16_kernel<MF_, NT_, DA_, DB_, 4 * CQ>), grid, dim3(256), 0, s, p)
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
#undef WG_L32
}

}  // namespace ore
