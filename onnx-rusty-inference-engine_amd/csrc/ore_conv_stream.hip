// Stride-1 Conv (convolution_op.rs:94-517) as an LDS-free, barrier-free streaming implicit GEMM on
// v_mfma_f32_16x16x4_f32 (f32 in, f32 accumulate).  Two operand modes:
//   S1X1:  kh = kw = 1, no padding (SqueezeNet's squeeze / expand1x1 / conv10);
//   STAPS: 3x3, stride 1, Wo == W (horizontally "same": every expand3x3).
//
// The same GEMM as conv_gemm_kernel (ore_conv.hip): Y[m][n] = sum_k W[m][k] B[k][n] + bias[m],
// m = output channel, n = (image, output pixel), k = (cin, r, s) in the reference's order
// (convolution_op.rs:422-480).  Both f32 MFMA shapes are a k-ordered fmaf chain
// (cdna_hip_programming.md 'FP32-input MFMA'), so every output is bit-identical to the LDS-staged
// kernel's and tiles stay interchangeable (ore_model_autotune).
//
// No operand goes through LDS:
//   * B: lane l loads 16 B = 4 consecutive output pixels' values of k = 4s + (l >> 4) (16 lanes = one
//     256-B run).  With stride 1 and Wo == W, output pixel pix reads input element pix + tap offset
//     for every tap, row wraps included, so the 4 values are contiguous in the input (STAPS: 4-B
//     aligned only; taps outside the image are zeroed per element from a per-pixel tap mask -- the
//     reference's zero padding).  Element q of the float4 is the B operand of the q-th of four
//     16x16x4 MFMAs: column slot j = l & 15 of MFMA q is pixel 4j + q, so one load feeds four MFMAs
//     and each lane ends up owning 4 consecutive output pixels per row -> 16-B stores straight from
//     the accumulators.
//   * A: row slot j of fragment f is channel MF*j + f, so lane l's A operands of all MF fragments are
//     MF consecutive floats of the K-major packed weights Wp[k][m] (one 4/8/12/16-B load).
//   * D k-steps of operands are in flight in a register ring; waves never wait on each other.
// Wave tile: 16*MF channels x 64*NB pixels; block = 4 independent waves (consecutive m tiles of one
// pixel tile share the block when M > 16*MF, so the B rows they read hit the CU's L1).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "ore_kernels.h"

namespace ore {

typedef float cs_floatx4 __attribute__((ext_vector_type(4)));
enum { S1X1 = 0, STAPS = 1 };

template <int MF>
__device__ __forceinline__ void cs_load_a(__amdgpu_buffer_rsrc_t r, int voff, int soff, float (&a)[MF]) {
  if constexpr (MF == 8) {
    const cs_floatx4 v = __builtin_bit_cast(cs_floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
    const cs_floatx4 w = __builtin_bit_cast(cs_floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, voff + 16, soff, 0));
    a[0] = v[0]; a[1] = v[1]; a[2] = v[2]; a[3] = v[3];
    a[4] = w[0]; a[5] = w[1]; a[6] = w[2]; a[7] = w[3];
  } else if constexpr (MF == 4) {
    const cs_floatx4 v = __builtin_bit_cast(cs_floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
    a[0] = v[0]; a[1] = v[1]; a[2] = v[2]; a[3] = v[3];
  } else if constexpr (MF == 3) {
    typedef float f3 __attribute__((ext_vector_type(3)));
    const f3 v = __builtin_bit_cast(f3, __builtin_amdgcn_raw_buffer_load_b96(r, voff, soff, 0));
    a[0] = v[0]; a[1] = v[1]; a[2] = v[2];
  } else if constexpr (MF == 2) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 v = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
    a[0] = v[0]; a[1] = v[1];
  } else {
    a[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
  }
}

// MF: 16-row fragments per wave (channels MF*j + f), NB: 64-pixel groups per wave, D: ring depth,
// NT: non-temporal B loads (1x1 convs whose single m tile reads every input element once)
template <int MF, int NB, int D, int MODE, int NT = 0>
__global__ __launch_bounds__(256, 2) void conv_stream_kernel(ConvParams p) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-aware bijective block remap (consecutive block ids -> one XCD's L2), as in conv_gemm_kernel
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, rr8 = nwg & 7;
  const int wgid = (xcd < rr8 ? xcd * (q8 + 1) : rr8 * (q8 + 1) + (xcd - rr8) * q8) + (bid >> 3);
  const int gw = wgid * 4 + wave;
  const int mt = gw % p.mtiles, ct = gw / p.mtiles;
  if (ct >= p.ntiles) return;  // wave-uniform; no barrier anywhere in this kernel
  const int m0 = mt * (16 * MF);
  const int YPS = p.y_ps;      // output plane stride = columns per image (S1X1: == x_ps)
  const int lk = lane >> 4, lj = lane & 15;

  // this lane's 4-pixel column group per 64-pixel block g (clamped into range: the last tile's
  // surplus lanes re-read valid columns and are masked at the store)
  const int ntot = (int)p.Ntot;  // < 2^31 (host)
  int xoff[NB], yoff[NB];
  bool cok[NB];
  unsigned tmask[MODE == STAPS ? NB : 1][4];  // STAPS: bit t = tap t of pixel q reads inside the image
#pragma unroll
  for (int g = 0; g < NB; ++g) {
    int col = ct * (64 * NB) + 64 * g + 4 * lj;
    cok[g] = col < ntot;
    if (!cok[g]) col = ntot - 4;
    const int img = col / YPS;
    const int pix = col - img * YPS;
    yoff[g] = img * (int)p.y_nstride + pix;  // elements
    if constexpr (MODE == S1X1) {
      xoff[g] = (img * (int)p.x_nstride + lk * p.x_ps + pix) * 4;  // bytes; + 16 s x_ps per k-step
    } else {
      // input element of tap (r, s) = pix + (r - pt) W + (s - pl) (stride 1, Wo == W); the tap part
      // is added per k-step
      xoff[g] = (img * (int)p.x_nstride + pix) * 4;
      const int oh0 = pix / p.W, ow0 = pix - oh0 * p.W;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        // pixel pix + q (W >= 3: at most one row wrap); oh >= Ho: a pad column
        const bool wrap = ow0 + q >= p.W;
        const int oh = oh0 + (wrap ? 1 : 0), ow = ow0 + q - (wrap ? p.W : 0);
        unsigned cm = 0, m = 0;
#pragma unroll
        for (int s = 0; s < 3; ++s) cm |= ((unsigned)(ow - p.pl + s) < (unsigned)p.W ? 1u : 0u) << s;
#pragma unroll
        for (int r = 0; r < 3; ++r)
          if (oh < p.Ho && (unsigned)(oh - p.pt + r) < (unsigned)p.H) m |= cm << (r * 3);
        tmask[g][q] = m;
      }
    }
  }
  // STAPS: the resource starts xlead bytes before x so that no tap offset is negative (a negative
  // offset fails the range check for the whole 16-B access, zeroing its valid elements too); the
  // bytes read there belong to masked taps.  Past the end the check is per dword.
  const int xlead = MODE == STAPS ? p.x_lead : 0;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(reinterpret_cast<const char*>(p.x) - xlead), (short)0, (int)p.x_bytes + xlead, 0x00020000);
  const int kp = (p.K + 31) & ~31;
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.wp), (short)0, kp * p.Mp * 4, 0x00020000);
  const int aoff = (lk * p.Mp + m0 + MF * lj) * 4;  // bytes; + 16 s Mp per k-step
  const int xstep = 16 * p.x_ps, astep = 16 * p.Mp;  // bytes per k-step (S1X1: 4 channels)
  // STAPS (3x3 only): this lane's k = 4 s + lk as tap tt = 3 r + s' and channel byte offset cx,
  // advanced by 4 k per k-step (one tap row + one tap column, with carries) -- no table, no LDS
  int tt = lk, cx = 0;
  const int tap0 = xlead - (p.pt * p.W + p.pl) * 4;  // byte offset of tap (0, 0) from the output pixel (>= 0)

  cs_floatx4 acc[MF][NB][4];
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int g = 0; g < NB; ++g)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[f][g][q] = cs_floatx4{0.f, 0.f, 0.f, 0.f};

  cs_floatx4 rb[D][NB];
  float ra[D][MF];
  int rt[MODE == STAPS ? D : 1];  // STAPS: the tap of each ring slot's k (for its zero mask)
  const int nks = p.K >> 2;       // host: K % 16 == 0 and nks % D == 0
#define CS_LOAD(SLOT, S)                                                                          \
  {                                                                                               \
    const int s_ = (S);                                                                           \
    cs_load_a<MF>(wr, aoff, s_ * astep, ra[SLOT]);                                                \
    if constexpr (MODE == S1X1) {                                                                 \
      _Pragma("unroll") for (int g = 0; g < NB; ++g) rb[SLOT][g] = __builtin_bit_cast(          \
          cs_floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, xoff[g], s_ * xstep, NT ? 2 : 0)); \
    } else {                                                                                      \
      /* tt / 3 for tt < 9, 24-bit multiplies (v_mul_u32_u24, full rate; v_mul_lo_u32 is 1/4) */  \
      const int r_ = (int)(__umul24((unsigned)tt, 11u) >> 5);                                     \
      const int to_ = cx + tap0 + 4 * ((int)__umul24((unsigned)r_, (unsigned)(p.W - 3)) + tt);    \
      _Pragma("unroll") for (int g = 0; g < NB; ++g) rb[SLOT][g] = __builtin_bit_cast(          \
          cs_floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, xoff[g] + to_, 0, 0));            \
      rt[SLOT] = tt;                                                                              \
      tt += 4;                                                                                    \
      if (tt >= 9) { tt -= 9; cx += 4 * p.x_ps; }                                                 \
    }                                                                                             \
  }
  // STAPS: zero the taps outside the image (bit extract as a 0 / -1 mask, AND on the float bits)
#define CS_MASK(SLOT)                                                                             \
  if constexpr (MODE == STAPS) {                                                                  \
    _Pragma("unroll") for (int g = 0; g < NB; ++g)                                                \
    {                                                                                             \
      const int4 v_ = __builtin_bit_cast(int4, rb[SLOT][g]);                                      \
      int4 w_;                                                                                    \
      w_.x = v_.x & __builtin_amdgcn_sbfe((int)tmask[g][0], rt[SLOT], 1);                         \
      w_.y = v_.y & __builtin_amdgcn_sbfe((int)tmask[g][1], rt[SLOT], 1);                         \
      w_.z = v_.z & __builtin_amdgcn_sbfe((int)tmask[g][2], rt[SLOT], 1);                         \
      w_.w = v_.w & __builtin_amdgcn_sbfe((int)tmask[g][3], rt[SLOT], 1);                         \
      rb[SLOT][g] = __builtin_bit_cast(cs_floatx4, w_);                                           \
    }                                                                                             \
  }
// the wave's priority is raised around its MFMA group (the SIMD's arbiter then prefers a wave that
// is about to feed the matrix core over one doing address/mask VALU): 1-3 % on the 3x3 layers
#define CS_PRIO(X) __builtin_amdgcn_s_setprio(X);
#define CS_MFMA(SLOT)                                                                             \
  CS_MASK(SLOT)                                                                                   \
  CS_PRIO(1)                                                                                      \
  _Pragma("unroll") for (int f = 0; f < MF; ++f)                                                  \
  _Pragma("unroll") for (int g = 0; g < NB; ++g)                                                  \
  _Pragma("unroll") for (int q = 0; q < 4; ++q)                                                   \
      acc[f][g][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[SLOT][f], rb[SLOT][g][q], acc[f][g][q], 0, 0, 0); \
  CS_PRIO(0)

#pragma unroll
  for (int d = 0; d < D; ++d) CS_LOAD(d, d);
  int s0 = 0;
  for (; s0 < nks - D; s0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      CS_MFMA(d);
      // the refill of slot d issues right behind its MFMAs (left alone, the scheduler sinks every
      // refill below the last MFMA of the group: one load group in flight instead of D)
      __builtin_amdgcn_sched_barrier(0);
      CS_LOAD(d, s0 + D + d);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d) { CS_MFMA(d); }
#undef CS_LOAD
#undef CS_MASK
#undef CS_MFMA

  // epilogue: lane (lk, lj) of fragment f holds rows 4 lk + e = channel m0 + MF (4 lk + e) + f and,
  // in MFMA q, pixel 4 lj + q of each group: one float4 per (f, e, g)
  float* __restrict__ y = p.y;
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + MF * (4 * lk + e) + f;
      if (m >= p.M) continue;
      const float b = p.bias ? p.bias[m] : 0.0f;
#pragma unroll
      for (int g = 0; g < NB; ++g) {
        cs_floatx4 v = {acc[f][g][0][e] + b, acc[f][g][1][e] + b, acc[f][g][2][e] + b, acc[f][g][3][e] + b};
        if (p.relu) {
          v[0] = fmaxf(v[0], 0.0f); v[1] = fmaxf(v[1], 0.0f); v[2] = fmaxf(v[2], 0.0f); v[3] = fmaxf(v[3], 0.0f);
        }
        if (cok[g]) *reinterpret_cast<cs_floatx4*>(y + (unsigned)(yoff[g] + m * YPS)) = v;
      }
    }
}

// Persistent 1x1 variant (S1X1 only; tiles CONV_TILE_SP + 0..2): the HBM-bound 1x1 layers with a
// short K (squeeze / expand1x1: 16-64 k-steps) spent each wave's start waiting for its first loads and
// its end on stores with nothing else in flight.  Here a wave keeps its 16 MF output channels and walks
// pixel tiles ct = cs, cs + ncs, ... (ncs = resident waves / m tiles); the operand ring runs across
// tiles, so the next tile's first D k-steps are loading during this tile's last MFMAs and its stores.
// The same operands, k order and epilogue as conv_stream_kernel: bit-identical.
template <int MF, int NB, int D, int NT = 0>
__global__ __launch_bounds__(256, 2) void conv_stream1x1_persist_kernel(ConvParams p) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, rr8 = nwg & 7;
  const int wgid = (xcd < rr8 ? xcd * (q8 + 1) : rr8 * (q8 + 1) + (xcd - rr8) * q8) + (bid >> 3);
  const int gw = wgid * 4 + wave;
  const int ncs = (nwg * 4) / p.mtiles;  // host: nwg * 4 >= mtiles
  const int mt = gw % p.mtiles, cs = gw / p.mtiles;
  if (cs >= ncs || cs >= p.ntiles) return;  // wave-uniform; no barrier in this kernel
  const int m0 = mt * (16 * MF);
  const int YPS = p.y_ps;
  const int lk = lane >> 4, lj = lane & 15;
  const int ntot = (int)p.Ntot;
  // a pixel tile's per-lane input / output offsets (clamped columns re-read valid data, masked at the store)
  auto geo = [&](int ct, int (&xo)[NB], int (&yo)[NB], bool (&ok)[NB]) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < NB; ++g) {
      int col = ct * (64 * NB) + 64 * g + 4 * lj;
      ok[g] = col < ntot;
      if (!ok[g]) col = ntot - 4;
      const int img = col / YPS;
      const int pix = col - img * YPS;
      yo[g] = img * (int)p.y_nstride + pix;
      xo[g] = (img * (int)p.x_nstride + lk * p.x_ps + pix) * 4;
    }
  };
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.x), (short)0, (int)p.x_bytes, 0x00020000);
  const int kp = (p.K + 31) & ~31;
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.wp), (short)0, kp * p.Mp * 4, 0x00020000);
  const int aoff = (lk * p.Mp + m0 + MF * lj) * 4;
  const int xstep = 16 * p.x_ps, astep = 16 * p.Mp;
  const int nks = p.K >> 2;  // host: nks % D == 0, nks >= D

  float bias[MF][4];
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + MF * (4 * lk + e) + f;
      bias[f][e] = p.bias && m < p.M ? p.bias[m] : 0.0f;
    }

  cs_floatx4 acc[MF][NB][4];
  cs_floatx4 rb[D][NB];
  float ra[D][MF];
  int xoff[NB], yoff[NB];
  bool cok[NB];
  int ct = cs;
  geo(ct, xoff, yoff, cok);
#define SP_LOAD(SLOT, S, XO)                                                                      \
  {                                                                                               \
    cs_load_a<MF>(wr, aoff, (S) * astep, ra[SLOT]);                                               \
    _Pragma("unroll") for (int g = 0; g < NB; ++g) rb[SLOT][g] = __builtin_bit_cast(              \
        cs_floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, XO[g], (S) * xstep, NT ? 2 : 0));    \
  }
#define SP_MFMA(SLOT)                                                                             \
  __builtin_amdgcn_s_setprio(1);                                                                  \
  _Pragma("unroll") for (int f = 0; f < MF; ++f)                                                  \
  _Pragma("unroll") for (int g = 0; g < NB; ++g)                                                  \
  _Pragma("unroll") for (int q = 0; q < 4; ++q)                                                   \
      acc[f][g][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[SLOT][f], rb[SLOT][g][q], acc[f][g][q], 0, 0, 0); \
  __builtin_amdgcn_s_setprio(0);
#pragma unroll
  for (int d = 0; d < D; ++d) SP_LOAD(d, d, xoff);
  while (true) {
#pragma unroll
    for (int f = 0; f < MF; ++f)
#pragma unroll
      for (int g = 0; g < NB; ++g)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[f][g][q] = cs_floatx4{0.f, 0.f, 0.f, 0.f};
    const int ctn = ct + ncs;
    const bool hasn = ctn < p.ntiles;  // wave-uniform
    int xoffn[NB], yoffn[NB];
    bool cokn[NB];
    geo(hasn ? ctn : ct, xoffn, yoffn, cokn);
    for (int s0 = 0; s0 < nks - D; s0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        SP_MFMA(d);
        __builtin_amdgcn_sched_barrier(0);
        SP_LOAD(d, s0 + D + d, xoff);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // the last D k-steps; each slot refills with the next tile's k-step d
#pragma unroll
    for (int d = 0; d < D; ++d) {
      SP_MFMA(d);
      __builtin_amdgcn_sched_barrier(0);
      if (hasn) SP_LOAD(d, d, xoffn);
      __builtin_amdgcn_sched_barrier(0);
    }
    // epilogue (conv_stream_kernel's): lane (lk, lj) of fragment f holds channel m0 + MF (4 lk + e) + f,
    // pixels 4 lj + q of each group
    float* __restrict__ y = p.y;
#pragma unroll
    for (int f = 0; f < MF; ++f)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + MF * (4 * lk + e) + f;
        if (m >= p.M) continue;
        const float b = bias[f][e];
#pragma unroll
        for (int g = 0; g < NB; ++g) {
          cs_floatx4 v = {acc[f][g][0][e] + b, acc[f][g][1][e] + b, acc[f][g][2][e] + b, acc[f][g][3][e] + b};
          if (p.relu) {
            v[0] = fmaxf(v[0], 0.0f); v[1] = fmaxf(v[1], 0.0f); v[2] = fmaxf(v[2], 0.0f); v[3] = fmaxf(v[3], 0.0f);
          }
          if (cok[g]) *reinterpret_cast<cs_floatx4*>(y + (unsigned)(yoff[g] + m * YPS)) = v;
        }
      }
    if (!hasn) break;
    ct = ctn;
#pragma unroll
    for (int g = 0; g < NB; ++g) {
      xoff[g] = xoffn[g];
      yoff[g] = yoffn[g];
      cok[g] = cokn[g];
    }
  }
#undef SP_LOAD
#undef SP_MFMA
}

// bytes read before x by a 3x3 'same' conv: tap (0, 0) of output pixel 0, rounded to 16
static int stream_lead(const ConvParams& p) { return ((p.pt * p.W + p.pl) * 4 + 15) & ~15; }

// 0: not eligible, 1: S1X1, 2: STAPS
static int stream_mode(const ConvParams& p) {
  if (p.x_bytes <= 0 || !p.vec_out || p.K % 16 != 0 || p.Ntot % 4 != 0 || p.Ntot < 4) return 0;
  if (p.is1x1) {
    const uintptr_t xa = reinterpret_cast<uintptr_t>(p.x);
    return ((xa & 15) == 0 && p.x_ps % 4 == 0 && p.x_nstride % 4 == 0) ? 1 : 0;
  }
  if (p.kh != 3 || p.kw != 3 || p.sh != 1 || p.sw != 1 || p.Wo != p.W || p.W < 3 || p.pt > 1 || p.pl > 1) return 0;
  return ((reinterpret_cast<uintptr_t>(p.x) & 3) == 0 && p.x_guard >= stream_lead(p) &&
          p.x_bytes + stream_lead(p) < (1LL << 31)) ? 2 : 0;
}

static int stream_depth(int tile) {
  const int t = tile - CONV_TILE_STREAM;
  return t == 6 ? 8 : 4;
}

// the geometry allows the streaming kernel and the tile's ring depth divides the K steps; the
// persistent tiles (CONV_TILE_SP + t) run 1x1 convs only
bool conv_stream_eligible(const ConvParams& p, int tile) {
  if (tile >= CONV_TILE_SP) return stream_mode(p) == 1 && (p.K / 4) % 4 == 0 && p.K >= 16;
  return stream_mode(p) != 0 && (p.K / 4) % stream_depth(tile) == 0;
}

template <int MF, int NB, int D>
static void launch_sp(const ConvParams& p0, hipStream_t s) {
  ConvParams p = p0;
  p.mtiles = (p.M + 16 * MF - 1) / (16 * MF);
  p.ntiles = (int)((p.Ntot + 64 * NB - 1) / (64 * NB));
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ncu = v;
  }
  // resident waves (2 workgroups per CU), at least one per m tile, at most one per (m tile, pixel tile)
  const long long need = (long long)p.mtiles * p.ntiles;
  long long waves = std::min<long long>(8LL * ncu, need);
  waves = std::max<long long>(waves, p.mtiles);
  const unsigned grid = (unsigned)((waves + 3) / 4);
  if (p.mtiles == 1)  // every input element read once: non-temporal loads
    hipLaunchKernelGGL((conv_stream1x1_persist_kernel<MF, NB, D, 1>), dim3(grid), dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((conv_stream1x1_persist_kernel<MF, NB, D, 0>), dim3(grid), dim3(256), 0, s, p);
}

template <int MF, int NB, int D>
static void launch_cs(const ConvParams& p0, hipStream_t s) {
  ConvParams p = p0;
  p.x_lead = stream_lead(p);
  p.mtiles = (p.M + 16 * MF - 1) / (16 * MF);
  p.ntiles = (int)((p.Ntot + 64 * NB - 1) / (64 * NB));
  const long long waves = (long long)p.mtiles * p.ntiles;
  const dim3 grid((unsigned)((waves + 3) / 4)), block(256);
  if (stream_mode(p) == 1 && p.mtiles == 1)  // every input element read once: non-temporal loads
    hipLaunchKernelGGL((conv_stream_kernel<MF, NB, D, S1X1, 1>), grid, block, 0, s, p);
  else if (stream_mode(p) == 1)
    hipLaunchKernelGGL((conv_stream_kernel<MF, NB, D, S1X1>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((conv_stream_kernel<MF, NB, D, STAPS>), grid, block, 0, s, p);
}

// tiles CONV_TILE_STREAM + 0..8 (ConvPlan::cfg); 16 x 512 tiles (NB = 8) measured no faster
// on the 54 x 54 squeezes (tools/bench_1x1.py, profiles/r01y_bench_1x1.txt); the caller checks conv_stream_eligible
void launch_conv_stream(const ConvParams& p, int tile, hipStream_t s) {
  // (walking the pixel tiles from the last image back -- reading the producers' last-written images
  // while they are still in the Infinity Cache, as pool_conv1x1_f32_kernel does -- measured no faster
  // on the fire7 / fire8 squeezes, 85 vs 85 us, and slowed the next expand1x1, 46 -> 52 us)
  if (tile >= CONV_TILE_SP) {
    switch (tile - CONV_TILE_SP) {
      case 0: launch_sp<2, 2, 4>(p, s); break;  // 32 x 128
      case 1: launch_sp<4, 1, 4>(p, s); break;  // 64 x 64
      default: launch_sp<1, 4, 4>(p, s); break; // 16 x 256
    }
    return;
  }
  switch (tile - CONV_TILE_STREAM) {
    case 0: launch_cs<4, 2, 4>(p, s); break;   // 64 x 128
    case 1: launch_cs<2, 4, 4>(p, s); break;   // 32 x 256
    case 2: launch_cs<1, 4, 4>(p, s); break;   // 16 x 256
    case 3: launch_cs<3, 2, 4>(p, s); break;   // 48 x 128
    case 4: launch_cs<4, 1, 4>(p, s); break;   // 64 x 64
    case 5: launch_cs<8, 1, 4>(p, s); break;   // 128 x 64
    case 6: launch_cs<4, 1, 8>(p, s); break;   // 64 x 64, 8 k-steps in flight
    case 7: launch_cs<2, 2, 4>(p, s); break;   // 32 x 128
    default: launch_cs<3, 1, 4>(p, s); break;  // 48 x 64 (round 4; was 128 x 64 with 2 k-steps in flight)
  }
}

}  // namespace ore
