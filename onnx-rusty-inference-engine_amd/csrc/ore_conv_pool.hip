// Conv (stride 2, no padding) + Relu + MaxPool 3x3 / stride 2 / no padding in one launch: SqueezeNet's
// conv1 -> relu_conv1 -> pool1 (convolution_op.rs:94-517, relu_op.rs:31-33, max_pool_op.rs:157-360).
//
// Why a second pooled-conv kernel.  conv_gemm_kernel's pooled epilogue (ore_conv.hip) gives each block
// a 13 x 19 conv-output patch for a 6 x 9 pooled tile: the patch borders are recomputed by the
// neighbouring tiles (247 conv outputs per 216 needed) and the LDS-staged main loop runs ~100 TF/s.
// Here a block owns (image, 16 MF output channels) and WALKS the conv output plane row-major, 64 quads
// of 4 consecutive output columns per step (4 waves x 16 lanes), so no conv output is computed twice
// (only the 3 columns that pad a 109-wide row to 28 quads); the pooled rows live in an LDS ring.
//
// Main loop (as conv_stream_kernel, ore_conv_stream.hip): LDS-free implicit GEMM on
// v_mfma_f32_16x16x4_f32, k = (c, r, s) in the reference's order, lane (lk, lj) supplies k = 4 t + lk
// for the quad of lane lj.  With stride 2 the quad's four inputs of a tap are elements 0, 2, 4, 6 of an
// 8-float run: one 16-B + one 12-B load, element q feeding the q-th of four MFMAs.  The tap offset
// c x_ps + r W + s advances by 4 k per step (carries, no table).  Taps k >= K read past the buffer
// (0), against zero weights.  The operand ring runs ACROSS the block's steps: the next step's first
// k-steps are in flight while the epilogue of this one pools.
//
// Pooled epilogue without recomputation: after bias + Relu every conv output is >= +0, so its f32 bit
// pattern orders like the value and the 3x3 max is an LDS ds_max_u32 into the pooled cell (exact, any
// order; the ring starts at +0 = max(-FLT_MAX, values >= 0), the reference's start value,
// max_pool_op.rs:337).  A quad (4 columns 4qx..4qx+3 of conv row oy) contributes
//   max(v0, v1, v2) -> pooled column 2qx, max(v2, v3) -> 2qx + 1, v0 -> 2qx - 1,
// to pooled row oy / 2 and, for an even oy, also oy / 2 - 1.  After each step the block barrier
// publishes the maxima and the pooled rows whose three conv rows are done are stored and their ring
// slot cleared.  Every pooled output is the max of the same nine values as in the unfused graph, and
// each conv output is the same k-ordered MFMA chain + bias as conv_gemm_kernel's: bit-identical.
#include <hip/hip_runtime.h>

#include <atomic>

#include <algorithm>
#include <vector>

#include "ore_kernels.h"

namespace ore {

typedef float cp_floatx4 __attribute__((ext_vector_type(4)));
typedef float cp_floatx3 __attribute__((ext_vector_type(3)));

// pooled rows held in LDS (nring slots, pooled row py in slot py % nring): enough that the rows live
// during a step never share a slot AND a slot cleared after a step is not touched by the next one (no
// barrier separates the two).  Two consecutive steps of S quads span G2 = (qrow + 2 S - 2) / qrow conv
// rows at most; nring = (G2 + 4) / 2 covers both, checked by simulation over widths 6..229 and heights
// 5..229 for S = 64 and 128 (4 / 7 slots for a 28-quad row).
static int cp_nring(int qrow, int S) { return ((qrow + 2 * S - 2) / qrow + 4) / 2; }

template <int MF>
__device__ __forceinline__ void cp_load_a(__amdgpu_buffer_rsrc_t r, int voff, int soff, float (&a)[MF]) {
  if constexpr (MF == 6) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const cp_floatx4 v = __builtin_bit_cast(cp_floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
    const f2 w = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(r, voff + 16, soff, 0));
    a[0] = v[0]; a[1] = v[1]; a[2] = v[2]; a[3] = v[3]; a[4] = w[0]; a[5] = w[1];
  } else if constexpr (MF == 4) {
    const cp_floatx4 v = __builtin_bit_cast(cp_floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
    a[0] = v[0]; a[1] = v[1]; a[2] = v[2]; a[3] = v[3];
  } else if constexpr (MF == 3) {
    const cp_floatx3 v = __builtin_bit_cast(cp_floatx3, __builtin_amdgcn_raw_buffer_load_b96(r, voff, soff, 0));
    a[0] = v[0]; a[1] = v[1]; a[2] = v[2];
  } else {
    static_assert(MF == 2, "MF");
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 v = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
    a[0] = v[0]; a[1] = v[1];
  }
}

// operand modes: CP_S2 = stride-2 'valid' conv (kw >= 4; conv1), CP_1X1 = 1x1 stride 1, CP_T3 = 3x3
// stride 1 'same' (pads <= 1; taps outside the image zeroed per element from a per-pixel tap mask, as
// conv_stream_kernel's STAPS mode) -- the last two are SqueezeNet's expand convs ahead of pool3 / pool5
enum { CP_S2 = 0, CP_1X1 = 1, CP_T3 = 2 };
constexpr int CP_D = 4;  // k-steps in flight

// MF: 16-channel fragments per block (every wave computes all 16 MF channels of its 16 quads);
// D: k-steps in flight; NW: waves per block.  qrow = quads per conv row, nsteps = 16 NW-quad steps per
// image.
template <int MF, int D, int NW, int MODE>
__global__ __launch_bounds__(64 * NW, 8 / NW) void conv_pool_stream_kernel(ConvParams p, int qrow, int nbands, int nring) {
  extern __shared__ unsigned cp_lds[];  // [nring][16 MF][Wp] pooled maxima (f32 bits)
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lk = lane >> 4, lj = lane & 15;
  // XCD-aware bijective remap: the m tiles of one image (same input rows) share an XCD's L2
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, rr8 = nwg & 7;
  const int wgid = (xcd < rr8 ? xcd * (q8 + 1) : rr8 * (q8 + 1) + (xcd - rr8) * q8) + (bid >> 3);
  // block = (image, band of pooled rows, m tile); the m tiles of one band are adjacent
  const int ib = wgid / p.mtiles, mt = wgid - ib * p.mtiles;
  const int img = ib / nbands, band = ib - img * nbands;
  const int m0 = mt * (16 * MF);
  const int Wp = p.ep_Wo, Hp = p.ep_Ho;
  constexpr int CH = 16 * MF;
  const int slot = CH * Wp;

  for (int i = tid; i < nring * slot; i += 64 * NW) cp_lds[i] = 0u;
  // CP_T3: per k = 4 t + lk of a step, {c x_ps + r W + s (-1 past K), tap 3 r + s} behind the ring
  int2* tap_tab = reinterpret_cast<int2*>(cp_lds + nring * slot);
  if constexpr (MODE == CP_T3) {
    for (int k = tid; k < 4 * ((p.K + 3) >> 2); k += 64 * NW) {
      const int c = k / 9, t9 = k - 9 * c;
      tap_tab[k] = int2{c < p.C ? c * p.x_ps + (t9 / 3) * p.W + t9 % 3 : -1, t9};
    }
  }

  // band: pooled rows [py0, py1) from conv rows 2 py0 .. 2 py1 (the band's last pooled row reads
  // row 2 py1, which the next band recomputes as its first: one conv row per band boundary)
  const int pb = (Hp + nbands - 1) / nbands;
  const int py0 = band * pb, py1 = py0 + pb < Hp ? py0 + pb : Hp;
  const int q0 = 2 * py0 * qrow;
  const int nq = (2 * py1 + 1 < p.Ho ? 2 * py1 + 1 : p.Ho) * qrow;  // quads [q0, nq) of this band
  const bool colpad = 2 * (Wp - 1) + 2 >= p.Wo;  // a pooled window reaches a quad-padding column
  const int nsteps = py0 < py1 ? (nq - q0 + 16 * NW - 1) / (16 * NW) : 0;
  // CP_T3: the resource starts x_lead bytes before x so that no tap offset is negative (a negative
  // offset would zero the whole 16-B access, valid elements included); those bytes are masked taps
  const int xlead = MODE == CP_T3 ? p.x_lead : 0;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(reinterpret_cast<const char*>(p.x) - xlead), (short)0, (int)p.x_bytes + xlead, 0x00020000);
  const int kp = (p.K + 31) & ~31;
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.wp), (short)0, kp * p.Mp * 4, 0x00020000);
  const int aoff = (lk * p.Mp + m0 + MF * lj) * 4;  // bytes; + 16 t Mp per k-step
  const int astep = 16 * p.Mp;
  const int nks = (p.K + 3) >> 2;
  const int ximg = img * (int)p.x_nstride;

  // bias of this lane's channels m0 + MF (4 lk + e) + f
  float bias[MF][4];
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + MF * (4 * lk + e) + f;
      bias[f][e] = (p.bias && m < p.M) ? p.bias[m] : 0.0f;
    }

  // loader: step ls (wave-uniform), k-step lt, this lane's quad base and tap (c, r, s) of k = 4 lt + lk
  int ls = 0, lt = 0;
  // CP_S2: tap (lc, lr, lsx), offset loff; CP_1X1: channel lc, offset loff = lc x_ps; CP_T3: tap
  // tt = 3 r + s of channel lc, channel offset loff = lc x_ps
  int lc = MODE == CP_1X1 ? lk : 0, lr = 0, lsx = lk, loff = MODE == CP_S2 ? lk : MODE == CP_1X1 ? lk * p.x_ps : 0;
  int tt = lk;
  // CP_T3: bit 3 r + s = tap (r, s) of pixel q inside the image; the loader's copy (tmask, written
  // when it moves to the next step's quad, D k-steps ahead) and the consumer's (tmc, taken over at
  // the step's epilogue)
  unsigned tmask[4] = {0u, 0u, 0u, 0u}, tmc[4] = {0u, 0u, 0u, 0u};
  auto quad_base = [&](int st) -> int {
    int qd = q0 + st * (16 * NW) + wave * 16 + lj;
    if (qd >= nq) qd = nq - 1;  // surplus lanes of the last step re-read a valid quad (not pooled)
    const int oy = qd / qrow, qx = qd - oy * qrow;
    if constexpr (MODE == CP_S2) return ximg + 2 * oy * p.W + 8 * qx;  // input (2 oy, 2 (4 qx))
    if constexpr (MODE == CP_1X1) return ximg + oy * p.W + 4 * qx;
    // CP_T3: element of tap (0, 0) relative to the resource start
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ow = 4 * qx + q;
      unsigned cm = 0, m = 0;
#pragma unroll
      for (int c3 = 0; c3 < 3; ++c3) cm |= ((unsigned)(ow - p.pl + c3) < (unsigned)p.W ? 1u : 0u) << c3;
#pragma unroll
      for (int r3 = 0; r3 < 3; ++r3)
        if ((unsigned)(oy - p.pt + r3) < (unsigned)p.H) m |= cm << (3 * r3);
      tmask[q] = m;
    }
    return (xlead >> 2) + ximg + (oy - p.pt) * p.W + 4 * qx - p.pl;
  };
  int lbase = quad_base(0);
#pragma unroll
  for (int q = 0; q < 4; ++q) tmc[q] = tmask[q];

  cp_floatx4 acc[MF][4];
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[f][q] = cp_floatx4{0.f, 0.f, 0.f, 0.f};
  float ra[D][MF];
  cp_floatx4 rb0[D];
  cp_floatx3 rb1[MODE == CP_S2 ? D : 1];
  int rt[MODE == CP_T3 ? D : 1];  // CP_T3: the tap of each ring slot's k (for its zero mask)

#define CP_LOAD_B1(SLOT) \
  rb1[SLOT] = __builtin_bit_cast(cp_floatx3, __builtin_amdgcn_raw_buffer_load_b96(xr, o_ + 16, 0, 0));
#define CP_LOAD(SLOT)                                                                                  \
  {                                                                                                    \
    cp_load_a<MF>(wr, aoff, lt * astep, ra[SLOT]);                                                     \
    if constexpr (MODE == CP_S2) {                                                                     \
      const int o_ = lc < p.C ? (lbase + loff) * 4 : 0x7ff00000; /* k >= K: past the buffer -> 0 */    \
      rb0[SLOT] = __builtin_bit_cast(cp_floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, o_, 0, 0)); \
      CP_LOAD_B1(SLOT)                                                                                 \
      lsx += 4; loff += 4;                                                                             \
      if (lsx >= p.kw) {                                                                               \
        lsx -= p.kw; loff += p.W - p.kw; ++lr;                                                         \
        if (lr >= p.kh) { lr = 0; loff += p.x_ps - p.kh * p.W; ++lc; }                                 \
      }                                                                                                \
    } else if constexpr (MODE == CP_1X1) {                                                             \
      const int o_ = lc < p.C ? (lbase + loff) * 4 : 0x7ff00000;                                       \
      rb0[SLOT] = __builtin_bit_cast(cp_floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, o_, 0, 0)); \
      lc += 4; loff += 4 * p.x_ps;                                                                     \
    } else {                                                                                           \
      /* the k-step's (tap offset, tap) from the block's LDS table: the same every step */            \
      const int2 e_ = tap_tab[4 * lt + lk];                                                            \
      const int o_ = e_.x >= 0 ? (lbase + e_.x) * 4 : 0x7ff00000;                                      \
      rb0[SLOT] = __builtin_bit_cast(cp_floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, o_, 0, 0)); \
      rt[SLOT] = e_.y;                                                                                 \
    }                                                                                                  \
    if (++lt == nks) {                                                                                 \
      lt = 0; lr = 0; lsx = lk; tt = lk;                                                               \
      lc = MODE == CP_1X1 ? lk : 0;                                                                    \
      loff = MODE == CP_S2 ? lk : MODE == CP_1X1 ? lk * p.x_ps : 0;                                    \
      if (++ls < nsteps) lbase = quad_base(ls);                                                        \
    }                                                                                                  \
  }
#define CP_MFMA(SLOT)                                                                                  \
  if constexpr (MODE == CP_T3) { /* zero the taps outside the image (the reference's zero padding) */  \
    const int4 v_ = __builtin_bit_cast(int4, rb0[SLOT]);                                               \
    int4 w_;                                                                                           \
    w_.x = v_.x & __builtin_amdgcn_sbfe((int)tmc[0], rt[SLOT], 1);                                     \
    w_.y = v_.y & __builtin_amdgcn_sbfe((int)tmc[1], rt[SLOT], 1);                                     \
    w_.z = v_.z & __builtin_amdgcn_sbfe((int)tmc[2], rt[SLOT], 1);                                     \
    w_.w = v_.w & __builtin_amdgcn_sbfe((int)tmc[3], rt[SLOT], 1);                                     \
    rb0[SLOT] = __builtin_bit_cast(cp_floatx4, w_);                                                    \
  }                                                                                                    \
  __builtin_amdgcn_s_setprio(1);                                                                       \
  _Pragma("unroll") for (int f = 0; f < MF; ++f) {                                                     \
    if constexpr (MODE == CP_S2) {                                                                     \
      acc[f][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[SLOT][f], rb0[SLOT][0], acc[f][0], 0, 0, 0); \
      acc[f][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[SLOT][f], rb0[SLOT][2], acc[f][1], 0, 0, 0); \
      acc[f][2] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[SLOT][f], rb1[SLOT][0], acc[f][2], 0, 0, 0); \
      acc[f][3] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[SLOT][f], rb1[SLOT][2], acc[f][3], 0, 0, 0); \
    } else {                                                                                           \
      _Pragma("unroll") for (int q = 0; q < 4; ++q)                                                    \
        acc[f][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[SLOT][f], rb0[SLOT][q], acc[f][q], 0, 0, 0); \
    }                                                                                                  \
  }                                                                                                    \
  __builtin_amdgcn_s_setprio(0);

  __syncthreads();  // the ring is zero before the first ds_max
  const int total = nsteps * nks;
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (d < total) CP_LOAD(d);
  int ct = 0, cs = 0, py_next = py0;  // consumer k-step / step, first pooled row not yet stored
  // epilogue of step cs (once per step): bias + Relu, 3x3 maxima into the LDS ring, barrier, stores
  auto cp_epilogue = [&]() {
          // ---- epilogue of step cs: bias + Relu, 3x3 maxima into the LDS ring ----
          int qd = q0 + cs * (16 * NW) + wave * 16 + lj;
          const bool qv = qd < nq;
          if (!qv) qd = nq - 1;
          const int oy = qd / qrow, qx = qd - oy * qrow;
          const int pya = oy >> 1;                                 // top (even oy) / middle (odd oy) row
          const int pyb = ((oy & 1) == 0 && oy >= 2) ? pya - 1 : -1;  // bottom row (even oy)
          const int px0 = 2 * qx;
          // right: lane lj + 1 holds quad qd + 1 of this conv row (its column 4qx + 4 is folded into c1);
          // left: column 4qx still has to reach pooled column 2qx - 1 itself (no left lane folded it)
          const bool right = lj < 15 && qx < qrow - 1;
          const bool left = qx > 0 && lj == 0;
          const bool oka = qv && pya >= py0 && pya < py1, okb = qv && pyb >= py0 && pyb < py1;
          const int sa = (pya % nring) * slot, sb = (pyb < 0 ? 0 : pyb % nring) * slot;
#pragma unroll
          for (int f = 0; f < MF; ++f)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int cl = MF * (4 * lk + e) + f;
              float v[4];
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const float t = acc[f][q][e] + bias[f][e];
                v[q] = t > 0.0f ? t : 0.0f;  // Relu, canonical +0
              }
              if (colpad) {  // columns >= Wo (the quad padding) read by a window: the pool's zero padding
#pragma unroll
                for (int q = 0; q < 4; ++q)
                  if (px0 * 2 + q >= p.Wo) v[q] = 0.0f;
              }
              const unsigned c0 = __float_as_uint(fmaxf(fmaxf(v[0], v[1]), v[2]));
              const unsigned c2 = __float_as_uint(v[0]);
              // pooled column 2qx + 1 also takes the right neighbour quad's first column: lane lj + 1
              // (DPP row_shl:1 within the 16-lane row) when that quad continues this conv row
              const unsigned nb = (unsigned)__builtin_amdgcn_update_dpp((int)c2, (int)c2, 0x101, 0xf, 0xf, false);
              const unsigned c1 = __float_as_uint(fmaxf(v[2], v[3])) > nb || !right ? __float_as_uint(fmaxf(v[2], v[3]))
                                                                                  : nb;
              if (oka) {
                unsigned* row = cp_lds + sa + cl * Wp;
                if (px0 < Wp) atomicMax(row + px0, c0);
                if (px0 + 1 < Wp) atomicMax(row + px0 + 1, c1);
                if (left && px0 - 1 < Wp) atomicMax(row + px0 - 1, c2);
              }
              if (okb) {
                unsigned* row = cp_lds + sb + cl * Wp;
                if (px0 < Wp) atomicMax(row + px0, c0);
                if (px0 + 1 < Wp) atomicMax(row + px0 + 1, c1);
                if (left && px0 - 1 < Wp) atomicMax(row + px0 - 1, c2);
              }
            }
#pragma unroll
          for (int f = 0; f < MF; ++f)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[f][q] = cp_floatx4{0.f, 0.f, 0.f, 0.f};
          __syncthreads();
          // ---- store the pooled rows whose conv rows 2py .. 2py + 2 are all done ----
          const int qend = q0 + (cs + 1) * (16 * NW) < nq ? q0 + (cs + 1) * (16 * NW) : nq;
          const int rows_done = qend / qrow;
          int py_end = qend == nq ? py1 : (rows_done >= 3 ? ((rows_done - 3) >> 1) + 1 : 0);
          if (py_end > py1) py_end = py1;
          for (int py = py_next; py < py_end; ++py) {
            unsigned* src = cp_lds + (py % nring) * slot;
            float* dst = p.y + (long long)img * p.y_nstride + (long long)m0 * p.y_ps + py * Wp;
            // lane -> pooled column, wave -> channel (a 216-B run per channel row; no division)
            for (int px = lane; px < Wp; px += 64)
              for (int cl = wave; cl < CH; cl += NW) {
                if (m0 + cl < p.M) dst[cl * p.y_ps + px] = __uint_as_float(src[cl * Wp + px]);
                src[cl * Wp + px] = 0u;
              }
          }
          if (py_end > py_next) py_next = py_end;
#pragma unroll
    for (int q_ = 0; q_ < 4; ++q_) tmc[q_] = tmask[q_];
    ++cs;
  };
  if constexpr (MODE != CP_S2) {
    // stride-1 modes (host: nks % D == 0): the ring-slot pattern repeats every step, so the epilogue
    // follows the step's k-steps once in the code (conv1's 37 k-steps keep the rolling form below)
    for (int g0 = 0; g0 < total; g0 += nks) {
      for (int s0 = 0; s0 < nks; s0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
          CP_MFMA(d);
          __builtin_amdgcn_sched_barrier(0);
          if (g0 + s0 + d + D < total) CP_LOAD(d);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      cp_epilogue();
    }
  } else {
  for (int g0 = 0; g0 < total; g0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      if (g0 + d < total) {
        CP_MFMA(d);
        __builtin_amdgcn_sched_barrier(0);
        if (g0 + d + D < total) CP_LOAD(d);
        __builtin_amdgcn_sched_barrier(0);
        if (++ct == nks) {
          ct = 0;
          cp_epilogue();
        }
      }
    }
  }
  }
#undef CP_LOAD
#undef CP_MFMA
}

// variants (ConvParams::ep_variant): 2 = 48 channels x 64 quads per block (4 waves), 3 = 96 channels
// x 128 quads (8 waves: twice the MFMAs per operand load, one block per CU), 4 = 64 channels x 64
// quads (4 waves), 5 = variant 4 over 3 bands of pooled rows per image (3x the blocks).  (Variant 6,
// 96 x 64 over 2 bands with a second barrier per step, two blocks per CU, measured slower inside the
// graph -- 963 vs 913 us on conv1 + pool1, profiles/r01zg_conv1_walk96_b2.txt -- and is retired.)
static void cp_shape(int variant, int M, int* mf, int* nw) {
  *mf = variant == 3 ? 6 : (variant == 4 || variant == 5) ? 4 : (M > 32 ? 3 : 2);
  *nw = variant == 3 ? 8 : 4;
}
static int cp_bands(int variant) { return variant == 5 ? 3 : 1; }
static int cp_ring(const ConvParams& p, int variant) {
  int mf, nw;
  cp_shape(variant, p.M, &mf, &nw);
  const int qrow = (p.Wo + 3) / 4;
  return cp_nring(qrow, 16 * nw);
}
static int cp_mode(const ConvParams& p);
static size_t cp_lds_bytes(const ConvParams& p, int variant) {
  int mf, nw;
  cp_shape(variant, p.M, &mf, &nw);
  const size_t tab = cp_mode(p) == CP_T3 ? size_t(4 * ((p.K + 3) / 4)) * 8 : 0;  // the T3 tap table
  return size_t(cp_ring(p, variant)) * 16 * mf * p.ep_Wo * 4 + tab;
}
static int cp_lead(const ConvParams& p) { return ((p.pt * p.W + p.pl) * 4 + 15) & ~15; }

// -1: not eligible, else the operand mode
static int cp_mode(const ConvParams& p) {
  if (!p.relu || p.x_bytes <= 0 || (reinterpret_cast<uintptr_t>(p.x) & 3) != 0) return -1;
  // pooled windows start inside the conv plane; a window may reach one row / column past it (the
  // pool's bottom / right zero padding: neutral after the Relu)
  if (p.ep_pt != 0 || p.ep_pl != 0 || p.ep_Ho < 1 || p.ep_Wo < 1) return -1;
  if (2 * (p.ep_Ho - 1) + 2 > p.Ho || 2 * (p.ep_Wo - 1) + 2 > p.Wo) return -1;
  if (p.sh == 2 && p.sw == 2 && p.pt == 0 && p.pl == 0 && p.kw >= 4 && p.kh >= 1 && 2 * (p.Ho - 1) + p.kh <= p.H &&
      2 * (p.Wo - 1) + p.kw <= p.W)
    return CP_S2;
  if (p.kh == 1 && p.kw == 1 && p.sh == 1 && p.sw == 1 && p.pt == 0 && p.pl == 0 && p.Ho == p.H && p.Wo == p.W &&
      p.C % (4 * CP_D) == 0)
    return CP_1X1;
  if (p.kh == 3 && p.kw == 3 && p.sh == 1 && p.sw == 1 && p.pt <= 1 && p.pl <= 1 && p.Wo == p.W && p.Ho == p.H &&
      p.W >= 3 && p.x_guard >= cp_lead(p) && p.x_bytes + cp_lead(p) < (1LL << 31) && (9 * p.C) % (4 * CP_D) == 0)
    return CP_T3;
  return -1;
}

bool conv_pool_stream_eligible(const ConvParams& p, int variant) {
  if (variant < 2 || variant > 5 || cp_mode(p) < 0) return false;
  if (variant == 3 && (p.M < 64 || cp_mode(p) != CP_S2)) return false;  // idle rows / spills
  if ((variant == 4 || variant == 5) && p.M < 48) return false;
  if (variant == 5 && p.ep_Ho < 6) return false;
  return cp_lds_bytes(p, variant) <= size_t(variant == 3 ? 152 : 78) * 1024;
}

template <int MF, int D, int NW, int MODE>
static void launch_cp(const ConvParams& p0, size_t lds, int nbands, int nring, hipStream_t s) {
  ConvParams p = p0;
  p.mtiles = (p.M + 16 * MF - 1) / (16 * MF);
  p.x_lead = MODE == CP_T3 ? cp_lead(p) : 0;
  const int qrow = (p.Wo + 3) / 4;
  if (lds > 64 * 1024) {
    // above the default dynamic-LDS limit: raise it once per DEVICE and instantiation (the
    // attribute binds to the current device; one ore_ctx per device may call from its own thread)
    static std::atomic<unsigned long long> raised{0};
    ore_raise_lds_once(raised, reinterpret_cast<const void*>(&conv_pool_stream_kernel<MF, D, NW, MODE>), 160 * 1024);
  }
  hipLaunchKernelGGL((conv_pool_stream_kernel<MF, D, NW, MODE>), dim3((unsigned)(p.N * nbands * p.mtiles)),
                     dim3(64 * NW), lds, s, p, qrow, nbands, nring);
}

template <int MF, int NW>
static void launch_cp_mode(const ConvParams& p, size_t lds, int nbands, int nring, hipStream_t s) {
  if constexpr (MF == 6) {  // the 96-channel tiles: conv1 only (the stride-1 modes would spill)
    launch_cp<MF, CP_D, NW, CP_S2>(p, lds, nbands, nring, s);
  } else {
    switch (cp_mode(p)) {
      case CP_S2: launch_cp<MF, CP_D, NW, CP_S2>(p, lds, nbands, nring, s); break;
      case CP_1X1: launch_cp<MF, CP_D, NW, CP_1X1>(p, lds, nbands, nring, s); break;
      default: launch_cp<MF, CP_D, NW, CP_T3>(p, lds, nbands, nring, s); break;
    }
  }
}

void launch_conv_pool_stream(const ConvParams& p, int variant, hipStream_t s) {
  int mf, nw;
  cp_shape(variant, p.M, &mf, &nw);
  const size_t lds = cp_lds_bytes(p, variant);
  const int nb = cp_bands(variant), nr = cp_ring(p, variant);
  if (variant == 3)
    launch_cp_mode<6, 8>(p, lds, nb, nr, s);
  else if (variant == 4 || variant == 5)
    launch_cp_mode<4, 4>(p, lds, nb, nr, s);
  else if (mf == 3)
    launch_cp_mode<3, 4>(p, lds, nb, nr, s);
  else
    launch_cp_mode<2, 4>(p, lds, nb, nr, s);
}

}  // namespace ore
