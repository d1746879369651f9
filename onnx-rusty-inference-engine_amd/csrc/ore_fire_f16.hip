// Fused fire module for f16 models (ORE_LOAD_F16, config 5): expand1x1 + expand3x3 (+ Relu) of the
// squeeze output S, their Concat, and the NEXT fire's squeeze1x1 (+ Relu) in one launch -- the f16
// counterpart of fire_kernel (ore_fire.hip).  The reference runs these as five separate ops
// (convolution_op.rs:422-480 per conv, concat_op.rs, relu_op.rs); the unfused f16 graph runs three
// conv_f16_kernel launches and writes / re-reads the 2 x E channel concat through HBM.
//
// Layout (NHWC f16, element (n, c, h, w) at n * nstride + (h * W + w) * cs + c):
//   * one workgroup = 256 consecutive pixels of one image (4 waves x 2 fragments x 32 pixels).
//     Its input rows (the pixels' rows +- 1, columns -1 .. W, zeros outside the image = the conv's
//     zero padding) are staged once in LDS with a pixel stride of C + 8 halves (an odd multiple of
//     16 B: the ds_read_b128 fragment reads of 32 consecutive pixels are bank-conflict free).
//   * expand weights and the squeeze weights stream from L2 as the MFMA A operand, packed by
//     launch_fire_pack_f16 as [k-step][row][16 k] (one 1 KiB contiguous block per 32-row fragment
//     and k-step) with the rows of every 32-row block PERMUTED so that accumulator element e of lane
//     half h holds channel c0 + 16 (e >> 3) + 8 h + (e & 7).  Elements 8t .. 8t + 7 of a lane are then
//     exactly the 8 consecutive channels that lane supplies as the squeeze's B operand at k-step t of
//     the chunk: the expand output goes from accumulator to squeeze operand in registers (bias,
//     Relu, one rounding to f16 -- what conv_f16_kernel stores), never through LDS or HBM.
//   * each wave owns its 64 pixels for the whole module: per 32-channel chunk of the concat (e1
//     chunks, then e3 chunks: Concat order) it runs the chunk's expand k-steps (k order (r, s, c),
//     16 k per v_mfma_f32_32x32x16_f16, as conv_f16_kernel's F16_X_NHWC_VEC chain), then feeds the
//     chunk's two 16-channel k-steps into the squeeze accumulators.  Squeeze rows are permuted the
//     same way, so the epilogue stores 8 consecutive output channels per 16-B store.
// Same operands, same k order, same MFMA instruction and the same f32 epilogue arithmetic as the
// three separate conv_f16_kernel launches: bit-identical results (tests/test_f16_gpu.py).  Skipped
// zero k-steps (the separate kernels pad K to 32) add exact zeros to a never-negative-zero sum.
#include <float.h>
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

#include "ore_kernels.h"

namespace ore {

namespace {

typedef _Float16 fh8 __attribute__((ext_vector_type(8)));
typedef float ff16 __attribute__((ext_vector_type(16)));
typedef unsigned short fu8 __attribute__((ext_vector_type(8)));

constexpr int FF_PIX = 256;  // pixels per workgroup
// the expand biases (E1 + E3 <= FF_BIAS floats) are staged in LDS once per workgroup: read from L2 per
// chunk, their latency sat between the chunk's expand MFMAs and its squeeze
constexpr int FF_BIAS = 512;

// rows of the LDS halo for a tile of FF_PIX pixels of a W-wide image with H rows (host and device)
__host__ __device__ inline int ff_halo_rows(int H, int W) {
  int r = (FF_PIX - 1) / W + 2;
  if (r > H) r = H;
  return r + 2;
}

// A-operand (weight) loads as raw buffer loads: the lane's constant byte offset in a VGPR, the
// uniform fragment / k-step offset in an SGPR -- no per-load 64-bit address VALU (a flat global
// pointer per load cost a v_lshl_add_u64 each)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ff_rsrc(const void* w) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(w), (short)0, 0x7FFFFFF0, 0x00020000);
}
__device__ __forceinline__ fh8 ld_w(__amdgpu_buffer_rsrc_t r, int vbytes, int shalves) {
  return __builtin_bit_cast(fh8, __builtin_amdgcn_raw_buffer_load_b128(r, vbytes, shalves * 2, 0));
}
__device__ __forceinline__ fh8 ld_s(const _Float16* p) { return *reinterpret_cast<const fh8*>(p); }

// Stage input rows hr0 .. hr0 + nrows - 1 (columns -1 .. W, zeros outside the image) of image x into
// the LDS halo, pixel stride PS halves, 16-B chunks.  Raw buffer loads, 8 per thread in flight: an
// offset past the image's records reads zeros, so there is no branch around a load (behind one the
// compiler waits for each load before the next).
template <int NKC, int PS>
__device__ __forceinline__ void ff_stage_halo(_Float16* halo, const _Float16* __restrict__ x, int x_cs, int H, int W,
                                              int hr0, int nrows) {
  constexpr int B = 8;
  const int W2 = W + 2, nck = nrows * W2 * (2 * NKC);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(x), (short)0, H * W * x_cs * 2, 0x00020000);
  for (int i0 = 0; i0 < nck; i0 += 256 * B) {
    fh8 v[B];
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const int i = i0 + 256 * u + (int)threadIdx.x;
      const int px = i / (2 * NKC), ck = i - px * (2 * NKC);
      const int rr = px / W2, cc = px - rr * W2;
      const int ih = hr0 + rr, iw = cc - 1;
      const bool in = i < nck && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      v[u] = __builtin_bit_cast(fh8, __builtin_amdgcn_raw_buffer_load_b128(
                                         rs, in ? ((ih * W + iw) * x_cs + ck * 8) * 2 : (int)0x80000000, 0, 0));
    }
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const int i = i0 + 256 * u + (int)threadIdx.x;
      if (i < nck) *reinterpret_cast<fh8*>(halo + (i / (2 * NKC)) * PS + (i - (i / (2 * NKC)) * (2 * NKC)) * 8) = v[u];
    }
  }
}

template <int F>
__device__ __forceinline__ void ff_zero(ff16 (&acc)[F]) {
#pragma unroll
  for (int f = 0; f < F; ++f)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[f][e] = 0.0f;
}

// One 32-channel chunk (rows c0 .. c0 + 31 of the permuted packing) of expand1x1 over F pixel
// fragments: NKC k-steps on the centre tap (hb[f] + ctr)
template <int NKC, int F>
__device__ __forceinline__ void ff_e1_chunk(ff16 (&acc)[F], __amdgpu_buffer_rsrc_t w1, int E1, int c0, int arow,
                                            const _Float16* halo, const int (&hb)[F], int ctr) {
  fh8 a[NKC];
#pragma unroll
  for (int s = 0; s < NKC; ++s) a[s] = ld_w(w1, 2 * arow, (s * E1 + c0) * 16);
  ff_zero(acc);
#pragma unroll
  for (int s = 0; s < NKC; ++s) {
    fh8 b[F];
#pragma unroll
    for (int f = 0; f < F; ++f) b[f] = ld_s(halo + hb[f] + ctr + 16 * s);
#pragma unroll
    for (int f = 0; f < F; ++f) acc[f] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[s], b[f], acc[f], 0, 0, 0);
  }
}

// One 32-channel chunk of expand3x3: 9 taps x NKC k-steps, k order (r, s, c).  B fragments BD steps
// ahead, A PD steps ahead; the scheduling barrier keeps every step's loads in it (unpinned, the
// scheduler hoists all F x 9 NKC LDS reads and spills).  One step of B prefetch left the LDS latency
// exposed behind an lgkmcnt(0) per step (2 MFMAs cover ~64 clocks).
#define ORE_FF_BD 2
#define ORE_FF_PD 8
template <int NKC, int F, int PS>
__device__ __forceinline__ void ff_e3_chunk(ff16 (&acc)[F], __amdgpu_buffer_rsrc_t w3, int E3, int c0, int arow,
                                            const _Float16* halo, const int (&hb)[F], int W2) {
  constexpr int NS3 = 9 * NKC, PD = ORE_FF_PD < NS3 ? ORE_FF_PD : NS3, BD = ORE_FF_BD;
  fh8 a[PD];
#pragma unroll
  for (int s = 0; s < PD; ++s) a[s] = ld_w(w3, 2 * arow, (s * E3 + c0) * 16);
  ff_zero(acc);
  auto boff = [&](int s) __attribute__((always_inline)) {
    const int tap = s / NKC, cs = s - tap * NKC;
    return ((tap / 3) * W2 + tap % 3) * PS + 16 * cs;
  };
  fh8 bn[BD][F];
#pragma unroll
  for (int d = 0; d < BD; ++d)
#pragma unroll
    for (int f = 0; f < F; ++f)
      if (d < NS3) bn[d][f] = ld_s(halo + hb[f] + boff(d));
#pragma unroll
  for (int s = 0; s < NS3; ++s) {
    const fh8 cur = a[s % PD];
    fh8 b[F];
#pragma unroll
    for (int f = 0; f < F; ++f) b[f] = bn[s % BD][f];
    if (s + PD < NS3) a[s % PD] = ld_w(w3, 2 * arow, ((s + PD) * E3 + c0) * 16);
    if (s + BD < NS3) {
#pragma unroll
      for (int f = 0; f < F; ++f) bn[s % BD][f] = ld_s(halo + hb[f] + boff(s + BD));
    }
#pragma unroll
    for (int f = 0; f < F; ++f) acc[f] = __builtin_amdgcn_mfma_f32_32x32x16_f16(cur, b[f], acc[f], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// this lane's 16 bias values of a chunk: channel c0 + 16 (e >> 3) + 8 h + (e & 7) for element e
__device__ __forceinline__ void ff_bias16(float (&bv)[16], const float* __restrict__ bias, int c0, int h) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const float4 u0 = *reinterpret_cast<const float4*>(bias + c0 + 16 * t + 8 * h);
    const float4 u1 = *reinterpret_cast<const float4*>(bias + c0 + 16 * t + 8 * h + 4);
    bv[8 * t + 0] = u0.x; bv[8 * t + 1] = u0.y; bv[8 * t + 2] = u0.z; bv[8 * t + 3] = u0.w;
    bv[8 * t + 4] = u1.x; bv[8 * t + 5] = u1.y; bv[8 * t + 6] = u1.z; bv[8 * t + 7] = u1.w;
  }
}

// squeeze epilogue of F pixel fragments: bias + Relu + one rounding; element 8g + e of lane half h
// = channel 32 i + 16 g + 8 h + e, one 16-B store per (fragment, g) at y + yo[f] + 32 i + 16 g
template <int MSF, int F>
__device__ __forceinline__ void ff_store_squeeze(const ff16 (&sacc)[MSF][F], const FireF16Params& p, _Float16* y,
                                                 const int (&yo)[F], const bool (&pok)[F], int h) {
#pragma unroll
  for (int i = 0; i < MSF; ++i)
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int ch = 32 * i + 16 * g + 8 * h;
      if (ch >= p.Ms) continue;
      const float4 u0 = *reinterpret_cast<const float4*>(p.bs + ch);
      const float4 u1 = *reinterpret_cast<const float4*>(p.bs + ch + 4);
      const float bv[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
      for (int f = 0; f < F; ++f) {
        if (!pok[f]) continue;
        float av[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) av[e] = sacc[i][f][8 * g + e];
        *reinterpret_cast<fh8*>(y + yo[f] + 32 * i + 16 * g) = ore_f16_epilogue8<false>(av, bv, true);
      }
    }
}

template <int NKC, int MSF>
__global__ __launch_bounds__(256, 2) void fire_f16_kernel(FireF16Params p) {
  extern __shared__ __attribute__((aligned(16))) _Float16 halo[];
  constexpr int C = 16 * NKC, PS = C + 8;  // input channels; LDS pixel stride (halves)
  const int lane = threadIdx.x & 63, lr = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = p.H, W = p.W, HW = H * W, W2 = W + 2;
  const int img = blockIdx.x / p.tiles_per_img;
  const int q0 = (blockIdx.x - img * p.tiles_per_img) * FF_PIX;
  const int qlast = min(q0 + FF_PIX - 1, HW - 1);
  const int hr0 = q0 / W - 1;  // image row of halo row 0
  ff_stage_halo<NKC, PS>(halo, static_cast<const _Float16*>(p.x) + (long long)img * p.x_nstride, p.x_cs, H, W, hr0,
                         qlast / W - q0 / W + 3);
  float* sb = reinterpret_cast<float*>(halo + ff_halo_rows(H, W) * W2 * PS);  // [E1 + E3] biases
  for (int q = threadIdx.x; q < p.E1 + p.E3; q += 256) sb[q] = q < p.E1 ? p.b1[q] : p.b3[q - p.E1];
  __syncthreads();
  if (q0 + 64 * wave >= HW) return;  // no pixel of this wave (after the only barrier)

  // this lane's two pixels: LDS offset of tap (0, 0) (its 8-channel half) and output offset
  int hb[2], yo[2];
  bool pok[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int q = q0 + 64 * wave + 32 * f + lr;
    pok[f] = q < HW;
    const int qq = pok[f] ? q : q0;
    const int hh = qq / W, ww = qq - hh * W;
    hb[f] = ((hh - hr0 - 1) * W2 + ww) * PS + 8 * h;
    yo[f] = qq * p.y_cs + 8 * h;
  }
  const int ctr = (W2 + 1) * PS;  // tap (1, 1)
  const __amdgpu_buffer_rsrc_t wsr = ff_rsrc(p.ws), w1r = ff_rsrc(p.w1), w3r = ff_rsrc(p.w3);
  const int arow = lr * 16 + 8 * h;  // this lane's 8 halves inside a [row][16] fragment block

  // MSF = 0: no squeeze -- the module writes its Concat (NHWC, pixel stride y_cs) instead (SqueezeNet
  // fire9, whose reader conv10 is no small squeeze)
  constexpr int MSA = MSF ? MSF : 1;
  ff16 sacc[MSA][2];
#pragma unroll
  for (int i = 0; i < MSF; ++i) ff_zero(sacc[i]);
  _Float16* __restrict__ yimg = static_cast<_Float16*>(p.y) + (long long)img * p.y_nstride;

  // bias + Relu + one rounding of a finished 32-channel chunk (c0 inside its conv, cat0 inside the
  // concat), then the squeeze's two k-steps over it (MSF = 0: its 16-B stores into the concat)
  auto feed = [&](const ff16 (&acc)[2], const float* __restrict__ bias, int c0, int cat0) __attribute__((always_inline)) {
    fh8 aq[2][MSA];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < MSF; ++i) aq[t][i] = ld_w(wsr, 2 * arow, ((cat0 / 16 + t) * p.Msp + 32 * i) * 16);
    float bv[16];
    ff_bias16(bv, bias, c0, h);
    fh8 bq[2][2];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        float av[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) av[e] = acc[f][8 * t + e];
        bq[t][f] = ore_f16_epilogue8<false>(av, bv + 8 * t, true);
      }
    if constexpr (MSF == 0) {
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          if (pok[f]) *reinterpret_cast<fh8*>(yimg + yo[f] + cat0 + 16 * t) = bq[t][f];
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < MSF; ++i)
#pragma unroll
        for (int f = 0; f < 2; ++f) sacc[i][f] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aq[t][i], bq[t][f], sacc[i][f], 0, 0, 0);
  };

  for (int c0 = 0; c0 < p.E1; c0 += 32) {  // expand1x1 chunks
    ff16 acc[2];
    ff_e1_chunk<NKC, 2>(acc, w1r, p.E1, c0, arow, halo, hb, ctr);
    feed(acc, sb, c0, c0);
  }
  for (int c0 = 0; c0 < p.E3; c0 += 32) {  // expand3x3 chunks
    ff16 acc[2];
    ff_e3_chunk<NKC, 2, PS>(acc, w3r, p.E3, c0, arow, halo, hb, W2);
    feed(acc, sb + p.E1, c0, p.E1 + c0);
  }
  if constexpr (MSF > 0) ff_store_squeeze<MSF, 2>(sacc, p, yimg, yo, pok, h);
}

// The pooled variant: Concat(e1, e3) -> 3x3 / stride-2 MaxPool -> squeeze.  One workgroup = a band
// of PR pooled rows of one image; it computes the conv rows that band's windows read (2 PR + 1,
// one row shared with the next band) as up to 4 waves x F fragments of 32 conv pixels.  Per 32-channel
// chunk every wave writes its conv values (bias, Relu, f16 -- what the separate conv stores) to an
// LDS conv tile [pixel][32 channels] (80-B rows); after a barrier each wave with pooled pixels takes
// one fragment of them (lane = pooled pixel), forms its 3x3 max in f32 from -FLT_MAX with the
// window's outside taps read as 0 (maxpool_nhwc_kernel's arithmetic: the separate pool's result bit
// for bit) and feeds it to the squeeze's two k-steps of the chunk; a second barrier frees the tile.
template <int NKC, int MSF, int F>
__global__ __launch_bounds__(256, 2) void fire_pool_f16_kernel(FireF16Params p) {
  extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
  constexpr int C = 16 * NKC, PS = C + 8, TS = 40;  // halo / conv tile pixel strides (halves)
  const int lane = threadIdx.x & 63, lr = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = p.H, W = p.W, W2 = W + 2, Wp = p.Wp;
  const int nbands = (p.Hp + p.PR - 1) / p.PR;
  const int img = blockIdx.x / nbands, band = blockIdx.x - img * nbands;
  const int pr0 = band * p.PR, npr = min(p.PR, p.Hp - pr0);
  const int cr0 = max(0, 2 * pr0 - p.ppt), cr1 = min(H - 1, 2 * (pr0 + npr - 1) - p.ppt + 2);
  const int ncp = (cr1 - cr0 + 1) * W;  // conv pixels of the band
  const int crmax = min(H, 2 * p.PR + 1);
  _Float16* halo = smem;
  _Float16* tile = smem + ((crmax + 2) * W2 * PS + 7) / 8 * 8;
  ff_stage_halo<NKC, PS>(halo, static_cast<const _Float16*>(p.x) + (long long)img * p.x_nstride, p.x_cs, H, W, cr0 - 1,
                         cr1 - cr0 + 3);

  // conv pixels of this wave: fragments F wave .. F wave + F - 1 (a wave with none of the band's
  // pixels skips the expand MFMAs: a short last band costs its live waves only); halo offset of
  // tap (0, 0) and conv-tile offset
  const bool clive = wave * F * 32 < ncp;
  int hb[F], tj[F];
  bool cok[F];
#pragma unroll
  for (int f = 0; f < F; ++f) {
    const int j = (wave * F + f) * 32 + lr;
    cok[f] = j < ncp;
    const int jj = cok[f] ? j : 0;
    const int rr = jj / W, cc = jj - rr * W;
    hb[f] = (rr * W2 + cc) * PS + 8 * h;
    tj[f] = jj * TS + 8 * h;
  }
  // the pooled pixel of this lane (waves with 32 w < P pooled pixels take part in the squeeze)
  const int P = npr * Wp;
  const bool wact = wave * 32 < P;
  const int k = wave * 32 + lr;
  bool pok[1] = {k < P};
  const int kk = pok[0] ? k : 0;
  const int pa = pr0 + kk / Wp, pb = kk - (kk / Wp) * Wp;
  const int ih0 = 2 * pa - p.ppt, iw0 = 2 * pb - p.ppl;
  int yo[1] = {(pa * Wp + pb) * p.y_cs + 8 * h};
  // the 3x3 window's conv-tile offsets (chunk-invariant; taps outside the image read a zero block past
  // the tile: with the max from +0 over Relu outputs that is the separate pool's skipped tap).  Nine
  // branch-free reads: behind per-tap bounds branches the compiler waited for every read in turn.
  const int zslot = crmax * W * TS;  // 32 zero halves (both 16-channel halves g, both lane halves h)
  int toff[9];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int ih = ih0 + r, iw = iw0 + s;
      const bool in = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      toff[3 * r + s] = (in ? ((ih - cr0) * W + iw) * TS : zslot) + 8 * h;
    }
  if (threadIdx.x < 4) *reinterpret_cast<fh8*>(tile + zslot + 8 * threadIdx.x) = fh8{};  // before the halo barrier
  float* sb = reinterpret_cast<float*>(tile + zslot + 32);  // [E1 + E3] biases
  for (int q = threadIdx.x; q < p.E1 + p.E3; q += 256) sb[q] = q < p.E1 ? p.b1[q] : p.b3[q - p.E1];
  const int ctr = (W2 + 1) * PS;
  const __amdgpu_buffer_rsrc_t wsr = ff_rsrc(p.ws), w1r = ff_rsrc(p.w1), w3r = ff_rsrc(p.w3);
  const int arow = lr * 16 + 8 * h;
  ff16 sacc[MSF][1];
#pragma unroll
  for (int i = 0; i < MSF; ++i) ff_zero(sacc[i]);
  __syncthreads();  // halo

  auto pool_feed = [&](const ff16 (&acc)[F], const float* __restrict__ bias, int c0, int cat0) __attribute__((always_inline)) {
    float bv[16];
    ff_bias16(bv, bias, c0, h);
#pragma unroll
    for (int f = 0; f < F; ++f) {
      if (!cok[f]) continue;
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        float av[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) av[e] = acc[f][8 * g + e];
        *reinterpret_cast<fh8*>(tile + tj[f] + 16 * g) = ore_f16_epilogue8<false>(av, bv + 8 * g, true);
      }
    }
    __syncthreads();  // conv tile of the chunk complete
    if (wact) {
      // (the A fragments loaded here, behind the barrier: hoisted ahead of the chunk's expand MFMAs
      // they measured slower, 115 -> 128 us for fire8 + pool at 16 more registers)
      fh8 aq[2][MSF];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < MSF; ++i) aq[t][i] = ld_w(wsr, 2 * arow, ((cat0 / 16 + t) * p.Msp + 32 * i) * 16);
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        // the 3x3 max (from -FLT_MAX in f32 in the separate pool, window taps outside the image read
        // as 0): after the Relu every value is +0 or positive and its f16 bits order like the value,
        // so the max is v_pk_max_u16 on the raw bits from +0 (exact; no f32 round trip)
        fu8 v[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) v[t] = __builtin_bit_cast(fu8, ld_s(tile + toff[t] + 16 * g));
        fu8 m = v[0];
#pragma unroll
        for (int t = 1; t < 9; ++t) m = __builtin_elementwise_max(m, v[t]);
        const fh8 bq = __builtin_bit_cast(fh8, m);
#pragma unroll
        for (int i = 0; i < MSF; ++i) sacc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aq[g][i], bq, sacc[i][0], 0, 0, 0);
      }
    }
    __syncthreads();  // the tile is free for the next chunk
  };

  for (int c0 = 0; c0 < p.E1; c0 += 32) {
    ff16 acc[F];
    if (clive) ff_e1_chunk<NKC, F>(acc, w1r, p.E1, c0, arow, halo, hb, ctr);
    pool_feed(acc, sb, c0, c0);
  }
  for (int c0 = 0; c0 < p.E3; c0 += 32) {
    ff16 acc[F];
    if (clive) ff_e3_chunk<NKC, F, PS>(acc, w3r, p.E3, c0, arow, halo, hb, W2);
    pool_feed(acc, sb + p.E1, c0, p.E1 + c0);
  }
  if (wact) ff_store_squeeze<MSF, 1>(sacc, p, static_cast<_Float16*>(p.y) + (long long)img * p.y_nstride, yo, pok, h);
}

// W [M][C][kh][kw] f32 (kh = kw = 1 or 3) -> [K / 16][Mp][16] f16, k = (r, s, c), rows of every
// 32-row block permuted: row R holds channel (R & ~31) + 16 (i >> 1) + 8 hh + 4 (i & 1) + j for
// R % 32 = 8 i + 4 hh + j (zero rows past M)
__global__ __launch_bounds__(256) void fire_pack_f16_kernel(const float* __restrict__ w, int M, int C, int kk, int Mp,
                                                            _Float16* __restrict__ out) {
  const int K = C * kk;
  const long long total = (long long)(K / 16) * Mp * 16;
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int k16 = (int)(t & 15);
    const long long rest = t >> 4;
    const int R = (int)(rest % Mp), js = (int)(rest / Mp);
    const int r = R & 31, i = r >> 3, hh = (r >> 2) & 1, j = r & 3;
    const int m = (R & ~31) + 16 * (i >> 1) + 8 * hh + 4 * (i & 1) + j;
    const int k = 16 * js + k16, rs = k / C, c = k - rs * C;
    out[t] = m < M ? (_Float16)w[((long long)m * C + c) * kk + rs] : (_Float16)0.0f;
  }
}

}  // namespace

int fire_f16_lds_bytes(int C, int H, int W) { return ff_halo_rows(H, W) * (W + 2) * (C + 8) * 2 + FF_BIAS * 4; }

static int fire_pool_lds_bytes(int C, int H, int W, int PR) {
  const int crmax = std::min(H, 2 * PR + 1);
  return ((crmax + 2) * (W + 2) * (C + 8) + 7) / 8 * 8 * 2 + crmax * W * 40 * 2 + 64 + FF_BIAS * 4;  // + zero block, biases
}

bool fire_pool_f16_plan(FireF16Params* p) {
  // per F (conv fragments per wave): the largest band whose conv rows fit 128 F pixels, whose pooled
  // pixels fit the 4 waves' squeeze fragments and whose halo + conv tile fit the LDS budget; the
  // shape computing the fewest 32-pixel conv fragments (+ 4 per band: staging, barriers) wins
  long long best = -1;
  for (int F = 2; F <= 4; ++F) {
    int PR = 0;
    for (int r = 1; r <= p->Hp; ++r) {
      if ((2 * r + 1) * p->W > 128 * F || r * p->Wp > 128 || fire_pool_lds_bytes(p->C, p->H, p->W, r) > FIRE_F16_LDS_MAX) break;
      PR = r;
    }
    if (PR == 0) continue;
    long long cost = 0;
    for (int pr0 = 0; pr0 < p->Hp; pr0 += PR) {
      const int npr = std::min(PR, p->Hp - pr0);
      const int cr0 = std::max(0, 2 * pr0 - p->ppt), cr1 = std::min(p->H - 1, 2 * (pr0 + npr - 1) - p->ppt + 2);
      cost += ((cr1 - cr0 + 1) * p->W + 32 * F - 1) / (32 * F) * F + 4;  // live waves x F fragments
    }
    if (best < 0 || cost < best) {
      best = cost;
      p->F = F;
      p->PR = PR;
    }
  }
  return best > 0;
}

bool fire_f16_eligible(const FireF16Params& p) {
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  const bool common = p.C % 16 == 0 && p.C >= 16 && p.C <= 64 && p.E1 % 32 == 0 && p.E3 % 32 == 0 && p.E1 > 0 &&
                      p.E1 + p.E3 <= FF_BIAS && p.E3 > 0 &&
                      (p.Ms == 0 ? !p.pool && p.y_cs >= p.E1 + p.E3  // no squeeze: the Concat is the output
                                 : p.Ms % 8 == 0 && p.Ms <= 64 && p.Msp == (p.Ms + 31) / 32 * 32 && p.y_cs >= p.Ms &&
                                       al16(p.ws) && al16(p.bs)) &&
                      p.x_cs % 8 == 0 && p.y_cs % 8 == 0 && p.x_cs >= p.C && p.x_nstride % 8 == 0 &&
                      p.y_nstride % 8 == 0 && al16(p.x) && al16(p.y) && al16(p.w1) && al16(p.w3) &&
                      al16(p.b1) && al16(p.b3) && p.H > 0 && p.W > 0 && p.N > 0 &&
                      (long long)p.H * p.W * p.x_cs < (1LL << 30) && (long long)p.H * p.W * p.y_cs < (1LL << 30);
  if (!common) return false;
  if (!p.pool) return fire_f16_lds_bytes(p.C, p.H, p.W) <= FIRE_F16_LDS_MAX;
  // pooled: 3x3 / stride 2, every window inside the padded plane and touching the image
  return p.F >= 2 && p.F <= 4 && p.PR >= 1 && p.Hp > 0 && p.Wp > 0 && p.ppt >= 0 && p.ppl >= 0 && p.ppt <= 2 &&
         p.ppl <= 2 && 2 * (p.Hp - 1) - p.ppt < p.H && 2 * (p.Wp - 1) - p.ppl < p.W && p.PR * p.Wp <= 128 &&
         (2 * p.PR + 1) * p.W <= 128 * p.F && fire_pool_lds_bytes(p.C, p.H, p.W, p.PR) <= FIRE_F16_LDS_MAX;
}

template <int NKC, int MSF>
static void launch_ff(FireF16Params p, hipStream_t s) {
  if (p.pool) {
    const unsigned lds = (unsigned)fire_pool_lds_bytes(p.C, p.H, p.W, p.PR);
    const dim3 grid((unsigned)(p.N * ((p.Hp + p.PR - 1) / p.PR)));
    switch (p.F) {
      case 2: hipLaunchKernelGGL((fire_pool_f16_kernel<NKC, MSF, 2>), grid, dim3(256), lds, s, p); break;
      case 3: hipLaunchKernelGGL((fire_pool_f16_kernel<NKC, MSF, 3>), grid, dim3(256), lds, s, p); break;
      default: hipLaunchKernelGGL((fire_pool_f16_kernel<NKC, MSF, 4>), grid, dim3(256), lds, s, p); break;
    }
    return;
  }
  p.tiles_per_img = (p.H * p.W + FF_PIX - 1) / FF_PIX;
  const unsigned lds = (unsigned)fire_f16_lds_bytes(p.C, p.H, p.W);
  hipLaunchKernelGGL((fire_f16_kernel<NKC, MSF>), dim3((unsigned)(p.N * p.tiles_per_img)), dim3(256), lds, s, p);
}

template <int NKC>
static void launch_ff_concat(FireF16Params p, hipStream_t s) {
  p.tiles_per_img = (p.H * p.W + FF_PIX - 1) / FF_PIX;
  const unsigned lds = (unsigned)fire_f16_lds_bytes(p.C, p.H, p.W);
  hipLaunchKernelGGL((fire_f16_kernel<NKC, 0>), dim3((unsigned)(p.N * p.tiles_per_img)), dim3(256), lds, s, p);
}

void launch_fire_f16(const FireF16Params& p, hipStream_t s) {
  if (p.Ms == 0) {  // the module without a squeeze: expands + Concat in one launch
    switch (p.C / 16) {
      case 1: launch_ff_concat<1>(p, s); break;
      case 2: launch_ff_concat<2>(p, s); break;
      case 3: launch_ff_concat<3>(p, s); break;
      default: launch_ff_concat<4>(p, s); break;
    }
    return;
  }
  const int msf = (p.Ms + 31) / 32;
  switch (p.C / 16 * 2 + msf - 1) {
    case 2: launch_ff<1, 1>(p, s); break;
    case 3: launch_ff<1, 2>(p, s); break;
    case 4: launch_ff<2, 1>(p, s); break;
    case 5: launch_ff<2, 2>(p, s); break;
    case 6: launch_ff<3, 1>(p, s); break;
    case 7: launch_ff<3, 2>(p, s); break;
    case 8: launch_ff<4, 1>(p, s); break;
    default: launch_ff<4, 2>(p, s); break;
  }
}

size_t fire_pack_f16_bytes(int M, int C, int kk) { return size_t(C * kk / 16) * size_t((M + 31) / 32 * 32) * 16 * 2; }

void launch_fire_pack_f16(const float* w, int M, int C, int kk, void* out, hipStream_t s) {
  const int Mp = (M + 31) / 32 * 32;
  const long long total = (long long)(C * kk / 16) * Mp * 16;
  long long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(fire_pack_f16_kernel, dim3((unsigned)blocks), dim3(256), 0, s, w, M, C, kk, Mp,
                     static_cast<_Float16*>(out));
}

}  // namespace ore
