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
#include <hip/hip_runtime.h>

#include "ore_kernels.h"

namespace ore {

namespace {

typedef _Float16 fh8 __attribute__((ext_vector_type(8)));
typedef float ff16 __attribute__((ext_vector_type(16)));

constexpr int FF_PIX = 256;  // pixels per workgroup

// rows of the LDS halo for a tile of FF_PIX pixels of a W-wide image with H rows (host and device)
__host__ __device__ inline int ff_halo_rows(int H, int W) {
  int r = (FF_PIX - 1) / W + 2;
  if (r > H) r = H;
  return r + 2;
}

__device__ __forceinline__ fh8 ld_g(const _Float16* p) { return *reinterpret_cast<const fh8*>(p); }
__device__ __forceinline__ fh8 ld_s(const _Float16* p) { return *reinterpret_cast<const fh8*>(p); }

template <int NKC, int MSF>
__global__ __launch_bounds__(256, 2) void fire_f16_kernel(FireF16Params p) {
  extern __shared__ __attribute__((aligned(16))) _Float16 halo[];
  constexpr int C = 16 * NKC, PS = C + 8;  // input channels; LDS pixel stride (halves)
  constexpr int NS3 = 9 * NKC;             // expand3x3 k-steps
  constexpr int PD = 6;                    // expand3x3 A-operand loads in flight
  const int tid = threadIdx.x, lane = tid & 63, lr = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.H, W = p.W, HW = H * W, W2 = W + 2;
  const int img = blockIdx.x / p.tiles_per_img;
  const int q0 = (blockIdx.x - img * p.tiles_per_img) * FF_PIX;
  const int qlast = min(q0 + FF_PIX - 1, HW - 1);
  const int hr0 = q0 / W - 1;                        // image row of halo row 0
  const int nrows = qlast / W - q0 / W + 3;
  const _Float16* __restrict__ x = static_cast<const _Float16*>(p.x) + (long long)img * p.x_nstride;

  // stage the halo: nrows x (W + 2) pixels x C channels, 16-B chunks
  {
    const int nck = nrows * W2 * (2 * NKC);
    for (int i = tid; i < nck; i += 256) {
      const int px = i / (2 * NKC), ck = i - px * (2 * NKC);
      const int rr = px / W2, cc = px - rr * W2;
      const int ih = hr0 + rr, iw = cc - 1;
      fh8 v = {};
      if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) v = ld_g(x + (ih * W + iw) * p.x_cs + ck * 8);
      *reinterpret_cast<fh8*>(halo + px * PS + ck * 8) = v;
    }
  }
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
  const _Float16* __restrict__ w1 = static_cast<const _Float16*>(p.w1);
  const _Float16* __restrict__ w3 = static_cast<const _Float16*>(p.w3);
  const _Float16* __restrict__ ws = static_cast<const _Float16*>(p.ws);
  const int E1 = p.E1, E3 = p.E3, Msp = p.Msp;
  const int arow = lr * 16 + 8 * h;  // this lane's 8 halves inside a [row][16] fragment block

  ff16 sacc[MSF][2];
#pragma unroll
  for (int i = 0; i < MSF; ++i)
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int e = 0; e < 16; ++e) sacc[i][f][e] = 0.0f;

  // bias + Relu + one rounding of a finished 32-channel chunk (c0 inside its conv, cat0 inside the
  // concat), then the squeeze's two k-steps over it
  auto feed = [&](const ff16 (&acc)[2], const float* __restrict__ bias, int c0, int cat0) __attribute__((always_inline)) {
    fh8 aq[2][MSF];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < MSF; ++i) aq[t][i] = ld_g(ws + ((cat0 / 16 + t) * Msp + 32 * i) * 16 + arow);
    float bv[16];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const float4 u0 = *reinterpret_cast<const float4*>(bias + c0 + 16 * t + 8 * h);
      const float4 u1 = *reinterpret_cast<const float4*>(bias + c0 + 16 * t + 8 * h + 4);
      bv[8 * t + 0] = u0.x; bv[8 * t + 1] = u0.y; bv[8 * t + 2] = u0.z; bv[8 * t + 3] = u0.w;
      bv[8 * t + 4] = u1.x; bv[8 * t + 5] = u1.y; bv[8 * t + 6] = u1.z; bv[8 * t + 7] = u1.w;
    }
    fh8 bq[2][2];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int e = 0; e < 16; ++e) bq[e >> 3][f][e & 7] = (_Float16)fmaxf(acc[f][e] + bv[e], 0.0f);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < MSF; ++i)
#pragma unroll
        for (int f = 0; f < 2; ++f) sacc[i][f] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aq[t][i], bq[t][f], sacc[i][f], 0, 0, 0);
  };

  // expand1x1 chunks: NKC k-steps on the centre tap
  for (int c0 = 0; c0 < E1; c0 += 32) {
    fh8 a[NKC];
#pragma unroll
    for (int s = 0; s < NKC; ++s) a[s] = ld_g(w1 + (s * E1 + c0) * 16 + arow);
    ff16 acc[2];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[f][e] = 0.0f;
#pragma unroll
    for (int s = 0; s < NKC; ++s) {
      const fh8 b0 = ld_s(halo + hb[0] + ctr + 16 * s), b1 = ld_s(halo + hb[1] + ctr + 16 * s);
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[s], b0, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[s], b1, acc[1], 0, 0, 0);
    }
    feed(acc, p.b1, c0, c0);
  }
  // expand3x3 chunks: 9 taps x NKC k-steps, k order (r, s, c)
  for (int c0 = 0; c0 < E3; c0 += 32) {
    fh8 a[PD];
#pragma unroll
    for (int s = 0; s < PD; ++s)
      if (s < NS3) a[s] = ld_g(w3 + (s * E3 + c0) * 16 + arow);
    ff16 acc[2];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[f][e] = 0.0f;
    // B fragments one step ahead, A PD steps ahead; the barrier keeps every step's loads in it
    // (unpinned, the scheduler hoists all 2 x NS3 LDS reads and spills)
    auto boff = [&](int s) __attribute__((always_inline)) {
      const int tap = s / NKC, cs = s - tap * NKC;
      return ((tap / 3) * W2 + tap % 3) * PS + 16 * cs;
    };
    fh8 bn0 = ld_s(halo + hb[0] + boff(0)), bn1 = ld_s(halo + hb[1] + boff(0));
#pragma unroll
    for (int s = 0; s < NS3; ++s) {
      const fh8 cur = a[s % PD], b0 = bn0, b1 = bn1;
      if (s + PD < NS3) a[s % PD] = ld_g(w3 + ((s + PD) * E3 + c0) * 16 + arow);
      if (s + 1 < NS3) {
        bn0 = ld_s(halo + hb[0] + boff(s + 1));
        bn1 = ld_s(halo + hb[1] + boff(s + 1));
      }
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(cur, b0, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(cur, b1, acc[1], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    feed(acc, p.b3, c0, E1 + c0);
  }

  // squeeze epilogue: bias + Relu + one rounding; element 8g + e of lane half h = channel
  // 32 i + 16 g + 8 h + e, one 16-B store per (fragment, g)
  _Float16* __restrict__ y = static_cast<_Float16*>(p.y) + (long long)img * p.y_nstride;
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
      for (int f = 0; f < 2; ++f) {
        if (!pok[f]) continue;
        fh8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (_Float16)fmaxf(sacc[i][f][8 * g + e] + bv[e], 0.0f);
        *reinterpret_cast<fh8*>(y + yo[f] + 32 * i + 16 * g) = o;
      }
    }
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

int fire_f16_lds_bytes(int C, int H, int W) { return ff_halo_rows(H, W) * (W + 2) * (C + 8) * 2; }

bool fire_f16_eligible(const FireF16Params& p) {
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  return p.C % 16 == 0 && p.C >= 16 && p.C <= 64 && p.E1 % 32 == 0 && p.E3 % 32 == 0 && p.E1 > 0 && p.E3 > 0 &&
         p.Ms % 8 == 0 && p.Ms > 0 && p.Ms <= 64 && p.Msp == (p.Ms + 31) / 32 * 32 && p.x_cs % 8 == 0 &&
         p.y_cs % 8 == 0 && p.x_cs >= p.C && p.y_cs >= p.Ms && p.x_nstride % 8 == 0 && p.y_nstride % 8 == 0 &&
         al16(p.x) && al16(p.y) && al16(p.w1) && al16(p.w3) && al16(p.ws) && al16(p.b1) && al16(p.b3) && al16(p.bs) &&
         p.H > 0 && p.W > 0 && p.N > 0 && fire_f16_lds_bytes(p.C, p.H, p.W) <= FIRE_F16_LDS_MAX &&
         (long long)p.H * p.W * p.x_cs < (1LL << 30) && (long long)p.H * p.W * p.y_cs < (1LL << 30);
}

template <int NKC, int MSF>
static void launch_ff(FireF16Params p, hipStream_t s) {
  p.tiles_per_img = (p.H * p.W + FF_PIX - 1) / FF_PIX;
  const unsigned lds = (unsigned)fire_f16_lds_bytes(p.C, p.H, p.W);
  hipLaunchKernelGGL((fire_f16_kernel<NKC, MSF>), dim3((unsigned)(p.N * p.tiles_per_img)), dim3(256), lds, s, p);
}

void launch_fire_f16(const FireF16Params& p, hipStream_t s) {
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
