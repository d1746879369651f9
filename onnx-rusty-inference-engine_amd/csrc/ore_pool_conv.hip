// MaxPool 3x3 / stride 2 + the 1x1 Conv (+ Relu) that is its only reader, f32 NCHW, in one launch:
// SqueezeNet's pool5 -> fire9/squeeze1x1 (reference max_pool_op.rs:157-360, convolution_op.rs:94-517;
// the walker used to run maxpool_kernel (382 MB in, 95 MB out at B = 256) and then the squeeze
// (95 MB in again)).  The pooled map never reaches HBM.
//
// One workgroup = PS_PR (2) pooled rows of one image (Wp <= 16 NF columns each: NF 16-pixel
// fragments per row; NF = 1 for pool5's 13 columns, 2 for pool3's 27) x all M <= 64 output channels
// (four waves x 16 channels, v_mfma_f32_16x16x4_f32).  Per chunk of PS_CH (16) input channels:
//   * the 2 PS_PR + 1 input rows the pooled rows read (whole rows) go global -> registers
//     -> LDS as 16-B groups (4-B aligned raw buffer loads; rows outside the image read 0 past the
//     records, columns outside it are zeros in LDS: maxpool_kernel's zero padding); the next
//     chunk's loads are in flight while this one pools and multiplies;
//   * every thread takes (pooled pixel, channel) maxima from -FLT_MAX over the nine window values
//     (maxpool_kernel's arithmetic) into an LDS block [channels][16 PS_PR pixels];
//   * each wave runs the chunk's k-steps (k = channel, ascending over the chunks: the standalone
//     1x1 conv's fma chain) for its 16 channels x both pixel fragments; A from L2 in the conv's
//     K-major packing (wp[k][Mp]).
// Bit-identical to maxpool_kernel + the separate 1x1 conv (tests/test_model_gpu.py).
//
// ORE_FUSE_POOL_EXPAND (KS1 > 0): the pool input is a fire module's Concat(e1, e3) whose e1 slice (the
// expand1x1, E1 channels) is never stored: chunks ci < E1 / 16 are recomputed here from e1's own input
// S (C1 = 4 KS1 channels, the squeeze output of the same fire module), staged once per workgroup for
// the band's 2 PS_PR + 1 rows.  Per such chunk every wave runs 16x16x4 MFMAs over its pixel fragments
// (16 channels x 16 band pixels, k = 4 t + lk ascending from zero: the streaming 1x1 conv's fma chain),
// adds the bias and applies the Relu exactly as conv_stream_kernel's epilogue, and writes the values
// into the staged rows (rows outside the image: the pool's zero padding); pooling and the squeeze then
// run as for a loaded chunk.  fire4 -> pool3 -> fire5 and fire8 -> pool5 -> fire9 no longer write and
// re-read e1's map (386 / 193 MB at B = 256).  Bit-identical to the separate launches.
#include <float.h>
#include <hip/hip_runtime.h>

#include <atomic>

#include "ore_kernels.h"

namespace ore {

namespace {

typedef float ps4 __attribute__((ext_vector_type(4)));

#define ORE_PS_PR 2   // pooled rows per workgroup
#define ORE_PS_CH 16  // input channels per chunk
constexpr int PS_PR = ORE_PS_PR, PS_CH = ORE_PS_CH;
// input loads non-temporal (cache policy nt): read once, and a streamed read measured 10 % faster
// with it (profiles/r03k_hbm_probe.txt); pool5 + squeeze 110.3 -> 105.7 us, pool3 205 -> 204 us
constexpr int PS_AUX = 2;
constexpr int PS_ROWS = 2 * PS_PR + 1;  // input rows of PS_PR pooled rows (3x3, stride 2)

// LDS floats of the staged S band (KS1 > 0): C1 channels x PXS pixels; PXS = the band's 2 PS_PR + 1
// rows of W pixels rounded up to 16-pixel fragments, = 16 mod 32 (the lane groups lk = 0 / 1 of a
// ds_read_b32 hit opposite halves of the banks)
__host__ __device__ constexpr int ps_pxs(int W) {
  const int fr = ((2 * ORE_PS_PR + 1) * W + 15) / 16 * 16;
  return fr % 32 == 16 ? fr : fr + 16;
}

template <int NF, int KS1>  // NF: 16-pixel fragments per pooled row (Wp <= 16 NF); KS1: e1's k-steps (0: no e1)
__global__ __launch_bounds__(256) void pool_conv1x1_f32_kernel(PoolConvParams p) {
  // staged rows: input column iw at LDS column iw + PS_LC; columns left of the image and right of
  // the loaded 16-B groups are zero once (never written), loaded columns >= W are zeroed per element
  constexpr int PS_LC = 4;
  constexpr int PS_NQMAX = (32 * NF + 1 + 3) / 4;             // 16-B groups of the widest row
  constexpr int PS_RS = PS_LC + 4 * PS_NQMAX + 4;            // LDS row stride (floats, 16-B multiple)
  constexpr int PS_IN = PS_CH * PS_ROWS * PS_RS;             // floats of one staged chunk
  constexpr int PS_NQ = (PS_CH * PS_ROWS * PS_NQMAX + 255) / 256;  // 16-B loads per thread per chunk
  constexpr int PS_RW = 16 * NF;                             // pooled pixels held per row
  constexpr int PS_PX = PS_RW * PS_PR;                       // pooled pixels of a workgroup
  __shared__ __attribute__((aligned(16))) float in_s[PS_IN];  // [ch][row][col]
  __shared__ float pt[PS_CH][PS_PX + 1];   // pooled block [ch][pixel n * PS_RW + col] (+1 pad)
  const int tid = threadIdx.x, lane = tid & 63, lk = lane >> 4, lj = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bands = (p.Hp + PS_PR - 1) / PS_PR;
  // XCD-aware bijective block remap (consecutive bands of an image on one XCD: the input row a band
  // shares with the next one is read once from HBM)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, rr8 = nwg & 7;
  const int wgid = (xcd < rr8 ? xcd * (q8 + 1) : rr8 * (q8 + 1) + (xcd - rr8) * q8) + (bid >> 3);
  // images in reverse order: the producers (the expand convs of fire4 / fire8) write images in
  // ascending order, so their last images are still in the 256 MB Infinity Cache when this launch
  // starts (pool3 + squeeze 216 -> 206 us, pool5 + squeeze 121 -> 109 us at B = 256)
  const int img = p.N - 1 - wgid / bands, pr0 = (wgid - (wgid / bands) * bands) * PS_PR;
  const int ih0 = pr0 * 2 - p.pt;  // input row of staged row 0
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.x + (long long)img * p.x_nstride), (short)0, p.C * p.x_ps * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.wp), (short)0, p.Kp * p.Mp * 4, 0x00020000);
  for (int i = tid; i < PS_IN; i += 256) in_s[i] = 0.0f;

  // e1 recomputed (KS1 > 0): S's band rows [ih0, ih0 + PS_ROWS) as [C1][PXS] (dynamic LDS; rows outside
  // the image and the fragment padding are 0), e1's bias at the end
  extern __shared__ __attribute__((aligned(16))) float e1_s[];
  const int ne1 = KS1 > 0 ? p.E1 / PS_CH : 0;  // recomputed chunks
  const int pxs = ps_pxs(p.W), bpx = PS_ROWS * p.W;
  float* b1_s = e1_s + 4 * KS1 * pxs;
  if constexpr (KS1 > 0) {
    const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(p.s + (long long)img * p.s_nstride), (short)0, 4 * KS1 * p.s_ps * 4, 0x00020000);
    const int hw = p.H * p.W, g0 = ih0 * p.W;
    for (int i0 = 0; i0 < 4 * KS1 * pxs; i0 += 256 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {  // 8 loads in flight per thread
        const int i = i0 + 256 * u + tid, c = i / pxs, px = i - c * pxs, g = g0 + px;
        const bool in = i < 4 * KS1 * pxs && px < bpx && g >= 0 && g < hw;
        v[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                             sr, in ? (c * p.s_ps + g) * 4 : (int)0x80000000, 0, 0));
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + 256 * u + tid;
        if (i < 4 * KS1 * pxs) e1_s[i] = v[u];
      }
    }
    for (int i = tid; i < p.E1; i += 256) b1_s[i] = p.b1[i];
  }

  // this thread's 16-B groups q = tid + 256 u: (channel, row, group j) -> byte offset in the image
  // minus the chunk's channel offset (rows outside the image: past the records, 0), LDS float offset
  // and the mask of the group's elements inside the row (a group may run into the next row)
  const int nq = (p.W + 3) / 4, nld = PS_CH * PS_ROWS * nq;
  int qo[PS_NQ], qs[PS_NQ];
  unsigned qm[PS_NQ];
#pragma unroll
  for (int u = 0; u < PS_NQ; ++u) {
    const int q = tid + 256 * u;
    const int c = q / (PS_ROWS * nq), rc = q - c * (PS_ROWS * nq), r = rc / nq, j = rc - r * nq;
    const int ih = ih0 + r;
    const bool rin = (unsigned)ih < (unsigned)p.H;
    qo[u] = q < nld ? (rin ? (c * p.x_ps + ih * p.W + 4 * j) * 4 : (int)0x80000000) : -1;
    qs[u] = (c * PS_ROWS + r) * PS_RS + PS_LC + 4 * j;
    unsigned mk = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) mk |= (4 * j + e < p.W ? 1u : 0u) << e;
    qm[u] = mk;
  }
  ps4 xv[PS_NQ];
  auto load_chunk = [&](int c0) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < PS_NQ; ++u)
      xv[u] = __builtin_bit_cast(ps4, __builtin_amdgcn_raw_buffer_load_b128(
                                          xr, qo[u] < 0 ? (int)0x80000000 : qo[u] + c0 * p.x_ps * 4, 0, PS_AUX));
    __builtin_amdgcn_sched_barrier(0);
  };

  ps4 acc[PS_PR * NF];  // rows 4 lk + e of channels 16 wave .., pixel 16 fr + lj of pooled row n
#pragma unroll
  for (int n = 0; n < PS_PR * NF; ++n) acc[n] = ps4{0.f, 0.f, 0.f, 0.f};
  const int nch = p.C / PS_CH;
  const int m0 = 16 * wave;
  // the squeeze's A values of a chunk (k = PS_CH ci + 4 t + lk, row m0 + lj), one chunk ahead
  constexpr int KS = PS_CH / 4;  // k-steps per chunk
  float acur[KS], anxt[KS];
  auto load_a = [&](float (&dst)[KS], int ci) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < KS; ++t)
      dst[t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                             wr, ((ci * PS_CH + 4 * t + lk) * p.Mp + m0 + lj) * 4, 0, 0));
  };
  // e1's A values of a recomputed chunk (k = 4 t + lk, row 16 ci + lj of the K-major packing), one chunk ahead
  constexpr int KA1 = KS1 > 0 ? KS1 : 1;
  float a1cur[KA1], a1nxt[KA1];
  const __amdgpu_buffer_rsrc_t w1r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(KS1 > 0 ? p.w1 : p.wp), (short)0, 4 * KS1 * p.w1_Mp * 4, 0x00020000);
  auto load_a1 = [&](float (&dst)[KA1], int ci) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < KS1; ++t)
      dst[t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                             w1r, ((4 * t + lk) * p.w1_Mp + PS_CH * ci + lj) * 4, 0, 0));
  };
  load_a(acur, 0);
  if (ne1 > 0)
    load_a1(a1cur, 0);
  else
    load_chunk(0);
  const int nfr1 = (bpx + 15) / 16;  // e1 pixel fragments of the band
  for (int ci = 0; ci < nch; ++ci) {
    __syncthreads();  // the previous chunk's staged rows are pooled (and, before chunk 0, S is staged)
    if (KS1 > 0 && ci < ne1) {
      // e1 channels 16 ci + 4 lk + e at band pixel 16 fr + lj: the 1x1 conv, bias, Relu -> staged rows
      for (int fr = wave; fr < nfr1; fr += 4) {
        ps4 a = ps4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < KS1; ++t)
          a = __builtin_amdgcn_mfma_f32_16x16x4f32(a1cur[t], e1_s[(4 * t + lk) * pxs + 16 * fr + lj], a, 0, 0, 0);
        const int px = 16 * fr + lj, r = px / p.W, col = px - r * p.W;
        if (px < bpx) {
          const bool rin = (unsigned)(ih0 + r) < (unsigned)p.H;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int ch = 4 * lk + e;
            float v = a[e] + b1_s[PS_CH * ci + ch];
            v = fmaxf(v, 0.0f);
            in_s[(ch * PS_ROWS + r) * PS_RS + PS_LC + col] = rin ? v : 0.0f;
          }
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < PS_NQ; ++u) {
        if (qo[u] == -1) continue;  // no group
        ps4 v = xv[u];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (qm[u] >> e) & 1 ? v[e] : 0.0f;
        *reinterpret_cast<ps4*>(in_s + qs[u]) = v;
      }
    }
    __syncthreads();
    if (ci + 1 < nch) {  // in flight during this chunk
      if (ci + 1 >= ne1)
        load_chunk((ci + 1) * PS_CH);
      else
        load_a1(a1nxt, ci + 1);
      load_a(anxt, ci + 1);
    }
    // pooled maxima: channels x PS_PR rows x PS_RW columns (columns >= Wp: column 0's value, unused)
    for (int t = tid; t < PS_CH * PS_PX; t += 256) {
      const int c = t / PS_PX, pxi = t - c * PS_PX, n = pxi / PS_RW, col = pxi - n * PS_RW, cl = col < p.Wp ? col : 0;
      const float* base = in_s + (c * PS_ROWS + 2 * n) * PS_RS + PS_LC + 2 * cl - p.pl;
      float m = -FLT_MAX;
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s) m = fmaxf(m, base[r * PS_RS + s]);
      pt[c][pxi] = m;
    }
    __syncthreads();
    // squeeze k-steps of this chunk: k = PS_CH ci + 4 t + lk
    if (m0 < p.M) {
#pragma unroll
      for (int t = 0; t < KS; ++t)
#pragma unroll
        for (int n = 0; n < PS_PR * NF; ++n)
          acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(acur[t], pt[4 * t + lk][16 * n + lj], acc[n], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < KS; ++t) acur[t] = anxt[t];
    if (KS1 > 0 && ci + 1 < ne1) {
#pragma unroll
      for (int t = 0; t < KS1; ++t) a1cur[t] = a1nxt[t];
    }
  }
  // bias + Relu, NCHW stores: channel m0 + 4 lk + e, pooled pixel (pr0 + n / NF, 16 (n % NF) + lj)
  if (m0 >= p.M) return;
#pragma unroll
  for (int n = 0; n < PS_PR * NF; ++n) {
    const int prow = pr0 + n / NF, pcol = 16 * (n % NF) + lj;
    if (prow >= p.Hp || pcol >= p.Wp) continue;
    float* yp = p.y + (long long)img * p.y_nstride + prow * p.Wp + pcol;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + 4 * lk + e;
      if (m >= p.M) continue;
      float v = acc[n][e] + (p.bias ? p.bias[m] : 0.0f);
      if (p.relu) v = fmaxf(v, 0.0f);
      yp[(long long)m * p.y_ps] = v;
    }
  }
}

}  // namespace

// dynamic LDS of the recomputed-e1 variant: the S band and e1's bias
static size_t ps_e1_lds(const PoolConvParams& p) { return ((size_t)p.C1 * ps_pxs(p.W) + p.E1) * 4; }

bool pool_conv1x1_f32_eligible(const PoolConvParams& p) {
  const bool e1ok = p.E1 == 0 ||
                    ((p.C1 == 32 || p.C1 == 64) && p.E1 % PS_CH == 0 && p.E1 <= p.C && p.s && p.w1 && p.b1 &&
                     p.w1_Mp >= p.E1 && p.s_ps >= p.H * p.W && (long long)p.C1 * p.s_ps * 4 < (1LL << 31) &&
                     (long long)p.C1 * p.w1_Mp * 4 < (1LL << 31) && ps_e1_lds(p) <= 64 * 1024);
  return p.C % PS_CH == 0 && p.C > 0 && p.M >= 1 && p.M <= 64 && p.Wp >= 1 && p.Wp <= 32 && p.Hp >= 1 &&
         p.W <= 2 * (p.Wp <= 16 ? 16 : 32) + 1 && 2 * (p.Wp - 1) + 2 - p.pl <= p.W + 1 &&
         p.pt >= 0 && p.pl >= 0 && p.pt <= 2 && p.pl <= 2 && p.x_ps >= p.H * p.W &&
         (long long)p.C * p.x_ps * 4 < (1LL << 31) && (long long)p.Kp * p.Mp * 4 < (1LL << 31) && p.Kp >= p.C &&
         p.Mp >= p.M && p.y_ps >= p.Hp * p.Wp && e1ok;
}

template <int NF, int KS1>
static void ps_launch(const PoolConvParams& p, long long grid, hipStream_t s) {
  const size_t lds = KS1 > 0 ? ps_e1_lds(p) : 0;
  if (lds > 32 * 1024) {  // with the static arrays above the default 64 KB: raised once per device
    static std::atomic<unsigned long long> raised{0};
    ore_raise_lds_once(raised, reinterpret_cast<const void*>(&pool_conv1x1_f32_kernel<NF, KS1>), 96 * 1024);
  }
  hipLaunchKernelGGL((pool_conv1x1_f32_kernel<NF, KS1>), dim3((unsigned)grid), dim3(256), lds, s, p);
}

template <int NF>
static void ps_dispatch(const PoolConvParams& p, long long grid, hipStream_t s) {
  if (p.E1 == 0)
    ps_launch<NF, 0>(p, grid, s);
  else if (p.C1 == 32)
    ps_launch<NF, 8>(p, grid, s);
  else
    ps_launch<NF, 16>(p, grid, s);
}

void launch_pool_conv1x1_f32(const PoolConvParams& p, hipStream_t s) {
  const long long grid = (long long)p.N * ((p.Hp + PS_PR - 1) / PS_PR);
  if (p.Wp <= 16)
    ps_dispatch<1>(p, grid, s);
  else
    ps_dispatch<2>(p, grid, s);
}

}  // namespace ore
