// MaxPool 3x3 / stride 2 + the 1x1 Conv (+ Relu) that is its only reader, f32 NCHW, in one launch:
// SqueezeNet's pool5 -> fire9/squeeze1x1 (reference max_pool_op.rs:157-360, convolution_op.rs:94-517;
// the walker used to run maxpool_kernel (382 MB in, 95 MB out at B = 256) and then the squeeze
// (95 MB in again)).  The pooled map never reaches HBM.
//
// One workgroup = PS_PR (3) pooled rows of one image (Wp <= 16 NF columns each: NF 16-pixel
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
// S (C1 = 4 KS1 channels, the squeeze output of the same fire module): each wave loads its FRW 16-pixel
// fragments of the band's 2 PS_PR + 1 rows once, straight into the MFMA B registers (no LDS: the
// workgroup keeps the plain kernel's LDS size and occupancy).  Per such chunk every wave runs 16x16x4
// MFMAs over those fragments (16 channels x 16 band pixels, k = 4 t + lk ascending from zero, the
// fragments' chains interleaved: the streaming 1x1 conv's fma chain),
// adds the bias and applies the Relu exactly as conv_stream_kernel's epilogue, and writes the values
// into the staged rows (rows outside the image: the pool's zero padding); pooling and the squeeze then
// run as for a loaded chunk.  fire4 -> pool3 -> fire5 and fire8 -> pool5 -> fire9 no longer write and
// re-read e1's map (386 / 193 MB at B = 256).  Bit-identical to the separate launches.
#include <float.h>
#include <hip/hip_runtime.h>

#include <type_traits>


#include "ore_kernels.h"

namespace ore {

namespace {

typedef float ps4 __attribute__((ext_vector_type(4)));

#define ORE_PS_CH 16  // input channels per chunk
constexpr int PS_CH = ORE_PS_CH;
// input loads non-temporal (cache policy nt): read once, and a streamed read measured 10 % faster
// with it (profiles/r03k_hbm_probe.txt); pool5 + squeeze 110.3 -> 105.7 us, pool3 205 -> 204 us
constexpr int PS_AUX = 2;
// pooled rows per workgroup (PS_PR): 3 for both widths.  Against 2 (B = 256, tools/r05zi.sh,
// profiles/r05zi_ab_pool_rows.txt): pool3 + e1 + squeeze 274-276 -> 256-257 us (9 bands of 7 input rows
// instead of 14 of 5: e1 recomputed and input fetched 1.17x instead of 1.30x / 1.25x, still two waves per
// SIMD), pool5 + squeeze 107-109 -> 102 us; 4 rows for pool5 measured 110 us (four waves per SIMD)
__host__ __device__ constexpr int ps_pr(int /*nf: fragments per pooled row*/) { return 3; }

// n / d for 0 <= n < 2^11, 1 <= d < 2^9 by a multiply and a shift: mg = ceil(2^20 / d) (computed once, uniform);
// n mg / 2^20 is within n 2^-20 < 2^-9 above n / d, below the next integer: exact (round 6: the staging
// geometry's runtime divisions were ~40 VALU each, with quarter-rate multiplies)
__device__ __forceinline__ int ps_div(int n, unsigned mg) { return (int)(__umul24((unsigned)n, mg) >> 20); }
__device__ __forceinline__ unsigned ps_magic(int d) { return (unsigned)(((1u << 20) + d - 1) / d); }

// NF: 16-pixel fragments per pooled row (Wp <= 16 NF); KS1: e1's k-steps (0: no e1); FRW: e1 pixel fragments
// per wave (>= ceil(ceil((2 PS_PR + 1) W / 16) / 4)); SPLIT: waves per 16-channel block of the squeeze (2: M <= 32
// on two blocks, each wave takes half the pooled-pixel fragments, so all four waves issue squeeze MFMAs)
// Launch bounds: with e1 inside at C1 = 32 and the squeeze split (KS1 = 8, SPLIT = 2: fire4 -> pool3 -> fire5),
// three waves per SIMD (168 VGPRs, 100 B of scratch spills at FRW = 6) instead of two (189 VGPRs + 48 AGPRs):
// pool3 + e1 + squeeze 230 -> 210 us (round 6, profiles/r06_pool_lb3.txt); a third resident workgroup covers the
// other two's barrier and LDS chains.  The other instances keep the compiler's choice
template <int NF, int KS1, int FRW, int SPLIT>
__global__ __launch_bounds__(256, (KS1 == 8 && SPLIT == 2 ? 3 : 1)) void pool_conv1x1_f32_kernel(PoolConvParams p) {
  constexpr int PS_PR = ps_pr(NF);
  constexpr int PS_ROWS = 2 * PS_PR + 1;  // input rows of PS_PR pooled rows (3x3, stride 2)
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
  // pooled block [ch][pixel n * PS_RW + col]; row stride = 16 mod 32 floats at NF = 2 (the squeeze's B reads of
  // lane groups lk, lk + 1 on disjoint banks; 16-B aligned rows for the pooling's 16-B stores), PS_PX + 1 at NF = 1
  constexpr int PT_S = NF >= 2 ? PS_PX + 16 : PS_PX + 1;
  __shared__ __attribute__((aligned(16))) float pt[PS_CH][PT_S];
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

  // e1 recomputed (KS1 > 0): this wave's band pixels 16 (wave + 4 i) + lj of S's rows [ih0, ih0 + PS_ROWS),
  // k = 4 t + lk, as MFMA B operands (pixels past the band or rows outside the image read 0); e1's bias in LDS
  constexpr int KA1 = KS1 > 0 ? KS1 : 1, FA1 = KS1 > 0 ? FRW : 1;
  __shared__ float b1_s[KS1 > 0 ? 256 : 1];
  const int ne1 = KS1 > 0 ? p.E1 / PS_CH : 0;  // recomputed chunks
  const int bpx = PS_ROWS * p.W;
  float sb[FA1][KA1];
  // in_s offset of the lane's pixel of fragment i (channel 0); -1: past the band or on a row outside the
  // image (never written: the staged rows start zeroed, and the recomputed chunks come first)
  int e1_off[FA1];
  if constexpr (KS1 > 0) {
    const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(p.s + (long long)img * p.s_nstride), (short)0, 4 * KS1 * p.s_ps * 4, 0x00020000);
    const int hw = p.H * p.W;
    const unsigned mgw = ps_magic(p.W);
#pragma unroll
    for (int i = 0; i < FRW; ++i) {
      const int px = 16 * (wave + 4 * i) + lj, r = ps_div(px, mgw), g = ih0 * p.W + px;
      const bool in = px < bpx && g >= 0 && g < hw;
      // the lane's channel lk at pixel g; k-step t's channels 4 t + lk: + 16 t s_ps bytes, the scalar offset
      const int vo = in ? (lk * p.s_ps + g) * 4 : (int)0x80000000;
#pragma unroll
      for (int t = 0; t < KS1; ++t)
        sb[i][t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(sr, vo, 16 * t * p.s_ps, 0));
      e1_off[i] = px < bpx && (unsigned)(ih0 + r) < (unsigned)p.H ? r * PS_RS + PS_LC + (px - r * p.W) : -1;
    }
    for (int i = tid; i < p.E1; i += 256) b1_s[i] = p.b1[i];
  }

  // this thread's 16-B groups q = tid + 256 u: (channel, row, group j) -> byte offset in the image
  // minus the chunk's channel offset (rows outside the image: past the records, 0), LDS float offset
  // and the mask of the group's elements inside the row (a group may run into the next row)
  // (computed where the loaded chunks begin: with e1 recomputed they are not live during its chunks)
  int qo[PS_NQ], qs[PS_NQ];
  unsigned qm[PS_NQ];
  auto group_geom = [&]() __attribute__((always_inline)) {
    const int nq = (p.W + 3) / 4, nld = PS_CH * PS_ROWS * nq;
    const unsigned mrow = ps_magic(PS_ROWS * nq), mq = ps_magic(nq);
#pragma unroll
    for (int u = 0; u < PS_NQ; ++u) {
      const int q = tid + 256 * u;
      const int c = ps_div(q, mrow), rc = q - c * (PS_ROWS * nq), r = ps_div(rc, mq), j = rc - r * nq;
      const int ih = ih0 + r;
      const bool rin = (unsigned)ih < (unsigned)p.H;
      // -1: no group (not loaded, not stored); a row outside the image: past the records (reads 0)
      qo[u] = q < nld ? (rin ? (c * p.x_ps + ih * p.W + 4 * j) * 4 : (int)0x80000000) : -1;
      qs[u] = (c * PS_ROWS + r) * PS_RS + PS_LC + 4 * j;
      unsigned mk = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) mk |= (4 * j + e < p.W ? 1u : 0u) << e;
      qm[u] = mk;
    }
  };
  ps4 xv[PS_NQ];
  auto load_chunk = [&](int c0) __attribute__((always_inline)) {
    // the chunk's first channel as the scalar offset (qo < 0 lies past the records either way)
#pragma unroll
    for (int u = 0; u < PS_NQ; ++u)
      xv[u] = __builtin_bit_cast(ps4, __builtin_amdgcn_raw_buffer_load_b128(xr, qo[u], c0 * p.x_ps * 4, PS_AUX));
    __builtin_amdgcn_sched_barrier(0);
  };

  // the wave's squeeze share: channels m0 .. m0 + 15 at pooled-pixel fragments n0 .. n0 + NFW - 1 (fragment n:
  // pooled row n / NF, columns 16 (n % NF) ..)
  constexpr int NFW = PS_PR * NF / SPLIT;
  static_assert(PS_PR * NF % SPLIT == 0, "fragments split evenly");
  ps4 acc[NFW];  // rows 4 lk + e of channels m0 .., pixel 16 (n % NF) + lj of pooled row n / NF, n = n0 + i
#pragma unroll
  for (int n = 0; n < NFW; ++n) acc[n] = ps4{0.f, 0.f, 0.f, 0.f};
  const int nch = p.C / PS_CH;
  const int m0 = 16 * (wave / SPLIT), n0 = NFW * (wave % SPLIT);
  // the squeeze's A values of a chunk (k = PS_CH ci + 4 t + lk, row m0 + lj), one chunk ahead
  constexpr int KS = PS_CH / 4;  // k-steps per chunk
  float acur[KS], anxt[KS];
  auto load_a = [&](float (&dst)[KS], int ci) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < KS; ++t)
      dst[t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                             wr, ((ci * PS_CH + 4 * t + lk) * p.Mp + m0 + lj) * 4, 0, 0));
  };
  // e1's A values of a recomputed chunk (k = 4 t + lk, row 16 ci + lj of the K-major packing), reloaded with
  // the next chunk's as soon as this chunk's e1 MFMAs have issued
  float a1cur[KA1];
  const __amdgpu_buffer_rsrc_t w1r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(KS1 > 0 ? p.w1 : p.wp), (short)0, 4 * KS1 * p.w1_Mp * 4, 0x00020000);
  auto load_a1 = [&](float (&dst)[KA1], int ci) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < KS1; ++t)
      dst[t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                             w1r, ((4 * t + lk) * p.w1_Mp + PS_CH * ci + lj) * 4, 0, 0));
  };
  load_a(acur, 0);
  if (ne1 > 0) {
    load_a1(a1cur, 0);
  } else {
    group_geom();
    load_chunk(0);
  }
  // one chunk; RC: a recomputed e1 chunk, TR: the last of them (it starts the loaded chunks' loads).  The
  // kinds run as separate loops and the last recomputed chunk is peeled, so e1's B registers and the
  // loaded chunks' staging registers are never live together (two more waves per SIMD)
  auto chunk = [&](int ci, auto rc, auto tr) __attribute__((always_inline)) {
    constexpr bool RC = decltype(rc)::value, TR = decltype(tr)::value;
    __syncthreads();  // the previous chunk's staged rows are pooled
    if constexpr (RC) {
      // e1 channels 16 ci + 4 lk + e at the wave's band pixels: the 1x1 conv, bias, Relu -> staged rows
      ps4 a[FA1];
#pragma unroll
      for (int i = 0; i < FA1; ++i) a[i] = ps4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < KA1; ++t)
#pragma unroll
        for (int i = 0; i < FA1; ++i) a[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1cur[t], sb[i][t], a[i], 0, 0, 0);
      if constexpr (!TR) load_a1(a1cur, ci + 1);
      float bb[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) bb[e] = b1_s[PS_CH * ci + 4 * lk + e];
#pragma unroll
      for (int i = 0; i < FA1; ++i) {
        if (e1_off[i] < 0) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = a[i][e] + bb[e];
          v = fmaxf(v, 0.0f);
          in_s[(4 * lk + e) * PS_ROWS * PS_RS + e1_off[i]] = v;
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
      if constexpr (!RC || TR) {
        if constexpr (TR) group_geom();
        load_chunk((ci + 1) * PS_CH);
      }
      load_a(anxt, ci + 1);
    }
    // pooled maxima: channels x PS_PR rows x PS_RW columns (columns >= Wp: values of the staged row's
    // padding, unused).  pl = 0: a task is 4 pooled columns, whose 3 x 9 window values are 2 x 16-B + one
    // 4-B LDS read per row (16-B aligned: the rows start at PS_LC + 8 j); else one column per task.  Each
    // maximum runs from -FLT_MAX over rows then columns, as maxpool_kernel's
    if (NF >= 2 && p.pl == 0) {  // (NF = 1: 128 tasks for 256 threads measured slower, 106 -> 119 us)
      constexpr int NT = PS_CH * PS_PR * (PS_RW / 4);
      for (int t = tid; t < NT; t += 256) {
        const int c = t / (PS_PR * (PS_RW / 4)), rem = t - c * (PS_PR * (PS_RW / 4));
        const int n = rem / (PS_RW / 4), c4 = rem - n * (PS_RW / 4);
        const float* base = in_s + (c * PS_ROWS + 2 * n) * PS_RS + PS_LC + 8 * c4 - p.pl;
        float v[3][9];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const ps4 lo = *reinterpret_cast<const ps4*>(base + r * PS_RS);
          const ps4 hi = *reinterpret_cast<const ps4*>(base + r * PS_RS + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[r][e] = lo[e];
            v[r][4 + e] = hi[e];
          }
          v[r][8] = base[r * PS_RS + 8];
        }
        ps4 m4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float m = -FLT_MAX;
#pragma unroll
          for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int s = 0; s < 3; ++s) m = fmaxf(m, v[r][2 * j + s]);
          m4[j] = m;
        }
        *reinterpret_cast<ps4*>(&pt[c][n * PS_RW + 4 * c4]) = m4;  // one 16-B store (4 B at 16-B lane stride: 4-way)
      }
    } else {
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
    }
    __syncthreads();
    // squeeze k-steps of this chunk: k = PS_CH ci + 4 t + lk
    if (m0 < p.M) {  // every B value read before the MFMAs: one LDS round trip, not one per k-step
      float bq[KS][NFW];
#pragma unroll
      for (int t = 0; t < KS; ++t)
#pragma unroll
        for (int n = 0; n < NFW; ++n) bq[t][n] = pt[4 * t + lk][16 * (n0 + n) + lj];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < KS; ++t)
#pragma unroll
        for (int n = 0; n < NFW; ++n) acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(acur[t], bq[t][n], acc[n], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < KS; ++t) acur[t] = anxt[t];
  };
  int ci = 0;
  if constexpr (KS1 > 0) {
    for (; ci + 1 < ne1; ++ci) chunk(ci, std::true_type{}, std::false_type{});
    chunk(ci++, std::true_type{}, std::true_type{});
  }
  for (; ci < nch; ++ci) chunk(ci, std::false_type{}, std::false_type{});
  // bias + Relu, NCHW stores: channel m0 + 4 lk + e, pooled pixel (pr0 + n / NF, 16 (n % NF) + lj)
  if (m0 >= p.M) return;
#pragma unroll
  for (int i = 0; i < NFW; ++i) {
    const int n = n0 + i;
    const int prow = pr0 + n / NF, pcol = 16 * (n % NF) + lj;
    if (prow >= p.Hp || pcol >= p.Wp) continue;
    float* yp = p.y + (long long)img * p.y_nstride + prow * p.Wp + pcol;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + 4 * lk + e;
      if (m >= p.M) continue;
      float v = acc[i][e] + (p.bias ? p.bias[m] : 0.0f);
      if (p.relu) v = fmaxf(v, 0.0f);
      yp[(long long)m * p.y_ps] = v;
    }
  }
}

}  // namespace

// e1 pixel fragments per wave of the recomputed-e1 variant (the band's (2 PS_PR + 1) W pixels over 4 waves)
static int ps_nf(const PoolConvParams& p) { return p.Wp <= 16 ? 1 : 2; }
static int ps_frw(const PoolConvParams& p) { return (((2 * ps_pr(ps_nf(p)) + 1) * p.W + 15) / 16 + 3) / 4; }

bool pool_conv1x1_f32_eligible(const PoolConvParams& p) {
  const bool e1ok = p.E1 == 0 ||
                    ((p.C1 == 32 || p.C1 == 64) && p.E1 % PS_CH == 0 && p.E1 <= p.C && p.s && p.w1 && p.b1 &&
                     p.w1_Mp >= p.E1 && p.s_ps >= p.H * p.W && (long long)p.C1 * p.s_ps * 4 < (1LL << 31) &&
                     (long long)p.C1 * p.w1_Mp * 4 < (1LL << 31) && p.E1 <= 256 && ps_frw(p) <= 6);
  return p.C % PS_CH == 0 && p.C > 0 && p.M >= 1 && p.M <= 64 && p.Wp >= 1 && p.Wp <= 32 && p.Hp >= 1 &&
         p.W <= 2 * (p.Wp <= 16 ? 16 : 32) + 1 && 2 * (p.Wp - 1) + 2 - p.pl <= p.W + 1 &&
         p.pt >= 0 && p.pl >= 0 && p.pt <= 2 && p.pl <= 2 && p.x_ps >= p.H * p.W &&
         (long long)p.C * p.x_ps * 4 < (1LL << 31) && (long long)p.Kp * p.Mp * 4 < (1LL << 31) && p.Kp >= p.C &&
         p.Mp >= p.M && p.y_ps >= p.Hp * p.Wp && e1ok;
}

template <int NF, int KS1, int FRW>
static void ps_launch(const PoolConvParams& p, long long grid, hipStream_t s) {
  // two waves per 16-channel block when the squeeze has <= 32 channels and the fragments split evenly
  if constexpr (ps_pr(NF) * NF % 2 == 0) {
    if (p.M <= 32) {
      hipLaunchKernelGGL((pool_conv1x1_f32_kernel<NF, KS1, FRW, 2>), dim3((unsigned)grid), dim3(256), 0, s, p);
      return;
    }
  }
  hipLaunchKernelGGL((pool_conv1x1_f32_kernel<NF, KS1, FRW, 1>), dim3((unsigned)grid), dim3(256), 0, s, p);
}

template <int NF, int KS1>
static void ps_dispatch_frw(const PoolConvParams& p, long long grid, hipStream_t s) {
  switch (ps_frw(p)) {  // the fewest fragments per wave that cover the band
    case 1: case 2: ps_launch<NF, KS1, 2>(p, grid, s); break;
    case 3: ps_launch<NF, KS1, 3>(p, grid, s); break;
    case 4: ps_launch<NF, KS1, 4>(p, grid, s); break;
    case 5: ps_launch<NF, KS1, 5>(p, grid, s); break;
    default: ps_launch<NF, KS1, 6>(p, grid, s); break;
  }
}

template <int NF>
static void ps_dispatch(const PoolConvParams& p, long long grid, hipStream_t s) {
  if (p.E1 == 0)
    ps_launch<NF, 0, 0>(p, grid, s);
  else if (p.C1 == 32)
    ps_dispatch_frw<NF, 8>(p, grid, s);
  else
    ps_dispatch_frw<NF, 16>(p, grid, s);
}

int pool_conv1x1_f32_rows(int Wp) { return ps_pr(Wp <= 16 ? 1 : 2); }

void launch_pool_conv1x1_f32(const PoolConvParams& p, hipStream_t s) {
  const int pr = ps_pr(ps_nf(p));
  const long long grid = (long long)p.N * ((p.Hp + pr - 1) / pr);
  if (ps_nf(p) == 1)
    ps_dispatch<1>(p, grid, s);
  else
    ps_dispatch<2>(p, grid, s);
}

}  // namespace ore
