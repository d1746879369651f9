// Conv (convolution_op.rs:94-517) and MatMul (mul_op.rs:23) on the gfx950 f32 MFMA
// (v_mfma_f32_32x32x2_f32: exact f32, k-ordered fma chain, 157.3 TFLOP/s dense peak).
//
// Implicit GEMM:  Y[m][n] = sum_k Wp[k][m] * B[k][n] (+ bias[m], optional Relu)
//   m = output channel, n = (image, output pixel) flattened, k = (cin, r, s).
//   Weights are packed once into K-major, zero-padded Wp[Kp][Mp] (Kp % 32 == 0, Mp % 128 == 0)
//   so the A tile is a plain 16-B-vectorised copy with no bounds checks.
//   B (the im2col of the input) is never materialised: each K tile gathers it straight from
//   the NCHW input (B1X1: contiguous rows k*x_ps + pix; BGATHER: a per-layer (cin, r, s) offset
//   table read with scalar loads, plus per-column image/row/col bases).
//   Block = 256 threads = 4 waves (WM x WN); block tile BM x BN x BK; LDS double-buffered, the
//   next K tile prefetched into registers while the current one feeds the MFMAs.
//   Fragment maps (cdna_hip_programming.md §3): lane l holds A[l&31][k=l>>5] and
//   B[k=l>>5][l&31]; accumulator register e of lane l is row (e&3)+8*(e>>2)+4*(l>>5), column
//   l&31 -> one register = two 128-B runs of consecutive output pixels.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "ore_kernels.h"

namespace ore {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));  // first-class vector (no struct copies)
typedef int int4d __attribute__((ext_vector_type(4)));

// pooled-epilogue tile (ORE_FUSE_CONV_POOL, 3x3 / stride-2 pools): 6 x 9 pooled outputs per block
// from a 13 x 19 = 247-column conv-output patch of a 256-column N tile
constexpr int EPOOL_PR = EPOOL_TILE_PR, EPOOL_PC = EPOOL_TILE_PC, EPOOL_RC = 2 * EPOOL_PR + 1, EPOOL_CC = 2 * EPOOL_PC + 1;

constexpr bool A_DMA = true;  // A (weight) tile by 16-B LDS-DMA too (false: registers + ds_write_b128)
#define ORE_FRAG_PIN __builtin_amdgcn_sched_barrier(0)
constexpr int CONV_MINBLOCKS = 2;  // __launch_bounds__ minimum blocks per CU (VGPR budget)

enum { B1X1 = 0, BGATHER = 1 };

// DMA: the B tile goes global -> LDS by buffer_load ... lds (no VGPR staging, no LDS store
// pass); a tap outside the image gets an out-of-range offset, which the buffer bounds check
// turns into a 0 -- the reference's zero padding -- with no select.
template <int BM, int BN, int WM, int WN, int BK, int BMODE, int DMA, int EP = 0>
__global__ __launch_bounds__(256, CONV_MINBLOCKS) void conv_gemm_kernel(ConvParams p) {
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 32, FN = TN / 32;
  // ADMA: the A tile also goes global -> LDS by 16-B LDS-DMA (lane-linear, so unpadded rows; the
  // fragment reads -- 32 consecutive floats per half-wave -- are conflict-free without padding)
  // (measured: 96-row tiles gain 1-3 %, the 128x128 tile loses 4 % on fire4/expand3x3 -> off there)
  constexpr bool ADMA = DMA && A_DMA && BM != 128;
  constexpr int AS = ADMA ? BM : BM + 4;     // LDS row stride of the A tile (16-B aligned rows)
  constexpr int BROWS = 256 / BN;            // B rows loaded per pass
  constexpr int BLOADS = BK / BROWS;         // B elements per thread per tile
  constexpr int AF4 = BM * BK / 4;           // float4s in the A tile
  constexpr int AVEC = (AF4 + 255) / 256;    // float4 A loads per thread per tile
  static_assert(WM * WN == 4 && FM >= 1 && FN >= 1 && BK % BROWS == 0 && AVEC >= 1, "tile");

  // one LDS array: the A/B double buffers of the main loop, reused by the epilogue's per-wave
  // [32][TN] output staging (all LDS in one __shared__ object, cdna_hip_programming.md §5)
  constexpr int NBUF = 2;
  constexpr int MAIN_FLOATS = NBUF * BK * AS + NBUF * BK * BN;
  constexpr int EPI_FLOATS = 4 * 32 * TN;
  __shared__ __attribute__((aligned(16))) float smem[MAIN_FLOATS > EPI_FLOATS ? MAIN_FLOATS : EPI_FLOATS];
  float(*As)[BK][AS] = reinterpret_cast<float(*)[BK][AS]>(smem);
  float(*Bs)[BK][BN] = reinterpret_cast<float(*)[BK][BN]>(smem + NBUF * BK * AS);
  __shared__ float sbias[BM];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm0 = (wave / WN) * TM;
  const int wn0 = (wave % WN) * TN;

  // XCD-aware bijective remap (cdna_hip_programming.md §5): consecutive tile ids (M fastest,
  // i.e. the M tiles sharing one B tile) land on one XCD and share its L2.
  const int nwg = p.mtiles * p.ntiles;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, rr8 = nwg & 7;
  const int wgid = (xcd < rr8 ? xcd * (q + 1) : rr8 * (q + 1) + (xcd - rr8) * q) + (bid >> 3);
  const int mt = wgid % p.mtiles;
  const int nt = wgid / p.mtiles;
  const int m0 = mt * BM;
  const int n0 = nt * BN;
  const int K = p.K;
  const int XPS = p.x_ps;  // channel-plane stride of x (>= H*W: planes may be padded)
  const int YPS = p.y_ps;  // channel-plane stride of y = columns iterated per image (>= Ho*Wo)

  for (int i = tid; i < BM; i += 256) sbias[i] = (p.bias && m0 + i < p.M) ? p.bias[m0 + i] : 0.0f;
  __syncthreads();

  // ---- this thread's B column (Ntot < 2^31 is checked on the host)
  const int bcol = tid % BN;
  const int krow = __builtin_amdgcn_readfirstlane(tid / BN);
  const int bn = n0 + bcol;
  bool bn_ok = bn < p.Ntot;
  // element offsets fit in 32 bits (checked on the host): uniform base + 32-bit lane offset
  int xoff;
  int ih0 = 0, iw0 = 0;
  // EP (pooled epilogue): N tile nt = (image, pooled tile row, pooled tile column); its BN columns
  // are an ep_rc x ep_cc patch of conv outputs (row-major), the conv pixels that the tile's
  // ep_pr x ep_pc pooled outputs read
  // (3x3 / stride-2 pool: EPOOL_PR x EPOOL_PC pooled outputs from an EPOOL_RC x EPOOL_CC patch)
  int ep_img = 0, ep_ph0 = 0, ep_pw0 = 0;
  if (EP) {
    const int tpi = p.ep_tr * p.ep_tc;
    ep_img = nt / tpi;
    const int t = nt - ep_img * tpi;
    ep_ph0 = (t / p.ep_tc) * EPOOL_PR;
    ep_pw0 = (t - (t / p.ep_tc) * p.ep_tc) * EPOOL_PC;
    const int prc = bcol / EPOOL_CC, pcc = bcol - prc * EPOOL_CC;
    const int oh = ep_ph0 * 2 - p.ep_pt + prc, ow = ep_pw0 * 2 - p.ep_pl + pcc;
    bn_ok = ep_img < p.N && bcol < EPOOL_RC * EPOOL_CC && (unsigned)oh < (unsigned)p.Ho && (unsigned)ow < (unsigned)p.Wo;
    xoff = ep_img * (int)p.x_nstride;
    if (BMODE == B1X1) {
      xoff += oh * p.W + ow;
    } else {
      ih0 = oh * p.sh - p.pt;
      iw0 = ow * p.sw - p.pl;
      xoff += ih0 * p.W + iw0;
    }
    if (!bn_ok) xoff = 0;
  } else {
    const int nn = bn_ok ? bn : 0;
    const int img = nn / YPS;
    const int pix = nn - img * YPS;  // pix >= Ho*Wo: a pad column, computed and never read
    xoff = img * (int)p.x_nstride;
    if (BMODE == B1X1) {
      xoff += pix;
    } else {
      const int oh = pix / p.Wo, ow = pix - oh * p.Wo;
      ih0 = oh * p.sh - p.pt;
      iw0 = ow * p.sw - p.pl;
      xoff += ih0 * p.W + iw0;
    }
  }
  const float* __restrict__ x = p.x;
  const float* __restrict__ wp = p.wp;
  const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.wp), (short)0, (int)(((p.K + 31) & ~31) * p.Mp * 4), 0x00020000);
  // DMA: buffer resource over x's valid extent (bytes < 2^32, checked on the host); each wave
  // writes 64 consecutive columns of one B row
  const __amdgpu_buffer_rsrc_t xrsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.x), (short)0, (int)p.x_bytes, 0x00020000);
  const int wcol0 = bcol & ~63;
  // the gather table through the constant address space: k is wave-uniform, so the entries
  // come in by scalar loads (s_load) into SGPRs instead of LDS / vector round trips
  typedef const __attribute__((address_space(4))) long long* ktab_cptr;  // int2 {x, y} as one 64-bit word
  const ktab_cptr ktab = (ktab_cptr)p.ktab;


  // Branch-free loads: every lane loads (masked lanes from x[0]) and selects 0 afterwards, so
  // the whole tile's loads issue back to back.
#define ORE_LOAD_TILE(RA, RB, ROK, K0, DBUF)                                                         \
  {                                                                                                  \
    const int k0_ = (K0);                                                                            \
    _Pragma("unroll") for (int v_ = 0; v_ < AVEC; ++v_) {                                            \
      /* the A tile's tail float4s (AF4 % 256 != 0) reload element 0 and are not stored */           \
      const int e_ = (AF4 % 256 == 0 || tid + v_ * 256 < AF4) ? tid + v_ * 256 : 0;                  \
      const int kk = e_ / (BM / 4), mm = (e_ % (BM / 4)) * 4;                                        \
      if (ADMA) {                                                                                    \
        /* wave-uniform: a wave's 64 chunks are all inside or all past the tile */                  \
        if (AF4 % 256 == 0 || v_ * 256 + wave * 64 < AF4)                                            \
          __builtin_amdgcn_raw_ptr_buffer_load_lds(                                                  \
              wrsrc, (__attribute__((address_space(3))) void*)(&As[(DBUF)][0][0] + (v_ * 256 + wave * 64) * 4), 16, \
              ((k0_ + kk) * p.Mp + m0 + mm) * 4, 0, 0, 0);                                           \
      } else {                                                                                       \
        RA[v_] = *reinterpret_cast<const floatx4*>(wp + (unsigned)((k0_ + kk) * p.Mp + m0 + mm));    \
      }                                                                                              \
    }                                                                                                \
    _Pragma("unroll") for (int j = 0; j < BLOADS; ++j) {                                             \
      const int k = k0_ + krow + j * BROWS;                                                          \
      bool ok;                                                                                       \
      int off;                                                                                       \
      if (BMODE == B1X1) {                                                                           \
        ok = bn_ok & (k < K);                                                                        \
        off = xoff + k * XPS;                                                                        \
      } else {                                                                                       \
        const long long w_ = ktab[k];                                                                \
        const int ex_ = (int)w_, ey_ = (int)(w_ >> 32);                                              \
        const int r = ey_ >> 16, s = ey_ & 0xffff;                                                   \
        ok = bn_ok & ((unsigned)(ih0 + r) < (unsigned)p.H) & ((unsigned)(iw0 + s) < (unsigned)p.W);  \
        off = xoff + ex_;                                                                            \
      }                                                                                              \
      if (DMA) {                                                                                     \
        __builtin_amdgcn_raw_ptr_buffer_load_lds(                                                    \
            xrsrc, (__attribute__((address_space(3))) void*)&Bs[(DBUF)][krow + j * BROWS][wcol0], 4,   \
            ok ? off * 4 : (int)0x80000000, 0, 0, 0);                                                \
      } else {                                                                                       \
        RB[j] = x[(unsigned)(ok ? off : 0)];                                                         \
        ROK[j] = ok; /* the zero select happens at the LDS store, after the MFMAs */                 \
      }                                                                                              \
    }                                                                                                \
  }
#define ORE_STORE_TILE(RA, RB, ROK, BUF)                                                             \
  {                                                                                                  \
    if (!ADMA)                                                                                       \
      _Pragma("unroll") for (int v_ = 0; v_ < AVEC; ++v_) {                                          \
        const int e_ = tid + v_ * 256;                                                               \
        const int kk = e_ / (BM / 4), mm = (e_ % (BM / 4)) * 4;                                      \
        if (AF4 % 256 == 0 || e_ < AF4) *reinterpret_cast<floatx4*>(&As[BUF][kk][mm]) = RA[v_];      \
      }                                                                                              \
    if (!DMA)                                                                                        \
      _Pragma("unroll") for (int j = 0; j < BLOADS; ++j)                                             \
        Bs[BUF][krow + j * BROWS][bcol] = ROK[j] ? RB[j] : 0.0f;                                     \
  }

  floatx16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  const int ntk = (K + BK - 1) / BK;
  {
    floatx4 ra[AVEC];
    float rb[BLOADS];
    bool rok[BLOADS];
    ORE_LOAD_TILE(ra, rb, rok, 0, 0);
    ORE_STORE_TILE(ra, rb, rok, 0);
    if (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the B tile has landed in LDS
  }
  __syncthreads();
  const int lrow = lane >> 5, lcol = lane & 31;
// fragments for k-step kk+2 are read from LDS before the MFMAs of k-step kk are issued
// KEND: k-steps of this tile that carry data (BK except on the last tile, where the zero rows
// past K are skipped: conv1's K = 147 pads to 160)
#define ORE_COMPUTE_TILE(BUF, KEND)                                                                  \
  {                                                                                                  \
    float af[2][FM], bf[2][FN];                                                                      \
    _Pragma("unroll") for (int i = 0; i < FM; ++i) af[0][i] = As[BUF][lrow][wm0 + i * 32 + lcol];    \
    _Pragma("unroll") for (int j = 0; j < FN; ++j) bf[0][j] = Bs[BUF][lrow][wn0 + j * 32 + lcol];    \
    _Pragma("unroll") for (int kk = 0; kk < BK; kk += 2) {                                           \
      const int cur = (kk >> 1) & 1;                                                                 \
      if (kk + 2 < BK) {                                                                             \
        _Pragma("unroll") for (int i = 0; i < FM; ++i)                                               \
          af[cur ^ 1][i] = As[BUF][kk + 2 + lrow][wm0 + i * 32 + lcol];                              \
        _Pragma("unroll") for (int j = 0; j < FN; ++j)                                               \
          bf[cur ^ 1][j] = Bs[BUF][kk + 2 + lrow][wn0 + j * 32 + lcol];                              \
      }                                                                                              \
      ORE_FRAG_PIN; /* next k-step's fragment reads stay ahead of this k-step's MFMAs */             \
      if (kk < (KEND)) {                                                                             \
        _Pragma("unroll") for (int i = 0; i < FM; ++i)                                               \
        _Pragma("unroll") for (int j = 0; j < FN; ++j)                                               \
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[cur][i], bf[cur][j], acc[i][j], 0, 0, 0); \
      }                                                                                              \
    }                                                                                                \
  }
  // steady state: prefetch tile t+1 into registers, MFMAs on tile t, publish t+1 to LDS
  for (int t = 0; t < ntk - 1; ++t) {
    const int buf = t & 1;
    floatx4 ra[AVEC];
    float rb[BLOADS];
    bool rok[BLOADS];
    ORE_LOAD_TILE(ra, rb, rok, (t + 1) * BK, buf ^ 1);
    __builtin_amdgcn_sched_barrier(0);  // keep the next tile's loads ahead of this tile's MFMAs
    ORE_COMPUTE_TILE(buf, BK);
    ORE_STORE_TILE(ra, rb, rok, buf ^ 1);
    if (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  {
    const int kend = __builtin_amdgcn_readfirstlane((K - (ntk - 1) * BK + 1) & ~1);
    ORE_COMPUTE_TILE((ntk - 1) & 1, kend);
  }
#undef ORE_COMPUTE_TILE
#undef ORE_LOAD_TILE
#undef ORE_STORE_TILE

  // ---- epilogue: + bias, optional Relu, store to NCHW (possibly a channel slice)
  float* __restrict__ y = p.y;
  if constexpr (EP) {
    // pooled epilogue: per 32-row fragment i the block's [32][BN] conv outputs (bias + Relu; 0 for
    // patch positions outside the conv plane = the pool's zero padding, max_pool_op.rs:265-276) go
    // to LDS, then each of the tile's 6 x 9 pooled outputs per row takes the 3x3 max starting from
    // -FLT_MAX (:337) and is stored to the pooled NCHW plane.  The pre-pool tensor never reaches HBM.
    static_assert(WM == 1, "all waves share the tile's rows");
    constexpr int SROW = BN + 4;
    static_assert(32 * SROW <= MAIN_FLOATS && EPOOL_RC * EPOOL_CC <= BN, "pooled epilogue staging");
    __syncthreads();  // every wave is done with the A/B tiles
    const int ohb = ep_ph0 * 2 - p.ep_pt, owb = ep_pw0 * 2 - p.ep_pl;  // conv position of patch (0, 0)
    bool cok[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = wn0 + j * 32 + lcol;
      const int prc = col / EPOOL_CC, pcc = col - prc * EPOOL_CC;
      cok[j] = col < EPOOL_RC * EPOOL_CC && (unsigned)(ohb + prc) < (unsigned)p.Ho && (unsigned)(owb + pcc) < (unsigned)p.Wo;
    }
    const int pch = tid >> 3, sub = tid & 7;  // pooling: 8 threads per channel row
#pragma unroll  // static acc indices (a runtime i would move the accumulators to scratch)
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int r = (e & 3) + 8 * (e >> 2) + 4 * lrow;
          float v = acc[i][j][e] + sbias[i * 32 + r];
          if (p.relu) v = fmaxf(v, 0.0f);
          smem[r * SROW + wn0 + j * 32 + lcol] = cok[j] ? v : 0.0f;
        }
      __syncthreads();
      const int m = m0 + i * 32 + pch;
      const float* row = smem + pch * SROW;
#pragma unroll
      for (int q = sub; q < EPOOL_PR * EPOOL_PC; q += 8) {
        const int a = q / EPOOL_PC, b = q - a * EPOOL_PC;
        const float* w0 = row + (2 * a) * EPOOL_CC + 2 * b;
        float mx = -FLT_MAX;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int sx = 0; sx < 3; ++sx) mx = fmaxf(mx, w0[r * EPOOL_CC + sx]);
        const int ph = ep_ph0 + a, pw = ep_pw0 + b;
        if (ph < p.ep_Ho && pw < p.ep_Wo && m < p.M && ep_img < p.N)
          y[(unsigned)(ep_img * (int)p.y_nstride + m * YPS + ph * p.ep_Wo + pw)] = mx;
      }
      __syncthreads();
    }
    return;
  }
  if (p.vec_out) {
    // 16-B stores: each wave stages 32 output rows x TN pixels in its own LDS slice (column
    // halves swapped every 4 rows so the two lane halves' writes hit different banks), then
    // writes whole pixel runs with float4 stores.  Host guarantees y_ps % 4 == 0, 16-B aligned
    // image/plane bases and Ntot % 4 == 0, so no float4 straddles an image.
    __syncthreads();  // every wave is done with the A/B tiles
    float* stg = smem + wave * (32 * TN);
    constexpr int V4 = TN / 4;            // float4 per staged row
    constexpr int RPI = 64 / V4;          // rows per wave-instruction
    // staging address of (row r, column c): rows r and r + 4 (the two lane halves of one MFMA
    // output register) land in opposite halves of the 64 banks
#define ORE_STG(R, C) (TN >= 64 ? (R) * TN + ((C) ^ ((((R) >> 2) & 1) * 32)) : ((R) ^ (((R) >> 2) & 1)) * TN + (C))
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int r = (e & 3) + 8 * (e >> 2) + 4 * lrow;
          float v = acc[i][j][e] + sbias[wm0 + i * 32 + r];
          if (p.relu) v = fmaxf(v, 0.0f);
          stg[ORE_STG(r, j * 32 + lcol)] = v;
        }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int c4 = (lane % V4) * 4;
      const int n = n0 + wn0 + c4;
      const int img = n / YPS;
      const int pix = n - img * YPS;
      const bool nok = n < p.Ntot;
#pragma unroll
      for (int rr = 0; rr < 32; rr += RPI) {
        const int r = rr + lane / V4;
        const int m = m0 + wm0 + i * 32 + r;
        const floatx4 v = *reinterpret_cast<const floatx4*>(stg + ORE_STG(r, c4));
        if (nok && m < p.M)
          *reinterpret_cast<floatx4*>(y + (unsigned)(img * (int)p.y_nstride + m * YPS + pix)) = v;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#undef ORE_STG
    return;
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn0 + j * 32 + lcol;
    if (n >= p.Ntot) continue;
    const int img = n / YPS;
    const int pix = n - img * YPS;
    const unsigned yb = (unsigned)(img * (int)p.y_nstride + pix);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int ml = wm0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * lrow;
        if (m0 + ml < p.M) {
          float v = acc[i][j][e] + sbias[ml];
          if (p.relu) v = fmaxf(v, 0.0f);
          y[yb + (unsigned)((m0 + ml) * YPS)] = v;
        }
      }
    }
  }
}

// ------------------------------------------------------------------ gather table
// ktab[k] = {c*x_ps + r*W + s, (r << 16) | s} for k = (c, r, s) < K; padded entries (k >= K)
// carry r = 1 << 14 so the bounds test of the gather fails and they read as zero.
__global__ __launch_bounds__(256) void ktab_kernel(int2* __restrict__ ktab, int K, int Kp, int kh, int kw, int ps,
                                                   int W) {
  for (int k = blockIdx.x * 256 + threadIdx.x; k < Kp; k += gridDim.x * 256) {
    int2 e = make_int2(0, (1 << 14) << 16);
    if (k < K) {
      const int KK = kh * kw;
      const int c = k / KK, rs = k - c * KK, r = rs / kw, s = rs - r * kw;
      e = make_int2(c * ps + r * W + s, (r << 16) | s);
    }
    ktab[k] = e;
  }
}

void launch_ktab(int2* ktab, int K, int kh, int kw, int x_ps, int W, hipStream_t s) {
  const int Kp = conv_packed_kp(K);
  hipLaunchKernelGGL(ktab_kernel, dim3((Kp + 255) / 256), dim3(256), 0, s, ktab, K, Kp, kh, kw, x_ps, W);
}

// ------------------------------------------------------------------ weight packing
// src ONNX [M][K] (kmajor_src = 0) or MatMul [K][M] (kmajor_src = 1) -> Wp[Kp][Mp], zero padded.
__global__ __launch_bounds__(256) void pack_weights_kernel(const float* __restrict__ w, float* __restrict__ wp,
                                                           int M, int K, int Mp, int Kp, int kmajor_src) {
  const long long total = (long long)Kp * Mp;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int k = (int)(i / Mp), m = (int)(i - (long long)k * Mp);
    float v = 0.0f;
    if (k < K && m < M) v = kmajor_src ? w[(long long)k * M + m] : w[(long long)m * K + k];
    wp[i] = v;
  }
}

int conv_packed_mp(int M) { return (M + 127) / 128 * 128; }
int conv_packed_kp(int K) { return (K + 31) / 32 * 32; }

void launch_pack_weights(const float* w, bool kmajor_src, int M, int K, int Mp, float* wp, hipStream_t s) {
  const int Kp = conv_packed_kp(K);
  long long total = (long long)Mp * Kp;
  long long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pack_weights_kernel, dim3((unsigned)blocks), dim3(256), 0, s, w, wp, M, K, Mp, Kp,
                     kmajor_src ? 1 : 0);
}

// the B tile by LDS-DMA (buffer_load ... lds): the host launches image chunks whose x extent fits the
// buffer resource (run_conv), so x_bytes > 0 here
template <int BM, int BN, int WM, int WN>
static void launch_conv_cfg(const ConvParams& p0, hipStream_t s) {
  constexpr int BK = 16;
  ConvParams p = p0;
  p.mtiles = (p.M + BM - 1) / BM;
  p.ntiles = (int)((p.Ntot + BN - 1) / BN);
  dim3 grid(p.mtiles * p.ntiles), block(256);
  if (p.is1x1)
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, BK, B1X1, 1>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, BK, BGATHER, 1>), grid, block, 0, s, p);
}

// Conv + MaxPool in one launch (ORE_FUSE_CONV_POOL): 1x4-wave tiles of BM x 256 (the N tile is a
// conv-output patch, run_conv_epool picks its shape)
template <int BM>
static void launch_conv_epool_cfg(const ConvParams& p0, hipStream_t s) {
  constexpr int BK = 16, BN = 256;
  ConvParams p = p0;
  p.mtiles = (p.M + BM - 1) / BM;
  p.ntiles = p.N * p.ep_tr * p.ep_tc;
  dim3 grid(p.mtiles * p.ntiles), block(256);
  if (p.is1x1)
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, 1, 4, BK, B1X1, 1, 1>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, 1, 4, BK, BGATHER, 1, 1>), grid, block, 0, s, p);
}

void launch_conv_epool(const ConvParams& p, hipStream_t s) {
  int v = p.ep_variant;
  if (p.sq1) {  // the fused squeeze: the band walker (variant 8) or the window kernel
    if (v == EPOOL_BAND_VARIANT && p.wc1 && conv_band_pool_f32_eligible(p, p.sq1)) {
      launch_conv_band_pool_f32(p, p.wc1, *p.sq1, s);
      last_conv_tile = EPOOL_BAND_TILE;
    } else if (p.wc1 && conv_win_pool_f32_eligible(p, p.sq1)) {
      launch_conv_win_pool_f32(p, p.wc1, p.sq1, s);
      last_conv_tile = EPOOL_WIN_TILE;
    } else {
      last_conv_tile = -2;  // declined: the walker reports an error
    }
    return;
  }
  // auto: a walker block owns a whole image (x its m tile), so below ~one block per CU (batch < 128
  // for conv1) the patch kernel's many small tiles fill the chip better
  if (v == 0 && p.N >= 128)
    v = conv_pool_stream_eligible(p, 3) ? 3 : conv_pool_stream_eligible(p, 4) ? 4 : conv_pool_stream_eligible(p, 2) ? 2 : 1;
  if (v == 0) v = 1;
  if (v == EPOOL_WIN_VARIANT) {
    if (p.wc1 && conv_win_pool_f32_eligible(p)) {
      launch_conv_win_pool_f32(p, p.wc1, nullptr, s);
      last_conv_tile = EPOOL_WIN_TILE;
      return;
    }
    v = 1;
  }
  if (v >= 2 && conv_pool_stream_eligible(p, v)) {
    launch_conv_pool_stream(p, v, s);
    last_conv_tile = EPOOL_TILE_BASE + v;
    return;
  }
  last_conv_tile = EPOOL_TILE_BASE + 1;
  // rows per tile: 96 when it divides the channel count (conv1's 96), else 128, or 32 for M <= 32
  if (p.M <= 32)
    launch_conv_epool_cfg<32>(p, s);
  else if (p.M % 96 == 0 || p.M < 96)
    launch_conv_epool_cfg<96>(p, s);
  else
    launch_conv_epool_cfg<128>(p, s);
}

// Block tiles, chosen per layer to minimise the padded output channels (MFMA work on rows
// >= M is wasted): BM = 128 (2x2 waves of 64x64), 96 (1x4 waves of 96x32), 64 (2x2 of 32x64),
// 32 (1x4 of 32x64).  Ties go to the larger tile (more reuse of each B element).
int conv_tile_config(int M) {
  static const int bms[4] = {128, 96, 64, 32};
  int best = 0;
  long long best_rows = 1LL << 60;
  for (int i = 0; i < 4; ++i) {
    const long long rows = (long long)((M + bms[i] - 1) / bms[i]) * bms[i];
    if (rows < best_rows) { best_rows = rows; best = i; }
  }
  return best;
}

static const int CFG_BM[4] = {128, 96, 64, 32};


ConvPlan plan_conv(int M, int C, int H, int W, int kh, int kw, int sh, int sw, int pt, int pl, int Ho, int Wo,
                   bool is1x1, bool f16, int xmode, bool wino, int forced) {
  (void)pt;
  ConvPlan pln{};
  if (wino && !f16 && conv_wino_geometry(C, kh, kw, sh, sw, pt, pl, H, W, Ho, Wo)) {
    pln.wino = 1;
    pln.cfg = WINO_TILE_BASE + 0;
    if (forced >= WINO_TILE_BASE && forced < WINO_TILE_BASE + WINO_TILES_N) pln.cfg = forced;
    pln.Mp = wino_packed_mp(M);
    pln.krows = 16 * C;  // U is 16 positions x C rows of Mp floats
    return pln;
  }
  pln.f16 = f16 ? 1 : 0;
  pln.xmode = f16 ? xmode : 0;
  pln.cfg = conv_tile_config(M);
  const int K = C * kh * kw;
  // short-K 1x1 layers (SqueezeNet's expand1x1, K <= 64) are epilogue/write bound: the 1x4-wave
  // 96-row tile measured fastest for them even with padded rows (tools/bench_ops.py)
  if (K <= 64 && M >= 64 && is1x1) pln.cfg = 1;
  if (forced >= 0 && forced < (f16 ? CONV_TILES_F16 : CONV_TILES_F32) && !conv_tile_retired(forced)) pln.cfg = forced;
  if (!f16 && is1x1 && forced >= CONV_TILE_SP && forced < CONV_TILE_SP + CONV_TILES_SP) pln.cfg = forced;
  // packed rows cover every block tile's rows (the 96-row tile can pass roundup(M, 128)), so
  // the tile can be changed after packing (ore_model_autotune)
  pln.Mp = conv_packed_mp(M);
  for (int c = 0; c < 4; ++c) {
    const int bm = CFG_BM[c], rows = (M + bm - 1) / bm * bm;
    if (rows > pln.Mp) pln.Mp = rows;
  }
  pln.krows = conv_packed_kp(f16 ? f16_conv_k(xmode, C, kh, kw) : K);
  return pln;
}

size_t conv_packed_bytes(const ConvPlan& pln) {
  return (size_t)pln.krows * pln.Mp * (pln.f16 ? sizeof(_Float16) : sizeof(float));
}

void launch_pack(const float* w, bool kmajor_src, int M, int C, int kh, int kw, const ConvPlan& pln, float* wp,
                 hipStream_t s) {
  if (pln.wino) {
    launch_pack_wino(w, M, C, pln.Mp, wp, s);
    return;
  }
  if (pln.f16) {
    (void)kmajor_src;  // f16 plans are convs only (MatMul stays f32)
    launch_pack_weights_f16(w, pln.xmode, M, C, kh, kw, pln.Mp, wp, s);
    return;
  }
  launch_pack_weights(w, kmajor_src, M, C * kh * kw, pln.Mp, wp, s);
}

thread_local int last_conv_tile = -1;

void launch_conv(const ConvParams& p, const ConvPlan& pln, hipStream_t s) {
  last_conv_tile = pln.cfg;
  if (pln.wino) {  // the caller (run_conv) keeps x_bytes within the buffer range
    int t = pln.cfg - WINO_TILE_BASE;  // the caller (run_conv) checked conv_wino_eligible
    last_conv_tile = WINO_TILE_BASE + t;
    launch_conv_wino(p, t, s);
    return;
  }
  if (pln.f16) {
    launch_conv_f16(p, pln.cfg, pln.xmode, s);
    return;
  }
  if (pln.cfg >= CONV_TILE_STREAM) {
    if (conv_stream_eligible(p, pln.cfg)) {
      launch_conv_stream(p, pln.cfg, s);
      return;
    }
    ConvPlan q = pln;  // not a stream geometry: the LDS-staged kernel
    q.cfg = 0;
    launch_conv(p, q, s);
    return;
  }
  switch (pln.cfg) {
    case 0: launch_conv_cfg<128, 128, 2, 2>(p, s); break;
    case 1: launch_conv_cfg<96, 128, 1, 4>(p, s); break;
    case 2: launch_conv_cfg<64, 128, 2, 2>(p, s); break;
    default: launch_conv_cfg<32, 256, 1, 4>(p, s); break;
  }
}

}  // namespace ore
