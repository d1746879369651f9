// A SqueezeNet fire module fused with the NEXT fire's squeeze (ORE_FUSE_FIRE): one launch computes
//   e1 = Relu(Conv1x1(S; W1, b1)), e3 = Relu(Conv3x3 pad 1(S; W3, b3)),
//   S' = Relu(Conv1x1(Concat(e1, e3); Ws, bs))
// for a 64-pixel column tile per wave.  e1, e3 and their Concat never leave the registers: each 64
// channels of e1 / e3 are computed (the streaming conv's K loop, ore_conv_stream.hip) and at once
// consumed as the B operand of the squeeze's MFMAs.  The reference runs these as five nodes
// (convolution_op.rs:94-517 x3, relu_op.rs:31-33 x3, concatenate_op.rs:22-32); the walker's
// unfused graph writes 2 x (E1 + E3) channels of activations to HBM and reads them back.
//
// Bit-identical to the unfused kernels:
//   * e1 / e3: the same k-ordered MFMA chain per output as the standalone conv (k = c, or (c, r, s)).
//     Only the A-row -> channel map differs: W1 / W3 are packed with the rows of each 64-channel
//     chunk permuted (fire_pack_kernel) so that accumulator row 4 lk + e of fragment f holds channel
//     c0 + 16 f + 4 e + lk.
//   * squeeze: with that map, squeeze k-step t = 4 f + e finds channel c0 + 4 t + lk of the concat in
//     lane group lk -- exactly the operand the streaming 1x1 kernel loads for k = 4 t + lk -- so the
//     squeeze accumulates over the concat channels in ascending order, one fmaf chain as in the
//     standalone squeeze, with its weights in the standard K-major packing (launch_pack).
#include <hip/hip_runtime.h>

#include <float.h>

#include <atomic>
#include <type_traits>

#include "ore_kernels.h"

namespace ore {

typedef float fi_floatx4 __attribute__((ext_vector_type(4)));

// W [M][K] (ONNX conv weights, K = C*kh*kw) -> Wf[Kp][M]: row slot p = c0 + 4 j + f of each 64-row
// chunk c0 holds channel c0 + 16 f + 4 (j & 3) + (j >> 2); rows k >= K zero
__global__ __launch_bounds__(256) void fire_pack_kernel(const float* __restrict__ w, float* __restrict__ wf, int M,
                                                        int K, int Kp) {
  const long long total = (long long)Kp * M;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int k = (int)(i / M), pslot = (int)(i - (long long)k * M);
    const int c0 = pslot & ~63, j = (pslot & 63) >> 2, f = pslot & 3;
    const int ch = c0 + 16 * f + 4 * (j & 3) + (j >> 2);
    wf[i] = k < K ? w[(long long)ch * K + k] : 0.0f;
  }
}

void launch_fire_pack(const float* w, int M, int K, float* wf, hipStream_t s) {
  const int Kp = (K + 31) & ~31;
  long long blocks = ((long long)Kp * M + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(fire_pack_kernel, dim3((unsigned)blocks), dim3(256), 0, s, w, wf, M, K, Kp);
}

// MFS: 16-row fragments of the squeeze output (Ms <= 16 MFS), D: K-loop ring depth
#define ORE_FIRE_MINB 2  // __launch_bounds__ minimum blocks per CU
template <int MFS, int D>
__global__ __launch_bounds__(256, ORE_FIRE_MINB) void fire_kernel(FireParams p) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, rr8 = nwg & 7;
  const int wgid = (xcd < rr8 ? xcd * (q8 + 1) : rr8 * (q8 + 1) + (xcd - rr8) * q8) + (bid >> 3);
  const int ct = wgid * 4 + wave;  // 64-column tile of this wave
  if (ct >= p.ntiles) return;      // wave-uniform; no barrier in this kernel
  const int lk = lane >> 4, lj = lane & 15;
  const int YPS = p.y_ps;

  // this lane's 4 output pixels (the last tile's surplus lanes re-read valid columns, stores masked)
  const int ntot = (int)p.Ntot;
  int col = ct * 64 + 4 * lj;
  const bool cok = col < ntot;
  if (!cok) col = ntot - 4;
  const int img = col / YPS;
  const int pix = col - img * YPS;
  const int ybase = img * (int)p.y_nstride + pix;
  // input byte offsets from the lead-shifted buffer base: 1x1 (channel lk of the k-step) and 3x3
  const int xlead = p.x_lead;
  const int xoff1 = xlead + (img * (int)p.x_nstride + lk * p.x_ps + pix) * 4;
  const int xoff3 = (img * (int)p.x_nstride + pix) * 4;
  unsigned tmask[4];  // bit 3r + s: tap (r, s) of pixel pix + q reads inside the image
  {
    const int oh0 = pix / p.W, ow0 = pix - oh0 * p.W;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool wrap = ow0 + q >= p.W;
      const int oh = oh0 + (wrap ? 1 : 0), ow = ow0 + q - (wrap ? p.W : 0);
      unsigned cm = 0, m = 0;
#pragma unroll
      for (int s = 0; s < 3; ++s) cm |= ((unsigned)(ow - 1 + s) < (unsigned)p.W ? 1u : 0u) << s;
#pragma unroll
      for (int r = 0; r < 3; ++r)
        if (oh < p.H && (unsigned)(oh - 1 + r) < (unsigned)p.H) m |= cm << (r * 3);
      tmask[q] = m;
    }
  }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(reinterpret_cast<const char*>(p.x) - xlead), (short)0, (int)p.x_bytes + xlead, 0x00020000);
  const int K1 = p.C, K3 = 9 * p.C;
  const __amdgpu_buffer_rsrc_t w1r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.w1), (short)0, ((K1 + 31) & ~31) * p.E1 * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t w3r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.w3), (short)0, ((K3 + 31) & ~31) * p.E3 * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t wsr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.ws), (short)0, (((p.E1 + p.E3) + 31) & ~31) * p.Msp * 4, 0x00020000);
  const int tap0 = xlead - (p.W + 1) * 4;  // byte offset of tap (0, 0) from the output pixel (pad 1)

  fi_floatx4 accs[MFS][4];  // the squeeze accumulators: row 4 lk + e of fragment fs, pixel 4 lj + q
#pragma unroll
  for (int fs = 0; fs < MFS; ++fs)
#pragma unroll
    for (int q = 0; q < 4; ++q) accs[fs][q] = fi_floatx4{0.f, 0.f, 0.f, 0.f};

  // ---- one 64-channel chunk of e1 (MODE 0) or e3 (MODE 1): K loop, bias + Relu, squeeze MFMAs
  auto chunk = [&](auto mode_tag, int c0, int cat0) __attribute__((always_inline)) {
    constexpr int MODE = decltype(mode_tag)::value;
    const __amdgpu_buffer_rsrc_t wr = MODE == 0 ? w1r : w3r;
    const int Mrow = MODE == 0 ? p.E1 : p.E3;
    const int nks = (MODE == 0 ? K1 : K3) >> 2;  // host: K % 16 == 0
    const int aoff = (lk * Mrow + c0 + 4 * lj) * 4, astep = 16 * Mrow;
    const int xstep = 16 * p.x_ps;
    int tt = lk, cx = 0;  // 3x3: tap and channel byte offset of k = 4 s + lk
    fi_floatx4 acc[4][4];
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[f][q] = fi_floatx4{0.f, 0.f, 0.f, 0.f};
    fi_floatx4 rb[D], ra[D];
    int rt[D];
#define FI_LOAD(SLOT, S)                                                                                 \
    {                                                                                                    \
      const int s_ = (S);                                                                                \
      ra[SLOT] = __builtin_bit_cast(fi_floatx4, __builtin_amdgcn_raw_buffer_load_b128(wr, aoff, s_ * astep, 0)); \
      if constexpr (MODE == 0) {                                                                         \
        rb[SLOT] = __builtin_bit_cast(fi_floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, xoff1, s_ * xstep, 0)); \
      } else {                                                                                           \
        const int r_ = (int)(__umul24((unsigned)tt, 11u) >> 5);                                          \
        const int to_ = cx + tap0 + 4 * ((int)__umul24((unsigned)r_, (unsigned)(p.W - 3)) + tt);         \
        rb[SLOT] = __builtin_bit_cast(fi_floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, xoff3 + to_, 0, 0)); \
        rt[SLOT] = tt;                                                                                   \
        tt += 4;                                                                                         \
        if (tt >= 9) { tt -= 9; cx += 4 * p.x_ps; }                                                      \
      }                                                                                                  \
    }
#define FI_MFMA(SLOT)                                                                                    \
    {                                                                                                    \
      if constexpr (MODE == 1) {                                                                         \
        const int4 v_ = __builtin_bit_cast(int4, rb[SLOT]);                                              \
        int4 w_;                                                                                         \
        w_.x = v_.x & __builtin_amdgcn_sbfe((int)tmask[0], rt[SLOT], 1);                                 \
        w_.y = v_.y & __builtin_amdgcn_sbfe((int)tmask[1], rt[SLOT], 1);                                 \
        w_.z = v_.z & __builtin_amdgcn_sbfe((int)tmask[2], rt[SLOT], 1);                                 \
        w_.w = v_.w & __builtin_amdgcn_sbfe((int)tmask[3], rt[SLOT], 1);                                 \
        rb[SLOT] = __builtin_bit_cast(fi_floatx4, w_);                                                   \
      }                                                                                                  \
      __builtin_amdgcn_s_setprio(1);                                                                     \
      _Pragma("unroll") for (int f = 0; f < 4; ++f)                                                      \
      _Pragma("unroll") for (int q = 0; q < 4; ++q)                                                      \
        acc[f][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[SLOT][f], rb[SLOT][q], acc[f][q], 0, 0, 0);  \
      __builtin_amdgcn_s_setprio(0);                                                                     \
    }
#pragma unroll
    for (int d = 0; d < D; ++d) FI_LOAD(d, d);
    for (int s0 = 0; s0 < nks - D; s0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        FI_MFMA(d);
        __builtin_amdgcn_sched_barrier(0);
        FI_LOAD(d, s0 + D + d);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // the squeeze's A operand (16 k-steps of this chunk) in 4 groups of 4 k-steps, one group ahead;
    // group 0 is issued before the ring drain.  (Loaded at their use, the compiler put a vmcnt(0)
    // behind every pair: 8 exposed L2 round trips per chunk, ~20 % of the module's time.)
    const int saoff = ((cat0 + lk) * p.Msp + MFS * lj) * 4;
    float asq[2][4][MFS];
    auto sload = [&](float (&dst)[4][MFS], int g) __attribute__((always_inline)) {
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const int so = saoff + (4 * g + tt) * 16 * p.Msp;
        if constexpr (MFS == 4) {
          const fi_floatx4 v = __builtin_bit_cast(fi_floatx4, __builtin_amdgcn_raw_buffer_load_b128(wsr, so, 0, 0));
          dst[tt][0] = v[0]; dst[tt][1] = v[1]; dst[tt][2] = v[2]; dst[tt][3] = v[3];
        } else if constexpr (MFS == 3) {
          typedef float f3 __attribute__((ext_vector_type(3)));
          const f3 v = __builtin_bit_cast(f3, __builtin_amdgcn_raw_buffer_load_b96(wsr, so, 0, 0));
          dst[tt][0] = v[0]; dst[tt][1] = v[1]; dst[tt][2] = v[2];
        } else if constexpr (MFS == 2) {
          typedef float f2 __attribute__((ext_vector_type(2)));
          const f2 v = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(wsr, so, 0, 0));
          dst[tt][0] = v[0]; dst[tt][1] = v[1];
        } else {
          dst[tt][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wsr, so, 0, 0));
        }
      }
    };
    sload(asq[0], 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int d = 0; d < D; ++d) FI_MFMA(d);
#undef FI_LOAD
#undef FI_MFMA
    // bias + Relu: accumulator row 4 lk + e of fragment f is channel c0 + 16 f + 4 e + lk
    const float* __restrict__ bias = MODE == 0 ? p.b1 : p.b3;
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float b = bias[c0 + 16 * f + 4 * e + lk];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[f][q][e] = fmaxf(acc[f][q][e] + b, 0.0f);
      }
    // squeeze over these 64 concat channels: k-step t = 4 f + e takes concat channel cat0 + 4 t + lk
    // from lane group lk (the value acc[f][q][e]); A = Ws packed K-major (row cat0 + 4 t + lk)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (g + 1 < 4) sload(asq[(g + 1) & 1], g + 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const int t = 4 * g + tt;
#pragma unroll
        for (int fs = 0; fs < MFS; ++fs)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            accs[fs][q] =
                __builtin_amdgcn_mfma_f32_16x16x4f32(asq[g & 1][tt][fs], acc[t >> 2][q][t & 3], accs[fs][q], 0, 0, 0);
      }
    }
  };
  for (int c0 = 0; c0 < p.E1; c0 += 64) chunk(std::integral_constant<int, 0>{}, c0, c0);
  for (int c0 = 0; c0 < p.E3; c0 += 64) chunk(std::integral_constant<int, 1>{}, c0, p.E1 + c0);

  // S' = Relu(squeeze + bs): squeeze channel MFS (4 lk + e) + fs, pixels 4 lj + q -> 16-B stores
  float* __restrict__ y = p.y;
#pragma unroll
  for (int fs = 0; fs < MFS; ++fs)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = MFS * (4 * lk + e) + fs;
      if (m >= p.Ms) continue;
      const float b = p.bs[m];
      fi_floatx4 v = {accs[fs][0][e] + b, accs[fs][1][e] + b, accs[fs][2][e] + b, accs[fs][3][e] + b};
      v[0] = fmaxf(v[0], 0.0f); v[1] = fmaxf(v[1], 0.0f); v[2] = fmaxf(v[2], 0.0f); v[3] = fmaxf(v[3], 0.0f);
      if (cok) *reinterpret_cast<fi_floatx4*>(y + (unsigned)(ybase + m * YPS)) = v;
    }
}


// ---- pooled form: fire module -> 3x3 / stride-2 MaxPool -> the next squeeze (SqueezeNet fire4 ->
// pool3 -> fire5/squeeze1x1).  The unfused f32 graph runs the two expands with pooled epilogues
// (conv_pool_stream_kernel, 2 launches, the pooled concat written to HBM) and the squeeze as a third
// launch that reads it back.  Here one workgroup (8 waves) owns a band of PR pooled rows of one image:
//   * the band's conv rows cr0 .. cr1 are a contiguous run of the NCHW plane; wave w computes its
//     64 pixels of it with fire_kernel's streaming K loop (same operands, same k = (c, r, s) chains);
//   * per 64-channel chunk of the concat (e1 chunks, then e3 chunks) every wave writes bias + Relu
//     of its pixels to an LDS conv tile [64 channels][FP_TS] (131 KB: one workgroup per CU, two
//     waves per SIMD), barrier; then waves 0-3 take the 3x3 maxima (from -FLT_MAX, outside taps read
//     0.0f from a zeroed pad slot: maxpool_kernel's arithmetic) of their two 16-pixel pooled
//     fragments and run the chunk's 16 squeeze k-steps (k = concat channel, ascending over the
//     chunks: the standalone 1x1 conv's chain) while waves 4-7 already run the next chunk's K loop;
//   * a barrier before the next tile write frees the tile.
// Bit-identical to the two pooled-epilogue convs + the separate squeeze (tests/test_model_gpu.py).
// conv tile row stride FP_TS (floats) odd: the pooling reads (lane groups of 32 = two channel rows x 16
// pooled pixels two columns apart) of the second row land on the odd banks; with a multiple of 4 (16-B
// stores) both rows shared the even banks, a 2-way conflict on every read
constexpr int FP_WAVES = 8, FP_PIX = 64 * FP_WAVES, FP_TS = FP_PIX + 1;
constexpr int FP_LDS = 64 * FP_TS * 4;

#define ORE_FP_NG 2  // pooled fragments per pooling wave (2: waves 0-3 pool, 1: all 8)
template <int MFS, int D>
__global__ __launch_bounds__(512, 1) void fire_pool_kernel(FireParams p) {
  constexpr int NG = ORE_FP_NG;
  extern __shared__ __attribute__((aligned(16))) float fp_tile[];
  const int lane = threadIdx.x & 63, lk = lane >> 4, lj = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = p.H, W = p.W, Wp = p.Wp;
  const int nbands = (p.Hp + p.PR - 1) / p.PR;
  const int img = blockIdx.x / nbands, band = blockIdx.x - img * nbands;
  const int pr0 = band * p.PR, npr = min(p.PR, p.Hp - pr0);
  const int cr0 = max(0, 2 * pr0 - p.ppt), cr1 = min(H - 1, 2 * (pr0 + npr - 1) - p.ppt + 2);
  const int ncp = (cr1 - cr0 + 1) * W;  // conv pixels of the band (<= FP_PIX: host)
  const bool clive = wave * 64 < ncp;   // a wave with none of them skips the K loops
  if (threadIdx.x < 64) fp_tile[threadIdx.x * FP_TS + FP_PIX] = 0.0f;  // pad slots: the pool's outside taps

  // ---- expand operands (fire_kernel's): this lane's 4 conv pixels pix .. pix + 3 of the plane
  const int pix = cr0 * W + wave * 64 + 4 * lj;
  const int xlead = p.x_lead;
  const int xoff1 = xlead + (img * (int)p.x_nstride + lk * p.x_ps + pix) * 4;
  const int xoff3 = (img * (int)p.x_nstride + pix) * 4;
  unsigned tmask[4];
  {
    const int oh0 = pix / W, ow0 = pix - oh0 * W;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool wrap = ow0 + q >= W;
      const int oh = oh0 + (wrap ? 1 : 0), ow = ow0 + q - (wrap ? W : 0);
      unsigned cm = 0, m = 0;
#pragma unroll
      for (int s = 0; s < 3; ++s) cm |= ((unsigned)(ow - 1 + s) < (unsigned)W ? 1u : 0u) << s;
#pragma unroll
      for (int r = 0; r < 3; ++r)
        if (oh < H && (unsigned)(oh - 1 + r) < (unsigned)H) m |= cm << (r * 3);
      tmask[q] = m;
    }
  }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(reinterpret_cast<const char*>(p.x) - xlead), (short)0, (int)p.x_bytes + xlead, 0x00020000);
  const int K1 = p.C, K3 = 9 * p.C;
  const __amdgpu_buffer_rsrc_t w1r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.w1), (short)0, ((K1 + 31) & ~31) * p.E1 * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t w3r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.w3), (short)0, ((K3 + 31) & ~31) * p.E3 * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t wsr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.ws), (short)0, (((p.E1 + p.E3) + 31) & ~31) * p.Msp * 4, 0x00020000);
  const int tap0 = xlead - (W + 1) * 4;

  // ---- pooled fragments: waves 0 .. 8 / NG - 1 take NG 16-pixel fragments each (fragment NG wave + g,
  // pooled pixel kp = 16 (NG wave + g) + lj of the band)
  const int P = npr * Wp, nfrag = (P + 15) >> 4;
  const bool pwave = wave < 8 / NG && NG * wave < nfrag;
  int tap[NG][9];  // conv-tile offsets of the 9 window taps (channel row lk; outside taps: the pad slot)
  int kp[NG];
  bool gon[NG];    // (wave-uniform) fragment g has pixels
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    kp[g] = 16 * (NG * wave + g) + lj;
    gon[g] = NG * wave + g < nfrag;
    const int kk = kp[g] < P ? kp[g] : 0;
    const int pa = pr0 + kk / Wp, pb = kk - (kk / Wp) * Wp;
    const int ih0 = 2 * pa - p.ppt, iw0 = 2 * pb - p.ppl;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int ih = ih0 + r, iw = iw0 + s;
        const bool in = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        tap[g][3 * r + s] = lk * FP_TS + (in ? (ih - cr0) * W + iw : FP_PIX);
      }
  }
  fi_floatx4 accs[MFS][NG];
#pragma unroll
  for (int fs = 0; fs < MFS; ++fs)
#pragma unroll
    for (int g = 0; g < NG; ++g) accs[fs][g] = fi_floatx4{0.f, 0.f, 0.f, 0.f};

  auto chunk = [&](auto mode_tag, int c0, int cat0) __attribute__((always_inline)) {
    constexpr int MODE = decltype(mode_tag)::value;
    const __amdgpu_buffer_rsrc_t wr = MODE == 0 ? w1r : w3r;
    const int Mrow = MODE == 0 ? p.E1 : p.E3;
    const int nks = (MODE == 0 ? K1 : K3) >> 2;
    const int aoff = (lk * Mrow + c0 + 4 * lj) * 4, astep = 16 * Mrow;
    const int xstep = 16 * p.x_ps;
    int tt = lk, cx = 0;
    fi_floatx4 acc[4][4];
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[f][q] = fi_floatx4{0.f, 0.f, 0.f, 0.f};
    if (clive) {
      fi_floatx4 rb[D], ra[D];
      int rt[D];
#define FP_LOAD(SLOT, S)                                                                                 \
      {                                                                                                  \
        const int s_ = (S);                                                                              \
        ra[SLOT] = __builtin_bit_cast(fi_floatx4, __builtin_amdgcn_raw_buffer_load_b128(wr, aoff, s_ * astep, 0)); \
        if constexpr (MODE == 0) {                                                                       \
          rb[SLOT] = __builtin_bit_cast(fi_floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, xoff1, s_ * xstep, 0)); \
        } else {                                                                                         \
          const int r_ = (int)(__umul24((unsigned)tt, 11u) >> 5);                                        \
          const int to_ = cx + tap0 + 4 * ((int)__umul24((unsigned)r_, (unsigned)(W - 3)) + tt);        \
          rb[SLOT] = __builtin_bit_cast(fi_floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, xoff3 + to_, 0, 0)); \
          rt[SLOT] = tt;                                                                                 \
          tt += 4;                                                                                       \
          if (tt >= 9) { tt -= 9; cx += 4 * p.x_ps; }                                                    \
        }                                                                                                \
      }
#define FP_MFMA(SLOT)                                                                                    \
      {                                                                                                  \
        if constexpr (MODE == 1) {                                                                       \
          const int4 v_ = __builtin_bit_cast(int4, rb[SLOT]);                                            \
          int4 w_;                                                                                       \
          w_.x = v_.x & __builtin_amdgcn_sbfe((int)tmask[0], rt[SLOT], 1);                               \
          w_.y = v_.y & __builtin_amdgcn_sbfe((int)tmask[1], rt[SLOT], 1);                               \
          w_.z = v_.z & __builtin_amdgcn_sbfe((int)tmask[2], rt[SLOT], 1);                               \
          w_.w = v_.w & __builtin_amdgcn_sbfe((int)tmask[3], rt[SLOT], 1);                               \
          rb[SLOT] = __builtin_bit_cast(fi_floatx4, w_);                                                 \
        }                                                                                                \
        __builtin_amdgcn_s_setprio(1);                                                                   \
        _Pragma("unroll") for (int f = 0; f < 4; ++f)                                                    \
        _Pragma("unroll") for (int q = 0; q < 4; ++q)                                                    \
          acc[f][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[SLOT][f], rb[SLOT][q], acc[f][q], 0, 0, 0); \
        __builtin_amdgcn_s_setprio(0);                                                                   \
      }
#pragma unroll
      for (int d = 0; d < D; ++d) FP_LOAD(d, d);
      for (int s0 = 0; s0 < nks - D; s0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
          FP_MFMA(d);
          __builtin_amdgcn_sched_barrier(0);
          FP_LOAD(d, s0 + D + d);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int d = 0; d < D; ++d) FP_MFMA(d);
#undef FP_LOAD
#undef FP_MFMA
    }
    // the squeeze's A operand of this chunk's 16 k-steps (pooling waves), in flight over the barrier
    float asq[16][MFS];
    if (pwave) {
      const int saoff = ((cat0 + lk) * p.Msp + MFS * lj) * 4;
#pragma unroll
      for (int t = 0; t < 16; ++t)
#pragma unroll
        for (int fs = 0; fs < MFS; ++fs)
          asq[t][fs] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wsr, saoff + t * 16 * p.Msp + fs * 4, 0, 0));
    }
    const float* __restrict__ bias = MODE == 0 ? p.b1 : p.b3;
    float bv[4][4];
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[f][e] = bias[c0 + 16 * f + 4 * e + lk];
    __syncthreads();  // the previous chunk's tile is pooled
    // bias + Relu -> conv tile row 16 f + 4 e + lk (= channel c0 + 16 f + 4 e + lk, the permuted packing)
    if (clive) {
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float* row = fp_tile + (16 * f + 4 * e + lk) * FP_TS + wave * 64 + 4 * lj;
#pragma unroll
          for (int q = 0; q < 4; ++q) row[q] = fmaxf(acc[f][q][e] + bv[f][e], 0.0f);
        }
    }
    __syncthreads();  // tile complete
    if (pwave) {
      // squeeze k-step t takes concat channel cat0 + 4 t + lk = tile row 4 t + lk (lane group lk); the
      // window reads of k-step t + 1 are issued before the maxima of t
      float v[2][NG][9];
      auto rd = [&](float (&d)[NG][9], int t) __attribute__((always_inline)) {
        // the k-step's row offset, opaque to the compiler: as constants, the 16 x 9 NG tap addresses
        // (past the 64 KB ds_read offset range from t = 8 on) were hoisted out of the chunk loop and spilled
        int tb = 4 * t * FP_TS;
        __asm__ volatile("" : "+s"(tb));
#pragma unroll
        for (int g = 0; g < NG; ++g)
#pragma unroll
          for (int i = 0; i < 9; ++i) d[g][i] = fp_tile[tap[g][i] + tb];
      };
      rd(v[0], 0);
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        if (t + 1 < 16) rd(v[(t + 1) & 1], t + 1);
        float m[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          m[g] = -FLT_MAX;
#pragma unroll
          for (int i = 0; i < 9; ++i) m[g] = fmaxf(m[g], v[t & 1][g][i]);
        }
#pragma unroll
        for (int fs = 0; fs < MFS; ++fs)
#pragma unroll
          for (int g = 0; g < NG; ++g)
            if (gon[g]) accs[fs][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(asq[t][fs], m[g], accs[fs][g], 0, 0, 0);
      }
    }
  };
  for (int c0 = 0; c0 < p.E1; c0 += 64) chunk(std::integral_constant<int, 0>{}, c0, c0);
  for (int c0 = 0; c0 < p.E3; c0 += 64) chunk(std::integral_constant<int, 1>{}, c0, p.E1 + c0);

  // S' = Relu(squeeze + bs): channel MFS (4 lk + e) + fs, pooled pixel kp[g] of the band
  if (!pwave) return;
  float* __restrict__ y = p.y + (long long)img * p.y_nstride + pr0 * Wp;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    if (kp[g] >= P) continue;
#pragma unroll
    for (int fs = 0; fs < MFS; ++fs)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = MFS * (4 * lk + e) + fs;
        if (m >= p.Ms) continue;
        y[(long long)m * p.y_ps + kp[g]] = fmaxf(accs[fs][g][e] + p.bs[m], 0.0f);
      }
  }
}

bool fire_pool_plan(FireParams* p) {
  // the most pooled rows per band whose conv rows fit the 8 waves' 512 pixels and whose pooled pixels
  // fit the 4 pooling waves' 8 fragments
  p->PR = 0;
  for (int r = 1; r <= p->Hp; ++r) {
    if ((2 * r + 1) * p->W > FP_PIX || r * p->Wp > 128) break;
    p->PR = r;
  }
  return p->PR > 0;
}

bool fire_eligible(const FireParams& p) {
  const uintptr_t xa = reinterpret_cast<uintptr_t>(p.x), ya = reinterpret_cast<uintptr_t>(p.y);
  const bool common = p.E1 % 64 == 0 && p.E3 % 64 == 0 && p.E1 > 0 && p.E3 > 0 && p.Ms >= 1 && p.Ms <= 64 &&
                      p.C % 16 == 0 && p.W >= 3 && p.x_ps % 4 == 0 && p.x_nstride % 4 == 0 && (xa & 15) == 0 &&
                      p.x_bytes > 0 && p.x_guard >= p.x_lead && p.x_bytes + p.x_lead < (1LL << 31) && p.Msp % 4 == 0;
  if (!common) return false;
  if (p.pool)  // 3x3 / stride-2 windows inside the padded plane, each touching the image; scalar stores
    return p.PR >= 1 && (2 * p.PR + 1) * p.W <= FP_PIX && p.PR * p.Wp <= 128 && p.Hp > 0 && p.Wp > 0 && p.ppt >= 0 &&
           p.ppl >= 0 && p.ppt <= 2 && p.ppl <= 2 && 2 * (p.Hp - 1) - p.ppt < p.H && 2 * (p.Wp - 1) - p.ppl < p.W &&
           p.y_ps >= p.Hp * p.Wp && p.N > 0;
  return p.y_ps % 4 == 0 && p.y_nstride % 4 == 0 && (ya & 15) == 0 && p.Ntot % 4 == 0 && p.Ntot >= 4;
}

#define ORE_FIRE_D 4  // K-loop ring depth
#define ORE_FIRE_POOL_D 4  // fire_pool_kernel's ring depth

template <int MFS>
static void launch_fire_cfg(const FireParams& p0, hipStream_t s) {
  FireParams p = p0;
  if (p.pool) {
    // 132 KB of LDS: above the default dynamic-LDS limit, raised once per device
    static std::atomic<unsigned long long> raised{0};
    ore_raise_lds_once(raised, reinterpret_cast<const void*>(&fire_pool_kernel<MFS, ORE_FIRE_POOL_D>), FP_LDS);
    const unsigned grid = (unsigned)(p.N * ((p.Hp + p.PR - 1) / p.PR));
    hipLaunchKernelGGL((fire_pool_kernel<MFS, ORE_FIRE_POOL_D>), dim3(grid), dim3(512), FP_LDS, s, p);
    return;
  }
  p.ntiles = (int)((p.Ntot + 63) / 64);
  hipLaunchKernelGGL((fire_kernel<MFS, ORE_FIRE_D>), dim3((unsigned)((p.ntiles + 3) / 4)), dim3(256), 0, s, p);
}

void launch_fire(const FireParams& p, hipStream_t s) {
  switch ((p.Ms + 15) / 16) {
    case 1: launch_fire_cfg<1>(p, s); break;
    case 2: launch_fire_cfg<2>(p, s); break;
    case 3: launch_fire_cfg<3>(p, s); break;
    default: launch_fire_cfg<4>(p, s); break;
  }
}

}  // namespace ore
