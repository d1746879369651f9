// Internal kernel launch interface (device pointers, resolved integer geometry).  The public
// C ABI (include/ore.h) sits on top of this in ore_api.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>

namespace ore {

// XCD-aware bijective workgroup id: the hardware deals block ids round-robin over the 8 XCDs,
// so neighbouring ids (bands or patches of one image whose input rows overlap) would fetch their
// shared rows into two L2s.  The remap puts consecutive logical ids on one XCD.  Used by the
// persistent f16 conv1 kernel (patches 232 -> 226 us); measured neutral on the f32 conv1 / fire_pool
// kernels and slower on pool_conv1x1_f32 (124 -> 129 us), which keep the plain block id
// (profiles/r02j_xcd_bands_ab.txt).
__device__ __forceinline__ int xcd_block_id() {
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, rr8 = nwg & 7;
  return (xcd < rr8 ? xcd * (q8 + 1) : rr8 * (q8 + 1) + (xcd - rr8) * q8) + (bid >> 3);
}

// f16 epilogue of 8 f32 accumulators: + bias, one rounding to f16, Relu -- as packed pairs
// (v_pk_add_f32, v_cvt_pk_f16_f32, v_pk_max_i16: 1.5 VALU per value against 3 for add / max / cvt).
// Relu after the rounding on the f16 bits as int16 (max with 0) equals Relu before it for every
// finite value: round-to-nearest keeps the sign, a negative or -0 result becomes +0 either way.
// PK_ADD = false keeps the bias adds scalar (v_add_f32): inside kernels whose epilogue runs beside
// MFMAs, where packed f32 VALU costs more than scalar pairs (MI355X_MICROARCH.md 'price of one filler
// beside MFMAs'; measured: the fire f16 kernels 10-20 % slower with v_pk_add_f32)
typedef _Float16 ore_h8 __attribute__((ext_vector_type(8)));
template <bool PK_ADD = true>
__device__ __forceinline__ ore_h8 ore_f16_epilogue8(const float* a, const float* b, bool relu) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  typedef short s2 __attribute__((ext_vector_type(2)));
  typedef short s8 __attribute__((ext_vector_type(8)));
  s8 o;
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    f2 v;
    if constexpr (PK_ADD) {
      v = f2{a[e], a[e + 1]} + f2{b[e], b[e + 1]};
    } else {
      v[0] = a[e] + b[e];
      v[1] = a[e + 1] + b[e + 1];
    }
    s2 q = __builtin_bit_cast(s2, __builtin_convertvector(v, h2));
    if (relu) q = __builtin_elementwise_max(q, s2{0, 0});
    o[e] = q[0];
    o[e + 1] = q[1];
  }
  return __builtin_bit_cast(ore_h8, o);
}

#define ORE_BAND_ID() xcd_block_id()

// Raise a kernel's dynamic-LDS limit (hipFuncAttributeMaxDynamicSharedMemorySize) once per device and
// template instance: the attribute binds to the current device, and one ore_ctx per device may launch
// from its own thread.  `raised` is the caller's per-instance static bit set (one bit per device).
inline void ore_raise_lds_once(std::atomic<unsigned long long>& raised, const void* kernel, int bytes) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  const unsigned long long bit = 1ull << (dev & 63);
  if (!(raised.load(std::memory_order_acquire) & bit)) {
    (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    raised.fetch_or(bit, std::memory_order_acq_rel);
  }
}

// 16-B LDS-DMA (buffer_load_dwordx4 ... lds): lane i's 16 bytes from rsrc + voffset + soffset land at
// LDS byte lds_addr + 16 i (lds_addr, soffset wave-uniform); offsets past the records read 0.  Counted by
// vmcnt like any buffer load; nothing orders a later ds_read behind it but the issuing wave's vmcnt
// (and a barrier for the other waves).
__device__ __forceinline__ void ore_lds_dma16(__amdgpu_buffer_rsrc_t rsrc, unsigned lds_addr, int voffset, int soffset) {
  int m0save;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(m0save)
      : "s"(__builtin_amdgcn_readfirstlane(lds_addr)), "v"(voffset), "s"(rsrc),
        "s"(__builtin_amdgcn_readfirstlane(soffset))
      : "memory");
}

struct ConvParams {
  const float* x;      // input  [N][C][H][W], image stride x_nstride
  const float* wp;     // packed weights Wp[Kp][Mp] (launch_pack_weights)
  const int2* ktab;    // gather table [Kp] (launch_ktab); unused by 1x1 geometry
  const float* bias;   // [M] or null
  float* y;            // output [N][..][Ho][Wo] starting at the channel slice; image stride y_nstride
  int N, C, H, W;
  int M, kh, kw, sh, sw, pt, pl;
  int Ho, Wo;
  int K;               // C*kh*kw
  int P;               // Ho*Wo
  int x_ps, y_ps;      // channel-plane strides (>= H*W, >= Ho*Wo); y_ps columns are computed per image
  long long Ntot;      // N*y_ps
  long long x_nstride;
  long long y_nstride;
  int relu;
  int is1x1;           // kh = kw = 1, stride 1, no padding, Ho*Wo == H*W
  int Mp;              // row stride of wp (conv_packed_mp(M))
  int mtiles, ntiles;  // filled by the launcher
  int vec_out;         // 16-B epilogue stores (y_ps, y_nstride % 4 == 0 and a 16-B aligned y)
  int x_f32;           // f16 kernel: the input is the f32 NCHW model input (rounded to f16 while staging);
                       // otherwise f16 NHWC with pixel stride x_ps (f16 kernels always write NHWC,
                       // pixel stride y_ps, columns dense over Ho*Wo: Ntot = N*P)
  long long x_bytes;   // bytes from x to the end of its last valid element (0: no buffer DMA path)
  int x_guard;         // bytes before x known to be mapped (the streaming 3x3 conv reads a few of them,
                       // zero-masked, instead of issuing negative buffer offsets)
  int x_lead;          // filled by the streaming launcher: bytes it reads before x (<= x_guard)
  // pooled epilogue (ORE_FUSE_CONV_POOL, launch_conv_epool; 3x3 / stride-2 pool): y is the MaxPool
  // output [..][ep_Ho][ep_Wo] (plane stride y_ps), pool pads ep_pt / ep_pl; a block's N tile is a
  // 13 x 19 patch of conv outputs feeding a 6 x 9 tile of pooled outputs, ep_tr x ep_tc tiles per image
  int ep_pt, ep_pl, ep_Ho, ep_Wo, ep_tr, ep_tc;
  int ep_variant;      // pooled-conv kernel (launch_conv_epool): 0 auto, 1 patch, 2 / 3 row walk
  const float* wc1;    // variant 7: weights in launch_pack_c1_f32 layout (null: variant 7 unavailable)
  const struct C1SqueezeF32* sq1;  // variant 7 with the next 1x1 conv fused in (forces variant 7)
};

// Per-layer kernel choice and weight layout (see plan_conv in ore_conv.hip).
struct ConvPlan {
  int f16;             // 1: conv_f16_kernel (f16 weights Wh[Mp][Kp] and f16 NHWC output)
  int xmode;           // f16: F16_X_NCHW32 / F16_X_NHWC_ELEM / F16_X_NHWC_VEC / F16_X_NHWC_PAIR
  int cfg;             // tile id (0-3: conv_gemm_kernel 128x128, 96x128, 64x128, 32x256; 12-20 streaming;
                       // WINO_TILE_BASE + t)
  int Mp, krows;       // packed weights are krows x Mp floats
  int epv = 0;         // pooled-epilogue steps: ConvParams::ep_variant (ore_model_autotune)
  int wino = 0;        // 1: conv_wino_kernel (Winograd F(2x2, 3x3), ore_conv_wino.hip); cfg = WINO_TILE_BASE + tile
};

struct PoolParams {
  const float* x;      // element type per es (f32 or f16 storage)
  float* y;
  int N, C, H, W;
  int kh, kw, sh, sw, pt, pl;
  int Ho, Wo;
  int x_ps, y_ps;      // channel-plane strides (elements)
  long long x_nstride, y_nstride;
  int es;              // element bytes: 4 (f32) or 2 (f16)
  int variant;         // 0: by layout (launch_maxpool); 1-4 force chunk / plane / strip / direct (ore_ctx_set_pool_variant)
};

// MaxPool over channels-last f16 (f16 models): element (n, c, h, w) at n*nstride + (h*W + w)*cs + c
struct NhwcPoolParams {
  const _Float16* x;
  _Float16* y;
  int N, C, H, W;
  int kh, kw, sh, sw, pt, pl;
  int Ho, Wo;
  int x_cs, y_cs;      // pixel strides (elements, >= C)
  long long x_nstride, y_nstride;
};

struct AddParams {
  const float* a;
  const float* b;
  float* y;
  long long d[4];   // a's (and y's) shape, right-aligned to rank 4
  long long bs[4];  // b strides in elements, 0 on broadcast axes
};

// A fire module fused with the next squeeze (ore_fire.hip, ORE_FUSE_FIRE): S' = Relu(Ws [e1; e3] + bs)
// with e1 = Relu(W1 S + b1) (1x1), e3 = Relu(W3 * S + b3) (3x3, pad 1), e1 / e3 never stored.
struct FireParams {
  const float* x;   // S [N][C][H][W], plane stride x_ps, image stride x_nstride
  const float* w1;  // W1 packed by launch_fire_pack: [roundup(C, 32)][E1]
  const float* b1;
  const float* w3;  // W3 packed by launch_fire_pack: [roundup(9C, 32)][E3], k = (c, r, s)
  const float* b3;
  const float* ws;  // the squeeze's standard K-major packing [roundup(E1 + E3, 32)][Msp] (launch_pack)
  const float* bs;
  float* y;         // S' [N][Ms][H][W], plane stride y_ps (= columns per image), image stride y_nstride
  int N, C, H, W, E1, E3, Ms, Msp;
  int x_ps, y_ps;
  long long x_nstride, y_nstride, Ntot;  // Ntot = N * y_ps
  long long x_bytes;                     // x's valid extent in bytes
  int x_guard, x_lead;                   // mapped bytes before x; bytes the 3x3 taps read before it
  int ntiles;                            // filled by the launcher
  // pooled form (fire_pool_kernel): a 3x3 / stride-2 MaxPool (Hp x Wp, pads ppt / ppl) between the
  // Concat and the squeeze; y is then [N][Ms][Hp][Wp]; PR pooled rows per workgroup (fire_pool_plan)
  int pool, Hp, Wp, ppt, ppl, PR;
};
bool fire_eligible(const FireParams& p);
void launch_fire(const FireParams& p, hipStream_t s);
bool fire_pool_plan(FireParams* p);  // picks PR; false when no band shape fits
// W [M][K] -> the fire kernel's row-permuted K-major packing (M % 64 == 0)
void launch_fire_pack(const float* w, int M, int K, float* wf, hipStream_t s);

// MaxPool 3x3 / stride 2 + its only reader, a 1x1 conv (+ Relu), f32 NCHW (ore_pool_conv.hip;
// SqueezeNet pool5 + fire9/squeeze1x1): x [C][H][W] (plane stride x_ps), wp the conv's K-major
// packing [Kp][Mp], y [M][Hp][Wp] (plane stride y_ps); C % 32 == 0, M <= 64, Wp <= 16
struct PoolConvParams {
  const float* x;
  const float* wp;
  const float* bias;
  float* y;
  int N, C, H, W, Hp, Wp, pt, pl, M, Mp, Kp;
  int x_ps, y_ps;
  long long x_nstride, y_nstride;
  int relu;
  // ORE_FUSE_POOL_EXPAND: the pool input's first E1 channels (a Concat's expand1x1 slice) are not read
  // from x but recomputed from that conv's own input s (C1 = 32 / 64 channels on the pool input's
  // plane): relu(w1 s + b1) with w1 the conv's K-major packing [k][w1_Mp].  E1 = 0: all from x.
  const float* s;
  const float* w1;
  const float* b1;
  int C1, E1, w1_Mp, s_ps;
  long long s_nstride;
};
bool pool_conv1x1_f32_eligible(const PoolConvParams& p);
void launch_pool_conv1x1_f32(const PoolConvParams& p, hipStream_t s);
int pool_conv1x1_f32_rows(int Wp);  // pooled rows per workgroup (band height) for Wp pooled columns

// f16 models: the fused fire module (ore_fire_f16.hip) on NHWC f16 values (pixel strides in
// elements, image strides in elements); weights packed by launch_fire_pack_f16
struct FireF16Params {
  const void* x;   // S: f16 NHWC, C channels, pixel stride x_cs
  const void* w1;  // expand1x1: launch_fire_pack_f16(w, E1, C, 1)
  const float* b1;
  const void* w3;  // expand3x3: launch_fire_pack_f16(w, E3, C, 9), k = (r, s, c)
  const float* b3;
  const void* ws;  // next squeeze: launch_fire_pack_f16(w, Ms, E1 + E3, 1)
  const float* bs;
  void* y;         // S': f16 NHWC, Ms channels, pixel stride y_cs
  int N, C, H, W, E1, E3, Ms, Msp;
  int x_cs, y_cs;
  long long x_nstride, y_nstride;
  int tiles_per_img;  // filled by the launcher
  // pool = 1: a 3x3 / stride-2 MaxPool (pads ppt / ppl, output Hp x Wp) sits between the Concat and
  // the squeeze (SqueezeNet fire4 -> pool3 -> fire5, fire8 -> pool5 -> fire9); y is then the squeeze
  // output on the pooled plane.  PR pooled rows per workgroup, F conv fragments per wave
  // (fire_pool_f16_plan)
  int pool, Hp, Wp, ppt, ppl, PR, F;
};
#define ORE_FIRE_F16_LDS_KB 80  // LDS budget per workgroup (two per CU)
constexpr int FIRE_F16_LDS_MAX = ORE_FIRE_F16_LDS_KB * 1024;  // the input halo of one workgroup (two per CU)
int fire_f16_lds_bytes(int C, int H, int W);
// pooled variant: picks p->F / p->PR (false: no band shape fits the LDS budget)
bool fire_pool_f16_plan(FireF16Params* p);
bool fire_f16_eligible(const FireF16Params& p);
void launch_fire_f16(const FireF16Params& p, hipStream_t s);
// f16 models: the first conv (f32 NCHW input, <= 4 channels, F16_X_NHWC_PAIR packing in p.wp) with
// its 3x3 / stride-2 MaxPool in one persistent launch (ore_conv1_f16.hip); p as for
// launch_conv_f16_epool but p.x is the f32 model input itself (no NHWC4 conversion)
// sq: the pooled map's only consumer, a 1x1 conv + Relu (<= 32 channels, weights by
// launch_fire_pack_f16(w, M, C, 1)), fused in (the pooled map is never stored; y = its output)
struct C1Squeeze {
  const void* w;
  const float* bias;
  int M;
  void* y;                // f16 NHWC on the pooled plane, pixel stride y_cs
  long long y_nstride;
  int y_cs;
};
bool conv_pair_pool_f16_eligible(const ConvParams& p, const C1Squeeze* sq = nullptr);
void launch_conv_pair_pool_f16(const ConvParams& p, const C1Squeeze* sq, hipStream_t s);
// round 6: the same fused first conv + pool + squeeze walked in steps of four conv rows, one workgroup per image
// (conv_band_pool_f16_kernel, tile C1_BAND_F16_TILE); bit-identical to the patch kernel
bool conv_band_pool_f16_geometry(int C, int M, int kh, int kw, int sh, int sw, int pt, int pl, int W, int Wo, int ep_Ho,
                                 int ep_Wo, int ep_pt, int ep_pl, int sq_M);
bool conv_band_pool_f16_eligible(const ConvParams& p, const C1Squeeze* sq);
void launch_conv_band_pool_f16(const ConvParams& p, const C1Squeeze& sq, hipStream_t s);
// W [M][C][kk] f32 (kk = 1 or 9) -> [C kk / 16][roundup(M, 32)][16] f16 with permuted rows
size_t fire_pack_f16_bytes(int M, int C, int kk);
void launch_fire_pack_f16(const float* w, int M, int C, int kk, void* out, hipStream_t s);

int conv_tile_config(int M);
int conv_packed_mp(int M);  // padded M of the packed weights
int conv_packed_kp(int K);  // padded K of the packed weights
// w: ONNX conv weights [M][K] (kmajor_src = false) or MatMul B [K][M] (true) -> wp[Kp][Mp]
void launch_pack_weights(const float* w, bool kmajor_src, int M, int K, int Mp, float* wp, hipStream_t s);
void launch_ktab(int2* ktab, int K, int kh, int kw, int x_ps, int W, hipStream_t s);
// forced >= 0: that tile id when it belongs to the plan's kernel family (ore_ctx_set_conv_tile), else
// the per-layer heuristic
ConvPlan plan_conv(int M, int C, int H, int W, int kh, int kw, int sh, int sw, int pt, int pl, int Ho, int Wo,
                   bool is1x1, bool f16 = false, int xmode = 0, bool wino = false, int forced = -1);
// f16 conv operand modes (ConvPlan::xmode), chosen by the input's layout:
enum {
  F16_X_NCHW32 = 0,     // f32 NCHW model input, per-element gather, k order (c, r, s) (the reference's)
  F16_X_NHWC_ELEM = 1,  // f16 NHWC input with C % 8 != 0: per-element gather, k order (r, s, c)
  F16_X_NHWC_VEC = 2,   // f16 NHWC input, C % 8 == 0: one 16-B load per (pixel, 8 channels), k order (r, s, c)
  F16_X_NHWC_PAIR = 3,  // f32 NCHW input with C <= 4, converted to NHWC4 f16 (launch_nchw_to_nhwc): two
                        // 8-B taps per 8-k group, k order (r, s', c') over kw rounded up to even x 4 channels
};
// GEMM K of an f16 conv (PAIR pads the taps and channels)
int f16_conv_k(int xmode, int C, int kh, int kw);
// f32 NCHW -> f16 NHWC with cs (4) channels per pixel, channels >= C zero
void launch_nchw_to_nhwc(const float* x, void* y, int N, int C, int HW, long long x_nstride, int x_ps, int cs,
                         hipStream_t s);
// Wh[Mp][Kp] = f16(W[M][C][kh][kw]) in the k order of `xmode` (MatMul stays f32)
void launch_pack_weights_f16(const float* w, int xmode, int M, int C, int kh, int kw, int Mp, void* wh, hipStream_t s);
// gather tables of the f16 conv over an NHWC input (F16_X_NCHW32 uses launch_ktab): per k for
// F16_X_NHWC_ELEM, per group of 8 k for F16_X_NHWC_VEC / _PAIR; cs = the input's pixel stride
void launch_ktab_nhwc(int2* ktab, int xmode, int C, int kh, int kw, int cs, int W, hipStream_t s);
void launch_maxpool_nhwc(const NhwcPoolParams& p, hipStream_t s);
// GlobalAveragePool of NHWC f16 -> f32 y[n][c]
void launch_gap_nhwc(const void* x, float* y, int N, int C, int HW, int cs, long long nstride, hipStream_t s);
// f16 models: a 1x1 conv (+ Relu) whose only reader is GlobalAveragePool, in one launch
// (conv1x1_gap_f16_kernel, ore_conv_f16.hip): SqueezeNet's conv10 -> relu10 -> pool10.  x NHWC f16
// [N][P][x_cs], wp the f16 conv packing Wh[Mp][Kp] (K = C), y f32 [N][M] (image stride y_nstride)
struct Conv1x1GapF16 {
  const void* x;
  const void* wp;
  const float* bias;
  float* y;
  int N, C, P, M, Mp, Kp, x_cs, relu;
  long long x_nstride, y_nstride;
};
bool conv1x1_gap_f16_eligible(const Conv1x1GapF16& p);
void launch_conv1x1_gap_f16(const Conv1x1GapF16& p, hipStream_t s);
// f32 models: the same fusion (conv1x1_gap_f32_kernel, ore_conv_gap.hip): x f32 NCHW [N][C][x_ps] (P <= 256
// pixels per plane), wc the weights in launch_pack_cg_f32's layout, y f32 [N][M] (image stride y_nstride)
struct Conv1x1GapF32 {
  const float* x;
  const float* wc;
  const float* bias;
  float* y;
  int N, C, P, M, x_ps, relu;
  long long x_nstride, y_nstride;
};
bool conv1x1_gap_f32_eligible(const Conv1x1GapF32& p);
// conv1x1_gap_f32_kernel's weights: [ceil(K/16)][Mp32][4 kq][4 s] = W[row][16 q + 4 s + kq] (zeros past M, K)
size_t cg_f32_pack_bytes(int M, int K);
void launch_pack_cg_f32(const float* w, int M, int K, float* out, hipStream_t s);
void launch_conv1x1_gap_f32(const Conv1x1GapF32& p, hipStream_t s);
// Concat along channels of two dense NHWC f16 values (pixels = N*H*W)
void launch_concat_nhwc(const void* a, const void* b, void* y, long long pixels, int Ca, int Cb, hipStream_t s);
void launch_conv_f16(const ConvParams& p, int cfg, int xmode, hipStream_t s);
// f16 Conv (+ Relu) with the following 3x3 / stride-2 MaxPool in its epilogue (ConvParams ep_*,
// NHWC f16 pooled output)
void launch_conv_f16_epool(const ConvParams& p, int xmode, hipStream_t s);
size_t conv_packed_bytes(const ConvPlan& pln);
// packs ONNX weights [M][C][kh][kw] (or MatMul [K][M]) in the layout the plan's kernel reads
void launch_pack(const float* w, bool kmajor_src, int M, int C, int kh, int kw, const ConvPlan& pln, float* wp,
                 hipStream_t s);
void launch_conv(const ConvParams& p, const ConvPlan& pln, hipStream_t s);
// Conv (+ Relu) with the following MaxPool in its epilogue (ConvParams ep_* set; f32)
void launch_conv_epool(const ConvParams& p, hipStream_t s);
// Stride-2 Conv + Relu + 3x3 / stride-2 MaxPool walking the conv plane row-major with the pooled rows
// in an LDS ring (ore_conv_pool.hip; conv1 + pool1): launch_conv_epool takes it when eligible.
// variants (ConvParams::ep_variant): 1 = the patch kernel, 2 = walk 48 channels x 64 quads per block,
// 3 = walk 96 channels x 128 quads, 4 = walk 64 x 64, 5 = 4 over 3 bands of pooled rows; 0 = the first
// eligible of 3, 4, 2, 1 at batch >= 128, else 1.  A model sets the variant per step (autotune,
// ore_model_set_step_tile with EPOOL_TILE_BASE + variant).  launch_conv_epool leaves last_conv_tile =
// EPOOL_TILE_BASE + the variant run.
constexpr int EPOOL_TILE_BASE = 21;
// variant 7 (ore_conv1_f32.hip): the first conv (7x7 / stride 2, C in {1, 3, 4}, 64 < M <= 128) with
// its input window in LDS, weights packed by launch_pack_c1_f32 (ConvPlan::wc1); reported as tile
// EPOOL_WIN_TILE (after the Winograd / fused-f16 tile ids: ore.Model.TILE_NAMES "epool window f32")
constexpr int EPOOL_WIN_VARIANT = 7, EPOOL_WIN_TILE = 44;

// the pooled f32 fire module (fire_pool_kernel): ore.Model.TILE_NAMES "fire pool f32"
constexpr int FIRE_POOL_TILE = 45;
// sq: the pooled map's only consumer, a 1x1 conv + Relu with <= 16 channels (ONNX weights [M][K]),
// fused in (conv1's geometry only); the pooled map is never stored, y = the squeeze's NCHW output
struct C1SqueezeF32 {
  const float* w;
  const float* bias;
  int M;
  float* y;
  long long y_nstride;
  int y_ps;
};
bool conv_win_pool_f32_eligible(const ConvParams& p, const C1SqueezeF32* sq = nullptr);
void launch_conv_win_pool_f32(const ConvParams& p, const float* wc, const C1SqueezeF32* sq, hipStream_t s);
// variant 8 (ore_conv1_f32.hip): the fused first conv + pool + squeeze walking bands of conv rows (no
// recomputed halo; 7x7 / stride 2, C = 3, 64 < M <= 96, inputs <= 224 wide); tile EPOOL_BAND_TILE
// ("epool band f32"), an autotune candidate beside the window kernel for the fused squeeze
constexpr int EPOOL_BAND_VARIANT = 8, EPOOL_BAND_TILE = 51;
// the layout-independent part of conv_band_pool_f32_eligible (the planner's candidate list)
bool conv_band_pool_f32_geometry(int C, int M, int kh, int kw, int sh, int sw, int pt, int pl, int W, int Wo, int ep_Ho,
                                 int ep_Wo, int ep_pt, int ep_pl, int sq_M, bool relu);
bool conv_band_pool_f32_eligible(const ConvParams& p, const C1SqueezeF32* sq);
void launch_conv_band_pool_f32(const ConvParams& p, const float* wc, const C1SqueezeF32& sq, hipStream_t s);
inline int epool_tile_id(int variant) {
  return variant == EPOOL_WIN_VARIANT ? EPOOL_WIN_TILE : variant == EPOOL_BAND_VARIANT ? EPOOL_BAND_TILE : EPOOL_TILE_BASE + variant;
}
size_t c1_f32_pack_bytes(int M, int K);
void launch_pack_c1_f32(const float* w, int M, int K, float* out, hipStream_t s);
bool conv_pool_stream_eligible(const ConvParams& p, int variant);
void launch_conv_pool_stream(const ConvParams& p, int variant, hipStream_t s);
constexpr int CONV_EPOOL_BN = 256;  // N tile of the pooled-epilogue kernel
constexpr int EPOOL_TILE_PR = 6, EPOOL_TILE_PC = 9;  // pooled outputs per block (13 x 19 conv patch)
// tile ids 4-11 are retired (the LDS-free direct and the warp-specialised conv_gemm variants, measured
// slower on every SqueezeNet layer: DESIGN.md section 7.1), and so are 28-35 (ABI 1's bf16x3 kernels);
// ore_ctx_set_conv_tile / ore_model_set_step_tile reject them
constexpr int CONV_TILES_F32 = 21;  // 0-3 conv_gemm_kernel, 12-20 conv_stream_kernel (stride-1 geometries)
constexpr int FIRE_TILE = 21;       // the fused f32 fire module (fire_kernel): ore.Model.TILE_NAMES "fire"
inline bool conv_tile_retired(int t) { return (t >= 4 && t < 12) || (t >= 28 && t < 36); }
// LDS-free streaming kernel (ore_conv_stream.hip): 1x1 convs and stride-1 convs with Wo == W (every
// expand3x3); tiles CONV_TILE_STREAM + 0..8 = 64x128, 32x256, 16x256, 48x128, 64x64, 128x64, 64x64 D8,
// 32x128, 48x64 (round 4; 128x64 D2 before) (channels x pixels per wave); other geometries fall back to tile 0
constexpr int CONV_TILE_STREAM = 12;
// persistent 1x1 streaming tiles (conv_stream1x1_persist_kernel): 32x128, 64x64, 16x256; ids after the
// fused-kernel ids (ore.Model.TILE_NAMES "stream1x1 persist ...")
constexpr int CONV_TILE_SP = 46, CONV_TILES_SP = 3;
bool conv_stream_eligible(const ConvParams& p, int tile);
void launch_conv_stream(const ConvParams& p, int tile, hipStream_t s);
// the tile launch_conv actually ran last on this thread (a 1x1 tile on an ineligible geometry runs
// tile 0); ore_model_autotune skips candidates that fell back
extern thread_local int last_conv_tile;
constexpr int CONV_TILES_F16 = 4;
// 3x3 / stride-1 / pad-1 f32 conv by Winograd F(2x2, 3x3) on the f32 MFMA (ore_conv_wino.hip).  Tiles
// WINO_TILE_BASE + 0..3 = 32 ch x 32 tiles (32x32x2 MFMA, ring 4 / 2), 32 x 16, 16 x 32 (16x16x4);
// 4 = the LDS-staged kernel (64 tiles x 32 channels per 4-wave block, windows and U from LDS; C % 16 == 0),
// results do not depend on the tile (not bit-identical to the direct kernels).  Weights packed by
// launch_pack_wino: U = s_xi (G g G^T)[xi] as [C][4][Mp][4] f32 (channel, position quad, m, position)
// (Mp = wino_packed_mp(M)), with the sign s_xi = -1 for positions xi % 4 == 3 (+1 otherwise): every kernel's
// V carries the same sign (wg_input_transform / _pk), so each product U_xi V_xi is the unsigned one.
// tile ids 28-35 are retired (ABI 1's opt-in bf16x3 kernels, ORE_LOAD_X3)
constexpr int WINO_TILE_BASE = 36;
constexpr int WINO_TILES_N = 5;
// fused-kernel ids after the Winograd tiles (ore.Model.TILE_NAMES): 41 is retired (the Winograd fire module)
constexpr int FIRE_F16_TILE = 42, C1_POOL_F16_TILE = 43;
// plan.epv of the f16 first conv + pool + squeeze: the band walker, the patch kernel (chosen explicitly)
constexpr int C1_BAND_F16_TILE = 52, C1_BAND_F16_VARIANT = 9, C1_PATCH_F16_VARIANT = 10;
constexpr int CONV_GAP_F16_TILE = 49;  // conv1x1_gap_f16_kernel: ore.Model.TILE_NAMES "conv1x1 gap f16"
constexpr int CONV_GAP_F32_TILE = 50;  // conv1x1_gap_f32_kernel: ore.Model.TILE_NAMES "conv1x1 gap f32"
bool conv_wino_geometry(int C, int kh, int kw, int sh, int sw, int pt, int pl, int H, int W, int Ho, int Wo);
bool conv_wino_eligible(const ConvParams& p, int tile);
int wino_packed_mp(int M);
void launch_pack_wino(const float* w, int M, int C, int Mp, float* u, hipStream_t s);
void launch_conv_wino(const ConvParams& p, int tile, hipStream_t s);
void launch_maxpool(const PoolParams& p, hipStream_t s);
void launch_relu(const float* x, float* y, long long n, hipStream_t s);
void launch_relu_f16(const void* x, void* y, long long n, hipStream_t s);
void launch_add_bcast(const AddParams& p, hipStream_t s);
void launch_softmax(const float* x, float* y, long long rows, int D, hipStream_t s);
// rows of HW elements at a row stride of ps (>= HW); es: 4 f32, 2 f16 input
void launch_gap(const void* x, int es, float* y, long long rows, int HW, int ps, hipStream_t s);
void launch_concat(const void* a, const void* b, void* y, int es, long long outer, long long ia, long long ib,
                   hipStream_t s);

}  // namespace ore
