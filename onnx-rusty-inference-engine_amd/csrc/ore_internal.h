// Host-side internals shared by the C ABI implementation files.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "../../include/ore.h"
#include "ore_kernels.h"

struct ore_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  float* scratch = nullptr;  // per-op weight packing (stream-ordered reuse)
  size_t scratch_bytes = 0;
  // a device range known to be mapped, set by the model walker around its conv launches (its arena,
  // which has a 4 KiB lead): the streaming conv may read a few bytes before an input inside it
  const char* mapped_lo = nullptr;
  const char* mapped_hi = nullptr;
  int conv_algo = 0;     // ore_ctx_set_conv_algo (per-op ore_conv2d_f32 only)
  int conv_tile = -1;    // ore_ctx_set_conv_tile: a forced tile id (-1: per-layer heuristic / autotune)
  int pool_variant = 0;  // ore_ctx_set_pool_variant: a forced MaxPool kernel (0: by layout)
};

namespace ore {

// ---------------------------------------------------------------- errors
ore_status set_error(ore_ctx* ctx, ore_status st, const char* fmt, ...);
#define ORE_HIP_CHECK(ctx, expr)                                                          \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return ::ore::set_error((ctx), ORE_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

// ---------------------------------------------------------------- ONNX subset (onnx.proto)
struct Attr {
  std::string name;
  int type = 0;
  float f = 0.f;
  int64_t i = 0;
  std::string s;
  std::vector<int64_t> ints;
  std::vector<float> floats;
  bool has_i = false, has_f = false, has_s = false;
};

struct Node {
  std::string op_type, name;
  std::vector<std::string> inputs, outputs;
  std::vector<Attr> attrs;
};

struct Initializer {
  std::string name;
  std::vector<int64_t> dims;
  int dtype = 0;
  std::vector<float> f32;
  std::vector<int64_t> i64;
};

struct ValueInfo {
  std::string name;
  std::vector<int64_t> shape;
};

struct Graph {
  std::vector<Node> nodes;
  std::vector<Initializer> inits;
  std::vector<ValueInfo> inputs, outputs;
};

// Parses a ModelProto; returns false with a message on malformed input.
bool parse_model(const uint8_t* data, size_t len, Graph* g, std::string* err);

// ---------------------------------------------------------------- reference geometry
// Resolved window geometry (convolution_op.rs:266-350, max_pool_op.rs:188-264).
struct Window {
  int64_t pt = 0, pl = 0, pb = 0, pr = 0;
  int64_t Ho = 0, Wo = 0;
};
// auto_pad as ore_auto_pad; pads in ONNX order.  Returns ORE_OK or an error status.
ore_status resolve_window(ore_ctx* ctx, int auto_pad, const int64_t* pads, int n_pads, int64_t H, int64_t W,
                          int64_t kh, int64_t kw, int64_t sh, int64_t sw, Window* out);

// ---------------------------------------------------------------- launches over resolved geometry
// Kernel plan of a conv (or MatMul as a 1x1 conv) over resolved geometry.
ConvPlan conv_plan(int64_t M, int64_t C, int64_t H, int64_t W, int64_t kh, int64_t kw, int64_t sh, int64_t sw,
                   const Window& win, bool f16 = false, int xmode = 0, bool wino = false,
                   int forced = -1);
// wp: weights packed by launch_pack for plan `pln`
// ktab: gather table (launch_ktab) for non-1x1 geometry on the gather kernel
ore_status run_conv(ore_ctx* ctx, const ConvPlan& pln, const float* x, int64_t N, int64_t C, int64_t H, int64_t W,
                    int64_t x_nstride, const float* wp, const int2* ktab, int64_t M, int64_t kh, int64_t kw,
                    const float* bias, const Window& win, int64_t sh, int64_t sw, bool relu, float* y,
                    int64_t y_nstride, int64_t x_ps = 0, int64_t y_ps = 0,  // plane strides, 0 = dense
                    int x_es = 4);  // input element bytes (f32 plans only)
// the MaxPool fused into an f16 conv's epilogue (ORE_FUSE_CONV_POOL; 3x3 / stride 2)
struct F16Epool {
  int64_t kh, kw, sh, sw;
  Window win;  // the pool's window over the conv output
};
// f16 first conv + pooled epilogue straight from the f32 NCHW input (ore_conv1_f16.hip) when its
// geometry allows; *ran = false (and ORE_OK) otherwise, for the two-launch path.
ore_status run_conv_pair_pool_f16(ore_ctx* ctx, const ConvPlan& pln, const float* x, int64_t N, int64_t C, int64_t H,
                                  int64_t W, int64_t x_nstride, int64_t x_ps, const void* wp, int64_t M, int64_t kh,
                                  int64_t kw, const float* bias, const Window& win, int64_t sh, int64_t sw, bool relu,
                                  void* y, int64_t y_nstride, int64_t y_ps, const F16Epool& ep, bool* ran,
                                  const C1Squeeze* sq = nullptr);
// f16 plan (f16 models): y is NHWC f16 with pixel stride y_ps; x is the f32 NCHW model input
// (F16_X_NCHW32, plane stride x_ps) or NHWC f16 with pixel stride x_ps.  ktab per plan.xmode.
// ep: the following MaxPool in the epilogue (y is then the pooled NHWC output)
ore_status run_conv_f16(ore_ctx* ctx, const ConvPlan& pln, const void* x, int64_t N, int64_t C, int64_t H, int64_t W,
                        int64_t x_nstride, int64_t x_ps, const void* wp, const int2* ktab, int64_t M, int64_t kh,
                        int64_t kw, const float* bias, const Window& win, int64_t sh, int64_t sw, bool relu, void* y,
                        int64_t y_nstride, int64_t y_ps, const F16Epool* ep = nullptr);
// Conv (+ Relu) and the MaxPool (pkh x pkw, strides psh/psw, window pwin over the conv's Ho x Wo
// output) in one launch: y is the pooled output (image stride y_nstride, plane stride y_ps)
ore_status run_conv_epool(ore_ctx* ctx, const ConvPlan& pln, const float* x, int64_t N, int64_t C, int64_t H, int64_t W,
                          int64_t x_nstride, int64_t x_ps, const float* wp, const int2* ktab, int64_t M, int64_t kh,
                          int64_t kw, const float* bias, const Window& win, int64_t sh, int64_t sw, bool relu,
                          int64_t pkh, int64_t pkw, int64_t psh, int64_t psw, const Window& pwin, float* y,
                          int64_t y_nstride, int64_t y_ps, const float* wc1 = nullptr,
                          const C1SqueezeF32* sq1 = nullptr);
// a fire module fused with the next squeeze (ORE_FUSE_FIRE, ore_fire.hip): x = S [C][H][W] (plane
// stride x_ps), w1 / w3 in launch_fire_pack layout, ws the squeeze's launch_pack layout (row stride
// Msp); y = S' [Ms][H][W] (plane stride y_ps, the column count per image)
ore_status run_fire(ore_ctx* ctx, const float* x, int64_t N, int64_t C, int64_t H, int64_t W, int64_t x_nstride,
                    int64_t x_ps, const float* w1, const float* b1, int64_t E1, const float* w3, const float* b3,
                    int64_t E3, const float* ws, int64_t Msp, const float* bs, int64_t Ms, float* y, int64_t y_nstride,
                    int64_t y_ps, const Window* pool = nullptr);
// the f16 fused fire module (ore_fire_f16.hip): x = S, y = S' NHWC f16 (pixel strides x_cs / y_cs,
// image strides in elements); w1 / w3 / ws in launch_fire_pack_f16 layout; pool: a 3x3 / stride-2
// MaxPool (window over the H x W conv plane) between the Concat and the squeeze, y on its plane
ore_status run_fire_f16(ore_ctx* ctx, const void* x, int64_t N, int64_t C, int64_t H, int64_t W, int64_t x_nstride,
                        int64_t x_cs, const void* w1, const float* b1, int64_t E1, const void* w3, const float* b3,
                        int64_t E3, const void* ws, const float* bs, int64_t Ms, void* y, int64_t y_nstride,
                        int64_t y_cs, const Window* pool = nullptr);
// pooled-epilogue tiling of a conv output (Ho x Wo) and its pool (3x3 / stride 2 only): *tr x *tc
// tiles of 6 x 9 pooled outputs per image; returns the work factor tiles * CONV_EPOOL_BN / (Ho * Wo)
// (the conv columns computed, recomputed overlap and padding included), 0 for other pools
double epool_tile(int64_t Ho, int64_t Wo, int64_t pkh, int64_t pkw, int64_t psh, int64_t psw, const Window& pwin,
                  int* tr, int* tc);
// the pooled squeeze's recomputed expand1x1 (walker pass pool_expand): x's first E1 channels are
// relu(w1 s + b1) of s [C1][pH][pW] (plane stride s_ps, image stride s_nstride), w1 K-major [k][w1_Mp]
struct PoolExpand {
  const float* s;
  const float* w1;
  const float* b1;
  int C1, E1, w1_Mp;
  int64_t s_ps, s_nstride;
};
// 1x1 conv over the 3x3 / stride-2 MaxPool (window pwin) of x [C][pH][pW] (plane stride x_ps) on
// pool_conv1x1_f32_kernel: the pooled tensor is never materialised (walker pass fuse_pool_squeeze)
ore_status run_conv_pool(ore_ctx* ctx, const ConvPlan& pln, const float* x, int64_t N, int64_t C, int64_t pH,
                         int64_t pW, int64_t x_nstride, int64_t x_ps, const Window& pwin, int64_t psh, int64_t psw,
                         const float* wp, int64_t M, const float* bias, bool relu, float* y, int64_t y_nstride,
                         int64_t y_ps, int x_es, const PoolExpand* pe = nullptr);
// packs w (and the gather table for an input of H x W) into the context scratch buffer;
// returns the packed weights (or null with the error set), *ktab receives the table
float* pack_to_scratch(ore_ctx* ctx, const ConvPlan& pln, const float* w, bool kmajor_src, int64_t M, int64_t C,
                       int64_t kh, int64_t kw, int64_t H, int64_t W, const int2** ktab);
// bytes of packed weights + gather table for one conv
size_t packed_bytes(const ConvPlan& pln);
ore_status run_maxpool(ore_ctx* ctx, const float* x, int64_t N, int64_t C, int64_t H, int64_t W,
                       int64_t x_nstride, int64_t kh, int64_t kw, const Window& win, int64_t sh, int64_t sw,
                       float* y, int64_t y_nstride, int64_t x_ps = 0, int64_t y_ps = 0,
                       int es = 4);  // element bytes of x and y; ctx->pool_variant selects a kernel
// MaxPool over NHWC f16 (f16 models); x_cs / y_cs: pixel strides
ore_status run_maxpool_nhwc(ore_ctx* ctx, const void* x, int64_t N, int64_t C, int64_t H, int64_t W, int64_t x_nstride,
                            int64_t x_cs, int64_t kh, int64_t kw, const Window& win, int64_t sh, int64_t sw, void* y,
                            int64_t y_nstride, int64_t y_cs);

}  // namespace ore
