// Internal kernel launch interface (device pointers, resolved integer geometry).  The public
// C ABI (include/ore.h) sits on top of this in ore_api.cpp.
#pragma once
#include <hip/hip_runtime.h>

namespace ore {

struct ConvParams {
  const float* x;      // input  [N][C][H][W], image stride x_nstride
  const float* w;      // weights [M][C*kh*kw] (ONNX layout) or [K][M] when w_kmajor
  const float* bias;   // [M] or null
  float* y;            // output [N][..][Ho][Wo] starting at the channel slice; image stride y_nstride
  int N, C, H, W;
  int M, kh, kw, sh, sw, pt, pl;
  int Ho, Wo;
  int K;               // C*kh*kw
  int P;               // Ho*Wo
  long long Ntot;      // N*P
  long long x_nstride;
  long long y_nstride;
  int relu;
  int is1x1;           // kh = kw = 1, stride 1, no padding, Ho*Wo == H*W
  int w_kmajor;
  int mtiles, ntiles;  // filled by the launcher
};

struct PoolParams {
  const float* x;
  float* y;
  int N, C, H, W;
  int kh, kw, sh, sw, pt, pl;
  int Ho, Wo;
  long long x_nstride, y_nstride;
};

struct AddParams {
  const float* a;
  const float* b;
  float* y;
  long long d[4];   // a's (and y's) shape, right-aligned to rank 4
  long long bs[4];  // b strides in elements, 0 on broadcast axes
};

int conv_tile_config(int M);
void launch_conv(const ConvParams& p, hipStream_t s);
void launch_maxpool(const PoolParams& p, hipStream_t s);
void launch_relu(const float* x, float* y, long long n, hipStream_t s);
void launch_add_bcast(const AddParams& p, hipStream_t s);
void launch_softmax(const float* x, float* y, long long rows, int D, hipStream_t s);
void launch_gap(const float* x, float* y, long long rows, int HW, hipStream_t s);
void launch_concat(const float* a, const float* b, float* y, long long outer, long long ia, long long ib,
                   hipStream_t s);

}  // namespace ore
