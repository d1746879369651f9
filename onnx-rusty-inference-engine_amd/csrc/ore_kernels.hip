// MI355X (gfx950 / CDNA4) kernels for the fp32 ONNX op path of
// jackperlo/onnx-rusty-inference-engine (src/inference_fp32_ops/*).  Written for 64-lane waves
// and the f32-input MFMA (v_mfma_f32_32x32x2_f32: exact f32 fma chain, 157 TFLOP/s peak).
//
//   (Conv / MatMul: ore_conv.hip)
//   maxpool_kernel     MaxPool (max_pool_op.rs:157-360): ZERO padding, start at -FLT_MAX.
//   relu_kernel        Relu (relu_op.rs:31-33).
//   add_bcast_kernel   Add with right-aligned broadcast (add_op.rs:74-84).
//   softmax_kernel     Softmax over rows (softmax_op.rs:45-57), max + the reference's own
//                      8-partial-sum order for the denominator.
//   gap_kernel         GlobalAveragePool (global_average_pool_op.rs:33-51), sequential sum per
//                      channel (bit-identical to the reference's Iterator::sum order).
//   concat_kernel      Concat of two tensors (concatenate_op.rs:31-32).
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>
#include <stdlib.h>

#include "ore_kernels.h"

namespace ore {

// ------------------------------------------------------------------------------------------
// MaxPool: grid.x = image planes (n, c), grid.y covers the plane's outputs; 32-bit index math
// inside a plane.  The window reads zeros outside the image (the reference pads with 0,
// max_pool_op.rs:265-276) and starts from -FLT_MAX (:337).  HBM-bound: in + out bytes.
// ------------------------------------------------------------------------------------------
template <typename T, int KH, int KW>  // T: float or _Float16 (element type of x and y); 0 = runtime window
__global__ __launch_bounds__(256) void maxpool_kernel(PoolParams p, int chunks) {
  // 1-D grid, chunk index fastest: consecutive blocks stream consecutive parts of one plane
  const int plane = blockIdx.x / chunks;  // n * C + c
  const int chunk = blockIdx.x - plane * chunks;
  const int n = plane / p.C, c = plane - n * p.C;
  const T* __restrict__ xp = reinterpret_cast<const T*>(p.x) + (long long)n * p.x_nstride + (long long)c * p.x_ps;
  T* __restrict__ yp = reinterpret_cast<T*>(p.y) + (long long)n * p.y_nstride + (long long)c * p.y_ps;
  const int P = p.Ho * p.Wo;
  for (int idx = chunk * 256 + threadIdx.x; idx < P; idx += chunks * 256) {
    const int oh = idx / p.Wo, ow = idx - oh * p.Wo;
    const int ih0 = oh * p.sh - p.pt, iw0 = ow * p.sw - p.pl;
    float m = -FLT_MAX;
    const int kh = KH ? KH : p.kh, kw = KW ? KW : p.kw;
#pragma unroll
    for (int r = 0; r < kh; ++r) {
      const int ih = ih0 + r;
      const bool rok = (unsigned)ih < (unsigned)p.H;
      const T* row = xp + ih * p.W;
#pragma unroll
      for (int s = 0; s < kw; ++s) {
        const int iw = iw0 + s;
        const float v = (rok && (unsigned)iw < (unsigned)p.W) ? (float)row[iw] : 0.0f;
        m = fmaxf(m, v);
      }
    }
    yp[idx] = (T)m;  // max of the inputs (or 0): exact in T
  }
}

// Column-strip MaxPool: one thread per (plane, output column, band of RB output rows).  The
// thread walks down its band; each input row is reduced across the KW window columns once
// and the row maxima shared by consecutive windows (KH > SH) stay in registers, so an output
// row costs SH*KW loads instead of KH*KW.  Lanes are consecutive output columns (then the next
// plane's), so loads are stride-SW and stores are coalesced.  Zero padding / -FLT_MAX start as
// above; max is exact, so the regrouping is bit-identical.
template <typename T, int KH, int KW, int SH, int RB>
__global__ __launch_bounds__(256) void maxpool_strip_kernel(PoolParams p, long long cols) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t >= cols) return;
  const long long plane = t / p.Wo;
  const int ow = (int)(t - plane * p.Wo);
  const int n = (int)(plane / p.C), c = (int)(plane - (long long)n * p.C);
  const T* __restrict__ xp = reinterpret_cast<const T*>(p.x) + (long long)n * p.x_nstride + (long long)c * p.x_ps;
  T* __restrict__ yp = reinterpret_cast<T*>(p.y) + (long long)n * p.y_nstride + (long long)c * p.y_ps;
  const int oh0 = blockIdx.y * RB;
  const int oh1 = min(p.Ho, oh0 + RB);
  const int iw0 = ow * p.sw - p.pl;
  bool cok[KW];
#pragma unroll
  for (int s = 0; s < KW; ++s) cok[s] = (unsigned)(iw0 + s) < (unsigned)p.W;
  constexpr int KEEP = KH > SH ? KH - SH : 0;
  float keep[KEEP > 0 ? KEEP : 1];
#define ORE_ROWMAX(DST, IH)                                                       \
  {                                                                               \
    const int ih_ = (IH);                                                         \
    const bool rok_ = (unsigned)ih_ < (unsigned)p.H;                              \
    const T* row_ = xp + (rok_ ? ih_ : 0) * p.W;                                  \
    float m_ = -FLT_MAX;                                                          \
    _Pragma("unroll") for (int s = 0; s < KW; ++s) {                              \
      const float v_ = (rok_ && cok[s]) ? (float)row_[iw0 + s] : 0.0f;            \
      m_ = fmaxf(m_, v_);                                                         \
    }                                                                             \
    DST = m_;                                                                     \
  }
  int ih = oh0 * SH - p.pt;
#pragma unroll
  for (int r = 0; r < KEEP; ++r) ORE_ROWMAX(keep[r], ih + r);
#pragma unroll 2
  for (int oh = oh0; oh < oh1; ++oh) {
    float m = -FLT_MAX;
#pragma unroll
    for (int r = 0; r < KEEP; ++r) m = fmaxf(m, keep[r]);
    float fresh[KH - KEEP];
#pragma unroll
    for (int r = 0; r < KH - KEEP; ++r) {
      ORE_ROWMAX(fresh[r], ih + KEEP + r);
      m = fmaxf(m, fresh[r]);
    }
    yp[oh * p.Wo + ow] = (T)m;
    // rows ih+SH .. ih+KH-1 open the next window
#pragma unroll
    for (int r = 0; r < KEEP; ++r) keep[r] = (r + SH < KEEP) ? keep[r + SH] : fresh[r + SH - KEEP];
    ih += SH;
  }
#undef ORE_ROWMAX
}

// Plane-staged MaxPool: one block per group of PB consecutive (n, c) planes.  The planes are
// copied to LDS with coalesced loads (every input element leaves HBM once, 8 loads in flight per
// thread), then every output window is evaluated from LDS and stored coalesced.
template <typename T, int KH, int KW>
__global__ __launch_bounds__(256) void maxpool_planes_kernel(PoolParams p, int pb, long long planes) {
  extern __shared__ __attribute__((aligned(16))) char tile_raw[];
  T* tile = reinterpret_cast<T*>(tile_raw);  // [pb][H*W]
  const int HW = p.H * p.W;
  const long long q0 = (long long)blockIdx.x * pb;
  const int nq = (int)min((long long)pb, planes - q0);
  const int tid = threadIdx.x;
  for (int q = 0; q < nq; ++q) {
    const long long pl = q0 + q;
    const int n = (int)(pl / p.C), c = (int)(pl - (long long)n * p.C);
    const T* __restrict__ xq = reinterpret_cast<const T*>(p.x) + (long long)n * p.x_nstride + (long long)c * p.x_ps;
    T* tq = tile + q * HW;
    int i0 = 0;  // elements copied by the 16-B path
    if (((reinterpret_cast<uintptr_t>(xq) | reinterpret_cast<uintptr_t>(tq)) & 15) == 0) {
      // 16-B copies (4 floats / 8 halves per lane), 4 in flight per thread
      constexpr int EV = 16 / (int)sizeof(T);
      const int nv = HW / EV;
      const uint4* __restrict__ xv = reinterpret_cast<const uint4*>(xq);
      uint4* tv = reinterpret_cast<uint4*>(tq);
      int i = tid;
      for (; i + 3 * 256 < nv; i += 4 * 256) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = xv[i + u * 256];
#pragma unroll
        for (int u = 0; u < 4; ++u) tv[i + u * 256] = v[u];
      }
      for (; i < nv; i += 256) tv[i] = xv[i];
      i0 = nv * EV;
    }
    int i = i0 + tid;
    for (; i + 7 * 256 < HW; i += 8 * 256) {
      T v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = xq[i + u * 256];
#pragma unroll
      for (int u = 0; u < 8; ++u) tq[i + u * 256] = v[u];
    }
    for (; i < HW; i += 256) tq[i] = xq[i];
  }
  __syncthreads();
  const int P = p.Ho * p.Wo;
  const int kh = KH ? KH : p.kh, kw = KW ? KW : p.kw;
  for (int q = 0; q < nq; ++q) {
    const long long pl = q0 + q;
    const int n = (int)(pl / p.C), c = (int)(pl - (long long)n * p.C);
    T* __restrict__ yq = reinterpret_cast<T*>(p.y) + (long long)n * p.y_nstride + (long long)c * p.y_ps;
    const T* tq = tile + q * HW;
    for (int o = tid; o < P; o += 256) {
      const int oh = o / p.Wo, ow = o - oh * p.Wo;
      const int ih0 = oh * p.sh - p.pt, iw0 = ow * p.sw - p.pl;
      float m = -FLT_MAX;
#pragma unroll
      for (int r = 0; r < kh; ++r) {
        const int ih = ih0 + r;
        const bool rok = (unsigned)ih < (unsigned)p.H;
#pragma unroll
        for (int s2 = 0; s2 < kw; ++s2) {
          const int iw = iw0 + s2;
          const float v = (rok && (unsigned)iw < (unsigned)p.W) ? (float)tq[ih * p.W + iw] : 0.0f;
          m = fmaxf(m, v);
        }
      }
      yq[o] = (T)m;
    }
  }
}

// Chunk-staged MaxPool: one block per PB consecutive (n, c) planes of a tensor whose planes are
// evenly spaced (x_nstride == C * x_ps, y_nstride == C * y_ps: one contiguous run of PB * x_ps
// elements, padded planes included).  The run goes to LDS by 16-B loads issued back to back (one
// plane of 27 x 27 is only 182 float4s: staging plane by plane leaves most lanes idle and one load
// round trip per plane), then all PB * Ho * Wo windows are evaluated from LDS.
template <typename T, int KH, int KW>
__global__ __launch_bounds__(256) void maxpool_chunk_kernel(PoolParams p, int pb, long long planes) {
  extern __shared__ __attribute__((aligned(16))) char tile_raw[];
  T* tile = reinterpret_cast<T*>(tile_raw);  // [pb][x_ps]
  const long long q0 = (long long)blockIdx.x * pb;
  const int nq = (int)min((long long)pb, planes - q0);
  const int tid = threadIdx.x;
  const T* __restrict__ src = reinterpret_cast<const T*>(p.x) + q0 * p.x_ps;
  const int cnt = (nq - 1) * p.x_ps + p.H * p.W;  // elements to stage (the last plane's padding skipped)
  constexpr int EV = 16 / (int)sizeof(T);
  const int nv = cnt / EV;  // host: x 16-B aligned, x_ps % EV == 0
  const uint4* __restrict__ xv = reinterpret_cast<const uint4*>(src);
  uint4* tv = reinterpret_cast<uint4*>(tile);
  int i = tid;
  for (; i + 7 * 256 < nv; i += 8 * 256) {
    uint4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = xv[i + u * 256];
#pragma unroll
    for (int u = 0; u < 8; ++u) tv[i + u * 256] = v[u];
  }
  for (; i < nv; i += 256) tv[i] = xv[i];
  for (int e = nv * EV + tid; e < cnt; e += 256) tile[e] = src[e];
  __syncthreads();
  const int P = p.Ho * p.Wo;
  const int total = nq * P;
  const int kh = KH ? KH : p.kh, kw = KW ? KW : p.kw;
  T* __restrict__ y = reinterpret_cast<T*>(p.y) + q0 * p.y_ps;
  for (int o = tid; o < total; o += 256) {
    const int q = o / P, r = o - q * P;
    const int oh = r / p.Wo, ow = r - oh * p.Wo;
    const int ih0 = oh * p.sh - p.pt, iw0 = ow * p.sw - p.pl;
    const T* tq = tile + q * p.x_ps;
    float m = -FLT_MAX;
#pragma unroll
    for (int rr = 0; rr < kh; ++rr) {
      const int ih = ih0 + rr;
      const bool rok = (unsigned)ih < (unsigned)p.H;
#pragma unroll
      for (int s2 = 0; s2 < kw; ++s2) {
        const int iw = iw0 + s2;
        const float v = (rok && (unsigned)iw < (unsigned)p.W) ? (float)tq[ih * p.W + iw] : 0.0f;
        m = fmaxf(m, v);
      }
    }
    y[q * p.y_ps + r] = (T)m;
  }
}

// variants (PoolParams::variant; 0 = by layout, others forced through ore_ctx_set_pool_variant for the
// parity tests -- max is exact, so every variant is bit-identical): 2 direct, 3 column strip, 4
// plane-staged (one plane per block), 5 chunk-staged (12 KB of LDS per block)
constexpr long long POOL_CHUNK_BYTES = 12 * 1024;
constexpr int POOL_STRIP_RB = 16;  // output rows per thread of the column strip

template <typename T>
static void launch_maxpool_t(const PoolParams& p, hipStream_t s) {
  const long long planes = (long long)p.N * p.C;
  const int P = p.Ho * p.Wo;
  if (planes <= 0 || P <= 0) return;
  const long long plane_bytes = (long long)p.H * p.W * (long long)sizeof(T);
  int v = p.variant;
  if (v == 0) {
    // measured on the SqueezeNet pools (batch 256): one plane per block from LDS for planes of
    // >= 2048 elements up to 48 KB (f32 pool1 485 -> 367 us, pool3 318 -> 227 us; f16 pool1 617 ->
    // 204, pool3 380 -> 186); 27x27 planes: the direct kernel for f32 (150 us vs strip 171), the
    // column strip for f16 (120 us vs direct 169)
    // Evenly spaced planes (every SqueezeNet pool in the fused graph): the chunk-staged kernel with
    // 12 KB of LDS per block (pool3 205 -> 196 us, pool5 162 -> 99 us; 24 / 48 KB measured slower)
    const bool s332 = p.kh == 3 && p.kw == 3 && p.sh == 2;
    constexpr int EV = 16 / (int)sizeof(T);
    if (p.x_nstride == (long long)p.C * p.x_ps && p.y_nstride == (long long)p.C * p.y_ps && p.x_ps % EV == 0 &&
        (reinterpret_cast<uintptr_t>(p.x) & 15) == 0 && (long long)p.x_ps * (long long)sizeof(T) <= 12 * 1024)
      v = 5;
    else if ((long long)p.H * p.W >= 2048 && plane_bytes <= 48 * 1024)
      v = 4;
    else if (s332 && (plane_bytes > 48 * 1024 || sizeof(T) == 2))
      v = 3;
    else
      v = 2;
  }
  if (v == 5) {  // chunk-staged (falls through when the planes are not evenly spaced)
    constexpr int EV = 16 / (int)sizeof(T);
    const long long lds_budget = POOL_CHUNK_BYTES;
    const long long pbytes = (long long)p.x_ps * (long long)sizeof(T);
    int pb = (int)(lds_budget / pbytes);
    if (pb > 64) pb = 64;
    if (p.x_nstride == (long long)p.C * p.x_ps && p.y_nstride == (long long)p.C * p.y_ps && p.x_ps % EV == 0 &&
        (reinterpret_cast<uintptr_t>(p.x) & 15) == 0 && pb >= 1) {
      const long long nblk = (planes + pb - 1) / pb;
      const size_t lds = (size_t)((pb - 1) * pbytes + plane_bytes);
      if (p.kh == 3 && p.kw == 3)
        hipLaunchKernelGGL((maxpool_chunk_kernel<T, 3, 3>), dim3((unsigned)nblk), dim3(256), lds, s, p, pb, planes);
      else
        hipLaunchKernelGGL((maxpool_chunk_kernel<T, 0, 0>), dim3((unsigned)nblk), dim3(256), lds, s, p, pb, planes);
      return;
    }
    v = 2;
  }
  if (v == 4 && plane_bytes <= 64 * 1024) {
    const int pb = 1;
    const long long nblk = (planes + pb - 1) / pb;
    const size_t lds = (size_t)(pb * plane_bytes);
    if (p.kh == 3 && p.kw == 3)
      hipLaunchKernelGGL((maxpool_planes_kernel<T, 3, 3>), dim3((unsigned)nblk), dim3(256), lds, s, p, pb, planes);
    else
      hipLaunchKernelGGL((maxpool_planes_kernel<T, 0, 0>), dim3((unsigned)nblk), dim3(256), lds, s, p, pb, planes);
    return;
  }
  if (v == 3 && p.kh == 3 && p.kw == 3 && p.sh == 2) {
    const long long cols = planes * p.Wo;
    const dim3 grid((unsigned)((cols + 255) / 256), (unsigned)((p.Ho + POOL_STRIP_RB - 1) / POOL_STRIP_RB));
    hipLaunchKernelGGL((maxpool_strip_kernel<T, 3, 3, 2, POOL_STRIP_RB>), grid, dim3(256), 0, s, p, cols);
    return;
  }
  int chunks = (P + 255) / 256;
  if (chunks > 64) chunks = 64;
  if (p.kh == 3 && p.kw == 3)
    hipLaunchKernelGGL((maxpool_kernel<T, 3, 3>), dim3((unsigned)(planes * chunks)), dim3(256), 0, s, p, chunks);
  else
    hipLaunchKernelGGL((maxpool_kernel<T, 0, 0>), dim3((unsigned)(planes * chunks)), dim3(256), 0, s, p, chunks);
}

void launch_maxpool(const PoolParams& p, hipStream_t s) {
  if (p.es == 2)
    launch_maxpool_t<_Float16>(p, s);
  else
    launch_maxpool_t<float>(p, s);
}

// ------------------------------------------------------------------------------------------
// Relu: 16-B vectorised grid-stride stream (HBM-bound: 8 bytes moved per element).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void relu_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                   long long n) {
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * 256;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  float4* y4 = reinterpret_cast<float4*>(y);
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
    float4 v = x4[i];
    v.x = fmaxf(v.x, 0.0f);
    v.y = fmaxf(v.y, 0.0f);
    v.z = fmaxf(v.z, 0.0f);
    v.w = fmaxf(v.w, 0.0f);
    y4[i] = v;
  }
  for (long long i = (n4 << 2) + (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    y[i] = fmaxf(x[i], 0.0f);
}

__global__ __launch_bounds__(256) void relu_scalar_kernel(const float* __restrict__ x,
                                                          float* __restrict__ y, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    y[i] = fmaxf(x[i], 0.0f);
}

__global__ __launch_bounds__(256) void relu_f16_kernel(const _Float16* __restrict__ x, _Float16* __restrict__ y,
                                                       long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const _Float16 v = x[i];
    y[i] = v > (_Float16)0 ? v : (_Float16)0;  // max(x, 0); -0 and NaN as f32 fmaxf would give
  }
}

static unsigned stream_blocks(long long work) {
  long long b = (work + 255) / 256;
  if (b > 256 * 8) b = 256 * 8;
  if (b < 1) b = 1;
  return (unsigned)b;
}

void launch_relu(const float* x, float* y, long long n, hipStream_t s) {
  const bool aligned = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0;
  if (aligned)
    hipLaunchKernelGGL(relu_kernel, dim3(stream_blocks(n >> 2)), dim3(256), 0, s, x, y, n);
  else
    hipLaunchKernelGGL(relu_scalar_kernel, dim3(stream_blocks(n)), dim3(256), 0, s, x, y, n);
}

void launch_relu_f16(const void* x, void* y, long long n, hipStream_t s) {
  hipLaunchKernelGGL(relu_f16_kernel, dim3(stream_blocks(n)), dim3(256), 0, s, static_cast<const _Float16*>(x),
                     static_cast<_Float16*>(y), n);
}

// ------------------------------------------------------------------------------------------
// Add with broadcast of b (4-D strides with 0 on broadcast axes) onto a's 4-D shape.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void add_bcast_kernel(AddParams p) {
  const long long total = p.d[0] * p.d[1] * p.d[2] * p.d[3];
  for (long long idx = (long long)blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * 256) {
    long long t = idx;
    const long long i3 = t % p.d[3]; t /= p.d[3];
    const long long i2 = t % p.d[2]; t /= p.d[2];
    const long long i1 = t % p.d[1];
    const long long i0 = t / p.d[1];
    p.y[idx] = p.a[idx] + p.b[i0 * p.bs[0] + i1 * p.bs[1] + i2 * p.bs[2] + i3 * p.bs[3]];
  }
}

void launch_add_bcast(const AddParams& p, hipStream_t s) {
  const long long total = p.d[0] * p.d[1] * p.d[2] * p.d[3];
  hipLaunchKernelGGL(add_bcast_kernel, dim3(stream_blocks(total)), dim3(256), 0, s, p);
}

// ------------------------------------------------------------------------------------------
// Softmax over rows of length D (softmax_wrapper, softmax_op.rs:45-57): one wavefront per row,
// no LDS and no barrier.  Lane l owns elements i = 64 k + l (coalesced 256-B row segments).
//  * max: each lane's running max, then a 6-step xor-shuffle butterfly (exact: max is
//    order-free).
//  * denominator in ndarray's unrolled_fold order, exactly: 8 partial sums p_j = e[j] + e[8 + j] +
//    e[16 + j] + ... folded sequentially over the chunks c < D / 8, combined as
//    ((p0 + p4) + (p1 + p5)) + (p2 + p6) + (p3 + p7), then the < 8 tail elements in order.  Since 64
//    is a multiple of 8, element i = 64 k + l of lane l belongs to partial j = l % 8 and chunk
//    c = 8 k + l / 8.  Per k the wave holds chunks 8k .. 8k+7 in registers; lane l folds partial
//    l % 8 over them in ascending chunk order, fetching chunk 8k + g's element from lane
//    8 g + l % 8 by a cross-lane shuffle (ds_bpermute).  Every lane of a partial runs the same
//    chain, so p_j is the reference's sequential fold, bit for bit given the same exponentials.
//  * y = e / sum (a division, as `exp_x / &sum_exp_x`).  Rows up to 1024 keep x and e in registers
//    (one read of x, one write of y); longer rows stage e in y, re-read only by the lane that wrote it.
// ------------------------------------------------------------------------------------------
template <int NE>  // elements per lane held in registers: D <= 64 NE
__global__ __launch_bounds__(256) void softmax_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                      long long rows, int D) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;  // wave-uniform; no barrier in this kernel
  const float* xr = x + row * D;
  float* yr = y + row * D;
  float e[NE];
#pragma unroll
  for (int k = 0; k < NE; ++k) e[k] = 64 * k + lane < D ? xr[64 * k + lane] : -INFINITY;  // all loads in flight
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < NE; ++k) m = fmaxf(e[k], m);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));

  const int nfull8 = D / 8 * 8;  // elements inside the 8-wide chunks
  const int j = lane & 7;
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    const int i = 64 * k + lane;
    e[k] = i < D ? expf(e[k] - m) : 0.0f;
    const float ec = i < nfull8 ? e[k] : 0.0f;  // s + 0 == s: elements past the chunks add nothing
    if (64 * k < nfull8) {  // wave-uniform
      float sh[8];
#pragma unroll
      for (int g = 0; g < 8; ++g) sh[g] = __shfl(ec, 8 * g + j);  // chunks 8k .. 8k+7 of partial j
#pragma unroll
      for (int g = 0; g < 8; ++g) s = s + sh[g];
    }
  }
  const float p0 = __shfl(s, 0), p1 = __shfl(s, 1), p2 = __shfl(s, 2), p3 = __shfl(s, 3);
  const float p4 = __shfl(s, 4), p5 = __shfl(s, 5), p6 = __shfl(s, 6), p7 = __shfl(s, 7);
  float sum = 0.0f;
  sum = sum + (p0 + p4);
  sum = sum + (p1 + p5);
  sum = sum + (p2 + p6);
  sum = sum + (p3 + p7);
  // the < 8 tail elements share one register slot (nfull8 is a multiple of 8); select it without
  // dynamic register indexing, then fold the tail in order
  const int kt = nfull8 / 64;
  float et = 0.0f;
#pragma unroll
  for (int k = 0; k < NE; ++k) et = k == kt ? e[k] : et;
  for (int i = nfull8; i < D; ++i) sum = sum + __shfl(et, i % 64);
#pragma unroll
  for (int k = 0; k < NE; ++k)
    if (64 * k + lane < D) yr[64 * k + lane] = e[k] / sum;
}

// rows longer than 1024: the same order, e staged in y (re-read only by the lane that wrote it)
__global__ __launch_bounds__(256) void softmax_long_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                           long long rows, int D) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + row * D;
  float* yr = y + row * D;
  float m = -INFINITY;
  for (int i = lane; i < D; i += 64) m = fmaxf(xr[i], m);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  const int nfull8 = D / 8 * 8;
  const int j = lane & 7;
  float s = 0.0f;
  for (int i0 = 0; i0 < D; i0 += 64) {  // wave-uniform trip count
    const int i = i0 + lane;
    float e = 0.0f;
    if (i < D) {
      e = expf(xr[i] - m);
      yr[i] = e;
    }
    const float ec = i < nfull8 ? e : 0.0f;
    if (i0 < nfull8) {
#pragma unroll
      for (int g = 0; g < 8; ++g) s = s + __shfl(ec, 8 * g + j);
    }
  }
  const float p0 = __shfl(s, 0), p1 = __shfl(s, 1), p2 = __shfl(s, 2), p3 = __shfl(s, 3);
  const float p4 = __shfl(s, 4), p5 = __shfl(s, 5), p6 = __shfl(s, 6), p7 = __shfl(s, 7);
  float sum = 0.0f;
  sum = sum + (p0 + p4);
  sum = sum + (p1 + p5);
  sum = sum + (p2 + p6);
  sum = sum + (p3 + p7);
  for (int i = nfull8; i < D; ++i) sum = sum + expf(xr[i] - m);  // the tail, in order (same e values)
  for (int i = lane; i < D; i += 64) yr[i] = yr[i] / sum;
}

void launch_softmax(const float* x, float* y, long long rows, int D, hipStream_t s) {
  if (rows <= 0) return;
  const dim3 grid((unsigned)((rows + 3) / 4));
  if (D <= 256)
    hipLaunchKernelGGL(softmax_kernel<4>, grid, dim3(256), 0, s, x, y, rows, D);
  else if (D <= 1024)
    hipLaunchKernelGGL(softmax_kernel<16>, grid, dim3(256), 0, s, x, y, rows, D);
  else
    hipLaunchKernelGGL(softmax_long_kernel, grid, dim3(256), 0, s, x, y, rows, D);
}

// ------------------------------------------------------------------------------------------
// GlobalAveragePool: 64 (image, channel) rows per block are staged through LDS with coalesced
// loads, then each lane sums its row sequentially (the reference's order) and divides.
// ------------------------------------------------------------------------------------------
template <typename T>  // input element type (f32 sums either way)
__global__ __launch_bounds__(256) void gap_kernel(const T* __restrict__ x, float* __restrict__ y,
                                                  long long rows, int HW, int ps) {
  // 64 rows of HW elements at an odd LDS row stride (HW | 1: the 64 summing lanes read 64 distinct
  // banks; a 172-float stride would put 4 lanes on each bank), each wave copying 16 rows with
  // coalesced loads along the row
  extern __shared__ float tile[];  // 64 * (HW | 1) floats
  const int ls = HW | 1;
  const long long r0 = (long long)blockIdx.x * 64;  // (reverse order measured equal: 39.7 vs 39.5 us)
  const int nr = (int)(rows - r0 < 64 ? rows - r0 : 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (HW <= 256) {  // every load of the wave's 16 rows in flight before the first LDS store
    float v[16][4];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int r = wave + 4 * j;
      const T* __restrict__ src = x + (r0 + (r < nr ? r : 0)) * ps;
#pragma unroll
      // non-temporal loads (read once): 39.3 -> 36.8 us for SqueezeNet's pool10 at B = 256
      for (int u = 0; u < 4; ++u) v[j][u] = (lane + 64 * u < HW) ? (float)__builtin_nontemporal_load(src + lane + 64 * u) : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int r = wave + 4 * j;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (r < nr && lane + 64 * u < HW) tile[r * ls + lane + 64 * u] = v[j][u];
    }
  } else {
    for (int r = wave; r < nr; r += 4) {
      const T* __restrict__ src = x + (r0 + r) * ps;
      for (int c = lane; c < HW; c += 64) tile[r * ls + c] = (float)src[c];
    }
  }
  __syncthreads();
  if (threadIdx.x < nr) {
    const float* tr = tile + threadIdx.x * ls;
    float s = 0.0f;
    for (int i = 0; i < HW; ++i) s = s + tr[i];
    y[r0 + threadIdx.x] = s / (float)HW;
  }
}


template <typename T>
__global__ __launch_bounds__(64) void gap_big_kernel(const T* __restrict__ x, float* __restrict__ y,
                                                     long long rows, int HW, int ps) {
  const long long r = (long long)blockIdx.x * 64 + threadIdx.x;
  if (r >= rows) return;
  const T* tr = x + r * ps;
  float s = 0.0f;
  for (int i = 0; i < HW; ++i) s = s + (float)tr[i];
  y[r] = s / (float)HW;
}

template <typename T>
static void launch_gap_t(const T* x, float* y, long long rows, int HW, int ps, hipStream_t s) {
  if (rows <= 0) return;
  const size_t lds = (size_t)64 * (HW | 1) * sizeof(float);
  if (lds <= 64 * 1024)
    hipLaunchKernelGGL(gap_kernel<T>, dim3((unsigned)((rows + 63) / 64)), dim3(256), lds, s, x, y, rows, HW, ps);
  else
    hipLaunchKernelGGL(gap_big_kernel<T>, dim3((unsigned)((rows + 63) / 64)), dim3(64), 0, s, x, y, rows, HW, ps);
}

void launch_gap(const void* x, int es, float* y, long long rows, int HW, int ps, hipStream_t s) {
  if (es == 2)
    launch_gap_t(static_cast<const _Float16*>(x), y, rows, HW, ps, s);
  else
    launch_gap_t(static_cast<const float*>(x), y, rows, HW, ps, s);
}

// ------------------------------------------------------------------------------------------
// Concat of two row-major tensors along an axis: outer blocks of (inner_a | inner_b).
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void concat_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                     T* __restrict__ y, long long outer,
                                                     long long ia, long long ib) {
  const long long row = ia + ib;
  const long long total = outer * row;
  for (long long idx = (long long)blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * 256) {
    const long long o = idx / row, r = idx - o * row;
    y[idx] = r < ia ? a[o * ia + r] : b[o * ib + (r - ia)];
  }
}

void launch_concat(const void* a, const void* b, void* y, int es, long long outer, long long ia, long long ib,
                   hipStream_t s) {
  const dim3 grid(stream_blocks(outer * (ia + ib)));
  if (es == 2)
    hipLaunchKernelGGL(concat_kernel<_Float16>, grid, dim3(256), 0, s, static_cast<const _Float16*>(a),
                       static_cast<const _Float16*>(b), static_cast<_Float16*>(y), outer, ia, ib);
  else
    hipLaunchKernelGGL(concat_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(a),
                       static_cast<const float*>(b), static_cast<float*>(y), outer, ia, ib);
}

}  // namespace ore
