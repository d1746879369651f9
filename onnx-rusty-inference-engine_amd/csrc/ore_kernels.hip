// MI355X (gfx950 / CDNA4) kernels for the fp32 ONNX op path of
// jackperlo/onnx-rusty-inference-engine (src/inference_fp32_ops/*).  Written for 64-lane waves
// and the f32-input MFMA (v_mfma_f32_32x32x2_f32: exact f32 fma chain, 157 TFLOP/s peak).
//
//   conv_gemm_kernel   Conv (convolution_op.rs:94-517) as an implicit GEMM, M = Cout,
//                      N = images*Ho*Wo, K = Cin*kh*kw, with the reference's resolved padding;
//                      bias (+ optional Relu) fused into the epilogue; output may be a channel
//                      slice of a wider tensor (Concat in place).  Also MatMul (mul_op.rs:23)
//                      as a 1x1 "conv" with K-major weights.
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

#include "ore_kernels.h"

namespace ore {

typedef float floatx16 __attribute__((ext_vector_type(16)));

// ------------------------------------------------------------------------------------------
// Implicit-GEMM convolution on MFMA 32x32x2 f32.
//   Block: 256 threads = 4 waves laid WAVES_M x WAVES_N; block tile BM x BN; BK = 16.
//   A (weights) tile staged in LDS as As[k][m]; B (im2col of the input, gathered on the fly)
//   as Bs[k][n].  Double-buffered LDS, register prefetch of the next K tile.
//   Fragment maps (cdna_hip_programming.md §3): lane l holds A[l&31][k=l>>5], B[k=l>>5][l&31];
//   accumulator reg r of lane l is row (r&3)+8*(r>>2)+4*(l>>5), column l&31.
//   Columns are output pixels, so each accumulator register is stored as two 128-B runs.
// ------------------------------------------------------------------------------------------
template <int BM, int BN, int WAVES_M, int WAVES_N, bool IS1X1, bool W_KMAJOR>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvParams p) {
  constexpr int BK = 16;
  constexpr int TM = BM / WAVES_M, TN = BN / WAVES_N;
  constexpr int FM = TM / 32, FN = TN / 32;
  constexpr int AS = BM + 2;  // pad: the transposing A store is bank-conflict free
  constexpr int B_ROWS_PER_PASS = 256 / BN;
  constexpr int B_LOADS = BK / B_ROWS_PER_PASS;
  constexpr int A_LOADS = BM * BK / 256;
  static_assert(FM >= 1 && FN >= 1 && WAVES_M * WAVES_N == 4, "bad tile");
  static_assert(BK % B_ROWS_PER_PASS == 0 && (BM * BK) % 256 == 0, "bad tile");

  __shared__ float As[2][BK][AS];
  __shared__ float Bs[2][BK][BN];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm0 = (wave / WAVES_N) * TM;
  const int wn0 = (wave % WAVES_N) * TN;

  // XCD-aware bijective remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
  // blocks dealt round-robin over 8 XCDs; give each XCD a contiguous run of tiles with the
  // M tile fastest, so the M tiles that share one input (B) tile share that XCD's L2.
  const int nwg = p.mtiles * p.ntiles;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int mt = wgid % p.mtiles;
  const int nt = wgid / p.mtiles;
  const int m0 = mt * BM;
  const long long n0 = (long long)nt * BN;

  const int K = p.K;
  const int KK = p.kh * p.kw;
  const int HW = p.H * p.W;

  // --- B gather: this thread owns column bcol, rows krow + j*B_ROWS_PER_PASS
  const int bcol = tid % BN;
  const int krow = __builtin_amdgcn_readfirstlane(tid / BN);
  const long long bn = n0 + bcol;
  const bool bn_ok = bn < p.Ntot;
  long long xoff = 0;
  int ih0 = 0, iw0 = 0;
  {
    long long nn = bn_ok ? bn : 0;
    int img = (int)(nn / p.P);
    int pix = (int)(nn - (long long)img * p.P);
    xoff = (long long)img * p.x_nstride;
    if (IS1X1) {
      xoff += pix;
    } else {
      int oh = pix / p.Wo, ow = pix - oh * p.Wo;
      ih0 = oh * p.sh - p.pt;
      iw0 = ow * p.sw - p.pl;
    }
  }
  const float* __restrict__ x = p.x;
  const float* __restrict__ w = p.w;

  float breg[B_LOADS];
  float areg[A_LOADS];

  auto load_tile = [&](int k0) {
#pragma unroll
    for (int j = 0; j < B_LOADS; ++j) {
      const int k = k0 + krow + j * B_ROWS_PER_PASS;  // wave-uniform
      float v = 0.0f;
      if (IS1X1) {
        if (bn_ok && k < K) v = x[xoff + (long long)k * HW];
      } else {
        const int c = k / KK;
        const int rs = k - c * KK;
        const int rr = rs / p.kw;
        const int ss = rs - rr * p.kw;
        const int ih = ih0 + rr, iw = iw0 + ss;
        if (bn_ok && k < K && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W)
          v = x[xoff + (long long)c * HW + ih * p.W + iw];
      }
      breg[j] = v;
    }
#pragma unroll
    for (int j = 0; j < A_LOADS; ++j) {
      const int e = tid + j * 256;
      float v = 0.0f;
      if (W_KMAJOR) {
        const int m = e % BM, k = e / BM;
        if (m0 + m < p.M && k0 + k < K) v = w[(long long)(k0 + k) * p.M + m0 + m];
      } else {
        const int k = e % BK, m = e / BK;
        if (m0 + m < p.M && k0 + k < K) v = w[(long long)(m0 + m) * K + k0 + k];
      }
      areg[j] = v;
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int j = 0; j < B_LOADS; ++j) Bs[buf][krow + j * B_ROWS_PER_PASS][bcol] = breg[j];
#pragma unroll
    for (int j = 0; j < A_LOADS; ++j) {
      const int e = tid + j * 256;
      if (W_KMAJOR) As[buf][e / BM][e % BM] = areg[j];
      else As[buf][e % BK][e / BK] = areg[j];
    }
  };

  floatx16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  const int ntk = (K + BK - 1) / BK;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  const int lrow = lane >> 5, lcol = lane & 31;
  for (int t = 0; t < ntk; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntk) load_tile((t + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = As[buf][kk + lrow][wm0 + i * 32 + lcol];
#pragma unroll
      for (int j = 0; j < FN; ++j) bf[j] = Bs[buf][kk + lrow][wn0 + j * 32 + lcol];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < ntk) store_tile(buf ^ 1);
    __syncthreads();
  }

  // --- epilogue: + bias, optional relu, scatter to NCHW (channel slice of y)
  float* __restrict__ y = p.y;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const long long n = n0 + wn0 + j * 32 + lcol;
    if (n >= p.Ntot) continue;
    const int img = (int)(n / p.P);
    const int pix = (int)(n - (long long)img * p.P);
    float* yb = y + (long long)img * p.y_nstride + pix;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wm0 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * lrow;
        if (m < p.M) {
          float v = acc[i][j][e];
          if (p.bias) v = v + p.bias[m];
          if (p.relu) v = fmaxf(v, 0.0f);
          yb[(long long)m * p.P] = v;
        }
      }
    }
  }
}

template <int BM, int BN, int WM, int WN>
static void launch_conv_cfg(const ConvParams& p0, hipStream_t s) {
  ConvParams p = p0;
  p.mtiles = (p.M + BM - 1) / BM;
  p.ntiles = (int)((p.Ntot + BN - 1) / BN);
  dim3 grid(p.mtiles * p.ntiles), block(256);
  if (p.w_kmajor)
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, true, true>), grid, block, 0, s, p);
  else if (p.is1x1)
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, true, false>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, false, false>), grid, block, 0, s, p);
}

int conv_tile_config(int M) {
  if (M >= 128) return 2;
  if (M > 32) return 1;
  return 0;
}

void launch_conv(const ConvParams& p, hipStream_t s) {
  switch (conv_tile_config(p.M)) {
    case 2: launch_conv_cfg<128, 128, 2, 2>(p, s); break;
    case 1: launch_conv_cfg<64, 128, 2, 2>(p, s); break;
    default: launch_conv_cfg<32, 256, 1, 4>(p, s); break;
  }
}

// ------------------------------------------------------------------------------------------
// MaxPool: one output element per thread; the window reads zeros outside the image (the
// reference pads with 0, max_pool_op.rs:265-276) and starts from -FLT_MAX (:337).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void maxpool_kernel(PoolParams p) {
  const long long total = (long long)p.N * p.C * p.Ho * p.Wo;
  for (long long idx = (long long)blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * 256) {
    const int ow = (int)(idx % p.Wo);
    long long t = idx / p.Wo;
    const int oh = (int)(t % p.Ho);
    t /= p.Ho;
    const int c = (int)(t % p.C);
    const int n = (int)(t / p.C);
    const float* xp = p.x + (long long)n * p.x_nstride + (long long)c * p.H * p.W;
    const int ih0 = oh * p.sh - p.pt, iw0 = ow * p.sw - p.pl;
    float m = -FLT_MAX;
    for (int r = 0; r < p.kh; ++r) {
      const int ih = ih0 + r;
      const bool rok = (unsigned)ih < (unsigned)p.H;
      for (int s = 0; s < p.kw; ++s) {
        const int iw = iw0 + s;
        const float v = (rok && (unsigned)iw < (unsigned)p.W) ? xp[ih * p.W + iw] : 0.0f;
        m = fmaxf(m, v);
      }
    }
    p.y[(long long)n * p.y_nstride + ((long long)c * p.Ho + oh) * p.Wo + ow] = m;
  }
}

void launch_maxpool(const PoolParams& p, hipStream_t s) {
  const long long total = (long long)p.N * p.C * p.Ho * p.Wo;
  long long blocks = (total + 255) / 256;
  if (blocks > 256 * 16) blocks = 256 * 16;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(maxpool_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p);
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
// Softmax over rows of length D.  One 256-thread block per row: the max is an exact
// reduction; e = expf(x - max) is written to y; the denominator is formed in the reference's
// own order (ndarray unrolled_fold: 8 partial sums over chunks of 8, combined (p0+p4),
// (p1+p5), (p2+p6), (p3+p7), then the tail) by 8 lanes; then y = e / sum.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void softmax_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                      int D) {
  __shared__ float red[4];
  __shared__ float part[8];
  const long long row = blockIdx.x;
  const float* xr = x + row * D;
  float* yr = y + row * D;
  const int tid = threadIdx.x;

  float m = -INFINITY;
  for (int i = tid; i < D; i += 256) m = fmaxf(xr[i], m);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  if ((tid & 63) == 0) red[tid >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));

  for (int i = tid; i < D; i += 256) yr[i] = expf(xr[i] - m);
  __syncthreads();  // block-scope visibility of yr for the 8 summing lanes (same CU, L1 write-through of own stores)
  const int nfull = D / 8;
  if (tid < 8) {
    float s = 0.0f;
    for (int c = 0; c < nfull; ++c) s = s + yr[c * 8 + tid];
    part[tid] = s;
  }
  __syncthreads();
  float sum = 0.0f;
  sum = sum + (part[0] + part[4]);
  sum = sum + (part[1] + part[5]);
  sum = sum + (part[2] + part[6]);
  sum = sum + (part[3] + part[7]);
  for (int i = nfull * 8; i < D; ++i) sum = sum + yr[i];
  __syncthreads();
  for (int i = tid; i < D; i += 256) yr[i] = yr[i] / sum;
}

void launch_softmax(const float* x, float* y, long long rows, int D, hipStream_t s) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(softmax_kernel, dim3((unsigned)rows), dim3(256), 0, s, x, y, D);
}

// ------------------------------------------------------------------------------------------
// GlobalAveragePool: 64 (image, channel) rows per block are staged through LDS with coalesced
// loads, then each lane sums its row sequentially (the reference's order) and divides.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gap_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                  long long rows, int HW) {
  extern __shared__ float tile[];  // 64 * HW floats
  const long long r0 = (long long)blockIdx.x * 64;
  const long long nr = rows - r0 < 64 ? rows - r0 : 64;
  const long long base = r0 * HW;
  const long long cnt = nr * HW;
  for (long long i = threadIdx.x; i < cnt; i += 256) tile[i] = x[base + i];
  __syncthreads();
  if (threadIdx.x < nr) {
    const float* tr = tile + (long long)threadIdx.x * HW;
    float s = 0.0f;
    for (int i = 0; i < HW; ++i) s = s + tr[i];
    y[r0 + threadIdx.x] = s / (float)HW;
  }
}

__global__ __launch_bounds__(64) void gap_big_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                     long long rows, int HW) {
  const long long r = (long long)blockIdx.x * 64 + threadIdx.x;
  if (r >= rows) return;
  const float* tr = x + r * HW;
  float s = 0.0f;
  for (int i = 0; i < HW; ++i) s = s + tr[i];
  y[r] = s / (float)HW;
}

void launch_gap(const float* x, float* y, long long rows, int HW, hipStream_t s) {
  if (rows <= 0) return;
  const unsigned blocks = (unsigned)((rows + 63) / 64);
  const size_t lds = (size_t)64 * HW * sizeof(float);
  if (lds <= 64 * 1024)
    hipLaunchKernelGGL(gap_kernel, dim3(blocks), dim3(256), lds, s, x, y, rows, HW);
  else
    hipLaunchKernelGGL(gap_big_kernel, dim3(blocks), dim3(64), 0, s, x, y, rows, HW);
}

// ------------------------------------------------------------------------------------------
// Concat of two row-major tensors along an axis: outer blocks of (inner_a | inner_b).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void concat_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                     float* __restrict__ y, long long outer,
                                                     long long ia, long long ib) {
  const long long row = ia + ib;
  const long long total = outer * row;
  for (long long idx = (long long)blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * 256) {
    const long long o = idx / row, r = idx - o * row;
    y[idx] = r < ia ? a[o * ia + r] : b[o * ib + (r - ia)];
  }
}

void launch_concat(const float* a, const float* b, float* y, long long outer, long long ia, long long ib,
                   hipStream_t s) {
  hipLaunchKernelGGL(concat_kernel, dim3(stream_blocks(outer * (ia + ib))), dim3(256), 0, s, a, b, y,
                     outer, ia, ib);
}

}  // namespace ore
