// Achievable-peak probes for the roofline denominators ("measure achievable
// peaks (copy kernel, MFMA loop) and report both"): an HBM stream copy, a dependent-free f32
// MFMA loop (v_mfma_f32_32x32x2_f32) and an f16 MFMA loop (v_mfma_f32_32x32x16_f16).
// Build + run: bash tools/peaks.sh  (prints one line per probe).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(256) void copy_kernel(const floatx4* __restrict__ x, floatx4* __restrict__ y, long long n4) {
  // 4 independent 16-B loads in flight per thread per trip (n4 is a multiple of 4 * grid)
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i + 3 * stride < n4; i += 4 * stride) {
    floatx4 v0 = x[i], v1 = x[i + stride], v2 = x[i + 2 * stride], v3 = x[i + 3 * stride];
    y[i] = v0; y[i + stride] = v1; y[i + 2 * stride] = v2; y[i + 3 * stride] = v3;
  }
}

template <int ACC>
__global__ __launch_bounds__(256) void mfma_f32_kernel(float* out, int iters, float a0) {
  floatx16 acc[ACC];
  for (int i = 0; i < ACC; ++i)
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.0f;
  float a = a0 + threadIdx.x, b = a0 - threadIdx.x;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  float s = 0.0f;
  for (int i = 0; i < ACC; ++i)
    for (int e = 0; e < 16; ++e) s += acc[i][e];
  if (s == 1234.5f) out[threadIdx.x] = s;  // keep the chain alive
}

template <int ACC>
__global__ __launch_bounds__(256) void mfma_f16_kernel(float* out, int iters, float a0) {
  floatx16 acc[ACC];
  for (int i = 0; i < ACC; ++i)
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.0f;
  half8 a, b;
  for (int e = 0; e < 8; ++e) { a[e] = (_Float16)(a0 + e); b[e] = (_Float16)(a0 - threadIdx.x); }
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[i], 0, 0, 0);
  float s = 0.0f;
  for (int i = 0; i < ACC; ++i)
    for (int e = 0; e < 16; ++e) s += acc[i][e];
  if (s == 1234.5f) out[threadIdx.x] = s;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms = 0;
  // HBM copy: 2 x 2 GiB buffers (far beyond the 256 MB MALL), read + write bytes
  const long long n4 = (2LL << 30) / 16;
  floatx4 *x, *y;
  CK(hipMalloc(&x, n4 * 16));
  CK(hipMalloc(&y, n4 * 16));
  CK(hipMemset(x, 0, n4 * 16));
  const int cblocks = cus * 8;  // 2 GiB / 16 B = 2^27 float4 = 4 * 2048 * 256 * 64 trips: divides evenly
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(copy_kernel, dim3(cblocks), dim3(256), 0, 0, x, y, n4);
  CK(hipEventRecord(e0));
  const int creps = 10;
  for (int r = 0; r < creps; ++r) hipLaunchKernelGGL(copy_kernel, dim3(cblocks), dim3(256), 0, 0, x, y, n4);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("hbm_copy_GBps %.1f  (2 GiB read + 2 GiB write per launch, %d launches)\n",
         2.0 * n4 * 16 * creps / (ms * 1e-3) / 1e9, creps);
  CK(hipFree(x));
  CK(hipFree(y));
  float* out;
  CK(hipMalloc(&out, 4096));
  const int iters = 4000, blocks = cus * 4;
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(mfma_f32_kernel<4>, dim3(blocks), dim3(256), 0, 0, out, 10, 1.0f);
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(mfma_f32_kernel<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  double flops = 2.0 * 32 * 32 * 2 * 4.0 * iters * (blocks * 4.0);
  printf("mfma_f32_32x32x2_TFLOPs %.1f\n", flops / (ms * 1e-3) / 1e12);
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(mfma_f16_kernel<4>, dim3(blocks), dim3(256), 0, 0, out, 10, 1.0f);
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(mfma_f16_kernel<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  flops = 2.0 * 32 * 32 * 16 * 4.0 * iters * (blocks * 4.0);
  printf("mfma_f16_32x32x16_TFLOPs %.1f\n", flops / (ms * 1e-3) / 1e12);
  CK(hipFree(out));
  return 0;
}
