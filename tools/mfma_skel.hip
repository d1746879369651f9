// MFMA-skeleton probe for the Winograd expand3x3 kernel design: how much of the
// f32 MFMA peak a grid of short-lived workgroups reaches with nothing but the MFMAs, the per-chunk
// barrier, the accumulator zeroing and a one-value-per-lane store -- the shape of conv_winol_kernel
// (4 waves x 16x16x4 f32, 128 accumulator registers, 2 workgroups per CU, 64 MFMAs per chunk and wave).
// Variants: barrier on / off, chunks per workgroup, persistent workgroups, the 32x32x2 shape.
// Build + run: hipcc --offload-arch=gfx950 -O3 tools/mfma_skel.hip -o gpurun_out/mfma_skel && ./gpurun_out/mfma_skel
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

// 16x16x4: 32 accumulators of 4 (128 registers); per chunk 2 k-steps x 32 MFMAs
template <bool BAR>
__global__ __launch_bounds__(256, 2) void skel16(float* out, int chunks, int items_per_wg, float a0) {
  extern __shared__ float lds[];  // 80 KB per workgroup: two workgroups per CU, as conv_winol_kernel
  if (a0 == 12345.f) lds[threadIdx.x] = a0;
  const int lane = threadIdx.x & 63;
  float a = a0 + lane, b = a0 - lane;
  for (int it = 0; it < items_per_wg; ++it) {
    f4 acc[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < chunks; ++c) {
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int i = 0; i < 32; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
      if (BAR) __syncthreads();
      a += 1.0f;
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[(blockIdx.x * items_per_wg + it) * 256 + threadIdx.x] = s;
  }
}

// 32x32x2 at 512 registers (one wave per SIMD): 16 accumulators of 16; per chunk 2 k-steps x 16 MFMAs
template <bool BAR>
__global__ __launch_bounds__(256, 1) void skel32(float* out, int chunks, int items_per_wg, float a0) {
  const int lane = threadIdx.x & 63;
  float a = a0 + lane, b = a0 - lane;
  for (int it = 0; it < items_per_wg; ++it) {
    f16v acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    for (int c = 0; c < chunks; ++c) {
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
      if (BAR) __syncthreads();
      a += 1.0f;
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) s += acc[i][e];
    out[(blockIdx.x * items_per_wg + it) * 256 + threadIdx.x] = s;
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <class K>
static int run(const char* name, K kern, int grid, int chunks, int items, double flops_per_mfma, int mfma_per_chunk_wave,
               float* out, size_t lds = 0) {
  if (lds) CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, out, chunks, items, 1.0f);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, out, chunks, items, 1.0f);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double flops = (double)grid * items * 4 * chunks * mfma_per_chunk_wave * flops_per_mfma;
  printf("%-44s grid %6d chunks %3d items %3d: %8.1f us  %6.1f TF/s\n", name, grid, chunks, items, 1000.0 * ms,
         flops / (ms * 1e-3) / 1e12);
  return 0;
}

int main() {
  float* out = nullptr;
  CK(hipMalloc(&out, sizeof(float) * 256 * 6272 * 4));
  const double F16 = 16.0 * 16 * 4 * 2, F32 = 32.0 * 32 * 2 * 2;
  // fire8/expand3x3 at batch 256: 6272 workgroups x 8 chunks (C = 64); fire4: 46656 waves / 4 = 11664 x 4
  run("16x16x4 2wg/CU barrier (winol shape f8)", skel16<true>, 6272, 8, 1, F16, 64, out, 80 * 1024);
  run("16x16x4 2wg/CU no barrier", skel16<false>, 6272, 8, 1, F16, 64, out, 80 * 1024);
  run("16x16x4 barrier, fire4 shape (4 chunks)", skel16<true>, 11664, 4, 1, F16, 64, out, 80 * 1024);
  run("16x16x4 barrier, 16 chunks (half the WGs)", skel16<true>, 3136, 16, 1, F16, 64, out, 80 * 1024);
  run("16x16x4 barrier, persistent 512 x 12", skel16<true>, 512, 8, 12, F16, 64, out, 80 * 1024);
  run("16x16x4 barrier, persistent 512 x 12 (no bar)", skel16<false>, 512, 8, 12, F16, 64, out, 80 * 1024);
  run("16x16x4 barrier, 512 WGs x 8 chunks (1 round)", skel16<true>, 512, 8, 1, F16, 64, out, 80 * 1024);
  run("16x16x4 barrier, 512 WGs x 96 chunks", skel16<true>, 512, 96, 1, F16, 64, out, 80 * 1024);
  run("32x32x2 1wg/CU barrier (f8: 3136 x 8)", skel32<true>, 3136, 8, 1, F32, 32, out);
  run("32x32x2 1wg/CU persistent 256 x 12", skel32<true>, 256, 8, 12, F32, 32, out);
  run("32x32x2 1wg/CU 256 WGs x 96 chunks", skel32<true>, 256, 96, 1, F32, 32, out);
  run("16x16x4 3 waves/SIMD (no LDS) barrier f8", skel16<true>, 6272, 8, 1, F16, 64, out);
  CK(hipFree(out));
  return 0;
}
