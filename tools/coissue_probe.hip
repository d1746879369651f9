// Co-issue probe: does a wave's VALU stream run beside its SIMD partner's back-to-back MFMAs?
// One 512-thread workgroup per CU (LDS request forces it), so waves w and w + 4 share a SIMD.  Waves
// 0-3 run N MFMAs (independent accumulators), waves 4-7 run V independent v_add / v_fma chains; each
// wave stamps s_memtime before and after its stream.  Kinds: MFMA f32 32x32x2, f32 16x16x4,
// bf16 32x32x16 (control); VALU alone / MFMA alone / both.
// Build + run: hipcc --offload-arch=gfx950 -O3 tools/coissue_probe.hip -o gpurun_out/coissue && gpurun_out/coissue
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));

// MODE 0: MFMA waves 0-3, VALU waves 4-7; 1: the VALU waves at s_setprio 3; 2: roles swapped (VALU
// waves 0-3 older)
template <int KIND, bool DO_MFMA, bool DO_VALU, int MODE = 0>
__global__ __launch_bounds__(512, 1) void probe(unsigned long long* t, float* out, int nm, int nv, float a0) {
  extern __shared__ float lds[];
  if (a0 == 12345.f) lds[threadIdx.x] = a0;
  const int wave = (MODE == 2 ? (threadIdx.x >> 6) ^ 4 : threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (MODE == 1 && wave >= 4) __builtin_amdgcn_s_setprio(3);
  float a = a0 + lane, b = a0 - lane;
  float s = 0.f;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (wave < 4) {
    if (DO_MFMA) {
      if (KIND == 0) {
        f16v acc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
        for (int k = 0; k < nm; k += 4) {
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][15];
      } else if (KIND == 1) {
        f4 acc[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < nm; k += 8) {
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][3];
      } else {
        bf8 av, bv;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          av[e] = (__bf16)(a + e);
          bv[e] = (__bf16)(b - e);
        }
        f16v acc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
        for (int k = 0; k < nm; k += 4) {
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc[i], 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][15];
      }
    }
  } else if (DO_VALU) {
    float x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = a + i;
    for (int k = 0; k < nv; k += 8) {
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], b, 1.0f);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) t[blockIdx.x * 8 + wave] = t1 - t0;
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

template <int KIND, bool M, bool V, int MODE = 0>
static void run(const char* name, unsigned long long* dt, float* dout, int nm, int nv, int nwg) {
  const size_t lds = 96 * 1024;
  hipFuncSetAttribute(reinterpret_cast<const void*>(&probe<KIND, M, V, MODE>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      160 * 1024);
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL((probe<KIND, M, V, MODE>), dim3(nwg), dim3(512), lds, 0, dt, dout, nm, nv, 1.0f);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(nwg * 8);
  hipMemcpy(h.data(), dt, h.size() * 8, hipMemcpyDeviceToHost);
  double mf = 0, va = 0;
  for (int b = 0; b < nwg; ++b) {
    for (int w = 0; w < 4; ++w) mf += h[b * 8 + w];
    for (int w = 4; w < 8; ++w) va += h[b * 8 + w];
  }
  mf /= 4.0 * nwg;
  va /= 4.0 * nwg;
  printf("%-34s mfma waves %9.0f cyc (%6.1f / mfma)   valu waves %9.0f cyc (%5.2f / valu)\n", name, mf,
         M ? mf / nm : 0.0, va, V ? va / nv : 0.0);
}

int main() {
  const int nwg = 256, nm = 2048, nv = 16384;
  unsigned long long* dt;
  float* dout;
  hipMalloc(&dt, nwg * 8 * 8);
  hipMalloc(&dout, nwg * 512 * 4);
  run<0, false, true>("VALU alone (fma)", dt, dout, nm, nv, nwg);
  run<0, true, false>("f32 32x32x2 alone", dt, dout, nm, nv, nwg);
  run<0, true, true>("f32 32x32x2 + partner VALU", dt, dout, nm, nv, nwg);
  run<1, true, false>("f32 16x16x4 alone", dt, dout, nm, nv, nwg);
  run<1, true, true>("f32 16x16x4 + partner VALU", dt, dout, nm, nv, nwg);
  run<2, true, false>("bf16 32x32x16 alone", dt, dout, nm, nv, nwg);
  run<2, true, true>("bf16 32x32x16 + partner VALU", dt, dout, nm, nv, nwg);
  run<0, true, true, 1>("f32 32x32x2 + VALU at prio 3", dt, dout, nm, nv, nwg);
  run<1, true, true, 1>("f32 16x16x4 + VALU at prio 3", dt, dout, nm, nv, nwg);
  run<2, true, true, 1>("bf16 32x32x16 + VALU at prio 3", dt, dout, nm, nv, nwg);
  run<0, true, true, 2>("f32 32x32x2 + older VALU waves", dt, dout, nm, nv, nwg);
  run<1, true, true, 2>("f32 16x16x4 + older VALU waves", dt, dout, nm, nv, nwg);
  return 0;
}
