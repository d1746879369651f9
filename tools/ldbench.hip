// Vector-memory throughput probe (tools/ldbench.sh): per-CU load rate of L2-resident data for the
// access shapes the conv kernels use, at 1 and 2 waves per SIMD.  Each wave loops over a 1 MiB
// table (L2-resident after the first pass), LOADS loads in flight per lane, and sums what it loaded
// so nothing is dead.  Prints bytes per clock per CU at the measured kernel time.
#include <hip/hip_runtime.h>
#pragma clang diagnostic ignored "-Wunused-result"

#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

// MODE 0: dwordx4, lane i at 16 i (1 KiB contiguous per wave-instruction)
// MODE 1: dword,   lane i at 4 i  (256 B contiguous)
// MODE 2: dwordx4, lane i at 8 i  (overlapping windows: 520 B span)
// MODE 3: dwordx4, lane i at 64 i (one 16-B piece per 64-B line: 4 KiB span)
// MODE 4: dwordx4 LDS-DMA (buffer_load_dwordx4 ... lds), lane i at 16 i
// MODE 5: dword LDS-DMA, lane i at 4 i
template <int MODE, int LOADS>
__global__ void ld_kernel(const float* __restrict__ x, float* out, int iters, int span_bytes) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), (short)0, 1 << 20, 0x00020000);
  const int stride = MODE == 0 || MODE == 4 ? 16 : MODE == 1 || MODE == 5 ? 4 : MODE == 2 ? 8 : 64;
  const int step = MODE == 3 ? 4096 : MODE == 2 ? 512 : MODE == 1 || MODE == 5 ? 256 : 1024;  // bytes per instruction
  int off = ((blockIdx.x * 8 + wave) * 4096 + lane * stride) & ((1 << 20) - 1);
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 4 || MODE == 5) {
#pragma unroll
      for (int l = 0; l < LOADS; ++l) {
        const unsigned la = (unsigned)(size_t)(__attribute__((address_space(3))) float*)lds + (wave * LOADS + l) * 1024;
        const int o = (off + l * step) & ((1 << 20) - 1 - 15);
        if constexpr (MODE == 4)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(size_t)la, 16, o, 0, 0, 0);
        else
          __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(size_t)la, 4, o, 0, 0, 0);
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (gfx9: bits 3:0 + 15:14)
      acc[0] += lds[(wave * LOADS) * 256 + lane];
    } else {
      f4 v[LOADS];
#pragma unroll
      for (int l = 0; l < LOADS; ++l) {
        const int o = (off + l * step) & ((1 << 20) - 1 - 15);
        if constexpr (MODE == 1) {
          v[l] = f4{__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, o, 0, 0)), 0.f, 0.f, 0.f};
        } else {
          v[l] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 0));
        }
      }
#pragma unroll
      for (int l = 0; l < LOADS; ++l) acc += v[l];
    }
    off = (off + LOADS * step) & ((1 << 20) - 1);
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 1.2345e-30f) out[threadIdx.x] = acc[0];
}

template <int MODE, int LOADS>
static void run(const char* name, const float* x, float* out, int waves_per_cu, int ncu, int bytes_per_lane) {
  const int blocks = ncu * (waves_per_cu / 4), iters = 2000;
  const size_t lds = (size_t)4 * LOADS * 1024;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((ld_kernel<MODE, LOADS>), dim3(blocks), dim3(256), lds, 0, x, out, 50, 1 << 20);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL((ld_kernel<MODE, LOADS>), dim3(blocks), dim3(256), lds, 0, x, out, iters, 1 << 20);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double bytes = (double)blocks * 256 * iters * LOADS * bytes_per_lane;
  const double clk = ms * 1e-3 * 2.4e9;  // nominal clock
  std::printf("%-34s waves/CU %d: %8.3f ms  %6.1f B/clk/CU  %7.2f TB/s  %6.3f lane-loads/clk/CU\n", name, waves_per_cu, ms,
              bytes / clk / ncu, bytes / (ms * 1e-3) / 1e12, bytes / bytes_per_lane / clk / ncu);
}

int main() {
  int dev = 0, ncu = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) == hipSuccess) ncu = prop.multiProcessorCount;
  float *x, *out;
  hipMalloc(&x, 1 << 20);
  hipMalloc(&out, 4096);
  hipMemset(x, 0, 1 << 20);
  for (int w : {4, 8}) {
    run<0, 8>("dwordx4 contiguous (16 B/lane)", x, out, w, ncu, 16);
    run<1, 8>("dword contiguous (4 B/lane)", x, out, w, ncu, 4);
    run<2, 8>("dwordx4 lanes 8 B apart", x, out, w, ncu, 16);
    run<3, 8>("dwordx4 lanes 64 B apart", x, out, w, ncu, 16);
    run<4, 4>("LDS-DMA dwordx4", x, out, w, ncu, 16);
    run<5, 4>("LDS-DMA dword", x, out, w, ncu, 4);
  }
  hipFree(x);
  hipFree(out);
  return 0;
}
