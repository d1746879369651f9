// HBM stream probes for the HBM-bound launches' roofline (SURVEY.md §8(d) "achievable peaks"):
// read-only, write-only and copy streams over 2 GiB buffers (far past the 256 MB MALL), each with
// plain and non-temporal (nt) accesses and 4 / 8 16-B accesses in flight per thread.
// Build + run: bash tools/peaks.sh hbm   (one line per probe, GB/s of algorithmic bytes).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void read_kernel(const floatx4* __restrict__ x, float* __restrict__ out, long long n4) {
  const long long stride = (long long)gridDim.x * 256;
  floatx4 s = {0, 0, 0, 0};
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i + (U - 1) * stride < n4; i += U * stride) {
    floatx4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(x + i + u * stride) : x[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u];
  }
  if (s.x + s.y + s.z + s.w == 1234.5f) out[threadIdx.x] = s.x;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void write_kernel(floatx4* __restrict__ y, long long n4, float v0) {
  const long long stride = (long long)gridDim.x * 256;
  const floatx4 v = {v0, v0, v0, v0};
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i + (U - 1) * stride < n4; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v, y + i + u * stride);
      else y[i + u * stride] = v;
    }
  }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_kernel(const floatx4* __restrict__ x, floatx4* __restrict__ y, long long n4) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i + (U - 1) * stride < n4; i += U * stride) {
    floatx4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], y + i + u * stride);
      else y[i + u * stride] = v[u];
    }
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

static hipEvent_t e0, e1;

template <typename F>
static double time_ms(F launch, int reps) {
  launch();
  launch();
  (void)hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) launch();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const long long n4 = (2LL << 30) / 16;
  const double bytes = n4 * 16.0;
  floatx4 *x, *y;
  float* out;
  CK(hipMalloc(&x, n4 * 16));
  CK(hipMalloc(&y, n4 * 16));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(x, 0, n4 * 16));
  for (int wpc : {4, 8, 16}) {
    const int g = cus * wpc;
#define RUN(NAME, K, MUL, ...)                                                                          \
  {                                                                                                    \
    double ms = time_ms([&] { hipLaunchKernelGGL(K, dim3(g), dim3(256), 0, 0, __VA_ARGS__); }, 10);    \
    printf("%-22s wg/cu %2d  %7.1f GB/s\n", NAME, wpc, MUL * bytes / (ms * 1e-3) / 1e9);                \
  }
    RUN("read u4", (read_kernel<4, false>), 1, x, out, n4);
    RUN("read u8", (read_kernel<8, false>), 1, x, out, n4);
    RUN("read u8 nt", (read_kernel<8, true>), 1, x, out, n4);
    RUN("write u4", (write_kernel<4, false>), 1, y, n4, 1.0f);
    RUN("write u4 nt", (write_kernel<4, true>), 1, y, n4, 1.0f);
    RUN("copy u4", (copy_kernel<4, false>), 2, x, y, n4);
    RUN("copy u8", (copy_kernel<8, false>), 2, x, y, n4);
    RUN("copy u8 nt", (copy_kernel<8, true>), 2, x, y, n4);
  }
  return 0;
}
