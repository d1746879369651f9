// f32 models: a 1x1 Conv (+ Relu) whose only reader is GlobalAveragePool, in one launch -- SqueezeNet's
// conv10 -> relu10 -> pool10 (reference convolution_op.rs:94-517, relu_op.rs:31-33,
// global_average_pool_op.rs:33-51); the f32 counterpart of conv1x1_gap_f16_kernel.  The unfused path
// writes the [N][1000][13][13] conv output (176 MB at batch 256) and gap_kernel reads it back.
//
// A workgroup is one image x 128 output channels (four waves x two 16-row tiles, v_mfma_f32_16x16x4_f32)
// x all of the image's P <= 16 NF pixels as NF 16-pixel fragments (169 -> 176 at 13x13: 16-pixel
// granularity wastes 4 %, 32-pixel fragments 14 %).  K in chunks of 32 input channels: a chunk is 32
// consecutive channel planes of the image, one contiguous run in HBM, copied global -> LDS by 16-B
// LDS-DMA into a double-buffered stage (the next chunk in flight during this one; plain loads when the
// planes are not 16-B aligned, e.g. an unpadded 13x13 map).  B (pixels) from the stage by one
// ds_read_b32 per fragment and k-step, each feeding both row tiles, the next k-step's read issued as
// the current one's MFMAs go out; A (weights) from L2 in launch_pack_cg_f32's layout (one 16-B load per
// lane and row tile covers four k-steps, in the lane's own k order: no selects).  The m-blocks of one image run consecutively on one XCD, so
// the image's map is read from HBM about once.  Epilogue: bias + Relu into an LDS tile [16 channels]
// [pixels] per wave (two passes), then one lane per channel sums the P pixels in order (gap_kernel's
// sequential sum) and divides by P.  Same operands, k order and f32 fma chain as the streaming conv
// kernels, the same summation as gap_kernel: bit-identical to the two launches
// (tests/test_conv_gap_gpu.py).  Three workgroups per CU (LDS and registers).
#include <hip/hip_runtime.h>

#include "ore_kernels.h"

namespace ore {

namespace {

typedef float cg4 __attribute__((ext_vector_type(4)));

constexpr int CG_KC = 32;         // input channels per chunk (8 k-steps of 4)
constexpr int CG_EPR = 16;        // channels per epilogue pass (per wave)
constexpr int CG_MB = 128;        // output channels per workgroup
constexpr int CG_RT = 2;          // 16-row tiles per wave
constexpr int CG_NW = 8 / CG_RT;  // waves per workgroup
constexpr int CG_NT = 64 * CG_NW;

__host__ __device__ constexpr int cg_ts(int nf) { return 16 * nf + 4; }  // epilogue tile row stride (floats)

template <int NF, bool DMA>  // NF 16-pixel fragments; DMA: 16-B aligned channel planes (else plain loads)
__global__ __launch_bounds__(CG_NT, (CG_RT * NF > 22 ? 2 : 3)) void conv1x1_gap_f32_kernel(Conv1x1GapF32 p, int stg) {
  extern __shared__ __attribute__((aligned(16))) float cg_lds[];
  const int tid = threadIdx.x, lane = tid & 63, lc = lane & 15, kq = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mblocks = (p.M + CG_MB - 1) / CG_MB;
  const int wgid = xcd_block_id();  // the m-blocks of one image consecutive: one XCD, one L2
  const int img = wgid / mblocks, m0 = (wgid - img * mblocks) * CG_MB + 16 * CG_RT * wave;
  const int Mp32 = (p.M + 31) / 32 * 32;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.x + (long long)img * p.x_nstride), (short)0, p.C * p.x_ps * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.wc), (short)0, ((p.C + 15) / 16) * Mp32 * 64, 0x00020000);
  const int chunk_bytes = CG_KC * p.x_ps * 4;
  const int ndma = (chunk_bytes + 1023) / 1024;  // 1 KiB per DMA instruction
  const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) float*)cg_lds;
  const float* xi = p.x + (long long)img * p.x_nstride;
  auto stage = [&](int c0, int buf) __attribute__((always_inline)) {
    if constexpr (DMA) {
      for (int i = wave; i < ndma; i += CG_NW)  // wave-uniform
        ore_lds_dma16(xr, lds0 + (unsigned)(buf * stg) * 4 + 1024u * i, 1024 * i + 16 * lane, c0 * p.x_ps * 4);
    } else {
      for (int i = tid; i < CG_KC * p.x_ps; i += CG_NT) cg_lds[buf * stg + i] = xi[(long long)c0 * p.x_ps + i];
    }
  };
  // A (v_mfma_f32_16x16x4f32: lane (lc, kq) holds row lc, k = 4 s + kq of k-step s): row tile r is rows
  // m0 + 16 r .. + 15.  The pack [k/16][row][kq][s] = W[row][16 q + 4 s + kq]: one 16-B load per lane and
  // row tile holds k-steps 4 q .. 4 q + 3 of the lane's kq, element s for k-step 4 q + s
  int arow[CG_RT];
#pragma unroll
  for (int r = 0; r < CG_RT; ++r) arow[r] = m0 + 16 * r + lc < Mp32 ? m0 + 16 * r + lc : 0;
  auto load_a = [&](int q, int r) __attribute__((always_inline)) {
    return __builtin_bit_cast(cg4, __builtin_amdgcn_raw_buffer_load_b128(wr, ((arow[r] * 4 + kq) * 4) * 4,
                                                                          q * Mp32 * 64, 0));
  };
  const int nq = (p.C + 15) / 16;
  cg4 acc[CG_RT][NF];
#pragma unroll
  for (int r = 0; r < CG_RT; ++r)
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[r][f] = cg4{0.0f, 0.0f, 0.0f, 0.0f};
  const int nch = p.C / CG_KC;
  const int bo = (kq * p.x_ps + lc) * 4;  // B: channel 4 j + kq, pixel 16 f + lc of the stage (bytes)
  const char* lb = reinterpret_cast<const char*>(cg_lds);
  stage(0, 0);
  cg4 a[2][CG_RT];  // [group parity][row tile]
#pragma unroll
  for (int r = 0; r < CG_RT; ++r) {
    a[0][r] = load_a(0, r);
    a[1][r] = load_a(1, r);
  }
  for (int ci = 0; ci < nch; ++ci) {
    const int buf = ci & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMAs of chunk ci (and its A groups)
    __syncthreads();  // every wave's; and every wave is done with the other stage (chunk ci - 1)
    if (ci + 1 < nch) stage((ci + 1) * CG_KC, buf ^ 1);
    const char* sb = lb + buf * stg * 4 + bo;
    float b[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) b[f] = *reinterpret_cast<const float*>(sb + f * 64);
#pragma unroll
    for (int j = 0; j < CG_KC / 4; ++j) {
      const int g = j >> 2, u = j & 3;  // group within the chunk (its parity = the global group's)
      float av[CG_RT];
#pragma unroll
      for (int r = 0; r < CG_RT; ++r) av[r] = a[g & 1][r][u];
#pragma unroll
      for (int f = 0; f < NF; ++f) {
#pragma unroll
        for (int r = 0; r < CG_RT; ++r) acc[r][f] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[r], b[f], acc[r][f], 0, 0, 0);
        if (j + 1 < CG_KC / 4) b[f] = *reinterpret_cast<const float*>(sb + (4 * (j + 1) * p.x_ps) * 4 + f * 64);
      }
      if (u == 3) {  // group consumed: refill its slot with the group two ahead
        const int q2 = ci * (CG_KC / 16) + g + 2;
        if (q2 < nq) {
#pragma unroll
          for (int r = 0; r < CG_RT; ++r) a[g & 1][r] = load_a(q2, r);
        }
      }
    }
  }
  // epilogue: lane (lc, kq) holds rows 16 r + 4 kq + e of pixel 16 f + lc.  Per pass CG_EPR rows of the
  // wave: bias + Relu into the wave's LDS tile [CG_EPR][TS], then lanes 0 .. CG_EPR - 1 each sum one
  // row's P pixels in order (gap_kernel's sequential sum) and divide by P
  __syncthreads();  // every wave is done with the stages: the tiles reuse the LDS
  constexpr int TS = cg_ts(NF);
  constexpr int KQP = CG_EPR / 4;  // kq values per pass
  float* tile = cg_lds + wave * CG_EPR * TS;
#pragma unroll
  for (int pass = 0; pass < 16 * CG_RT / CG_EPR; ++pass) {
    const int r = (pass * CG_EPR) / 16, kq0 = ((pass * CG_EPR) % 16) / 4;
    if (kq >= kq0 && kq < kq0 + KQP) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int tr = 4 * (kq - kq0) + e, m = m0 + CG_EPR * pass + tr;
        const float bv = p.bias && m < p.M ? p.bias[m] : 0.0f;
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          float v = acc[r][f][e] + bv;
          if (p.relu) v = fmaxf(v, 0.0f);
          tile[tr * TS + 16 * f + lc] = v;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int m = m0 + CG_EPR * pass + lane;
    if (lane < CG_EPR && m < p.M) {
      const float* tr = tile + lane * TS;
      float s = 0.0f;
      int i = 0;
      for (; i + 4 <= p.P; i += 4) {
        const cg4 v = *reinterpret_cast<const cg4*>(tr + i);
        s = s + v[0];
        s = s + v[1];
        s = s + v[2];
        s = s + v[3];
      }
      for (; i < p.P; ++i) s = s + tr[i];
      p.y[(long long)img * p.y_nstride + m] = s / (float)p.P;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

template <int NF, bool DMA>
static void cg_launch(const Conv1x1GapF32& p, hipStream_t s) {
  const int stg = (CG_KC * p.x_ps + 255) / 256 * 256 + 256;  // floats per stage (+ the last fragment's overrun)
  const size_t lds = (size_t)std::max(2 * stg, CG_NW * CG_EPR * cg_ts(NF)) * 4;
  if (lds > 64 * 1024) {  // above the default dynamic-LDS limit: raised once per device
    static std::atomic<unsigned long long> raised{0};
    ore_raise_lds_once(raised, reinterpret_cast<const void*>(&conv1x1_gap_f32_kernel<NF, DMA>), 160 * 1024);
  }
  const long long grid = (long long)p.N * ((p.M + CG_MB - 1) / CG_MB);
  hipLaunchKernelGGL((conv1x1_gap_f32_kernel<NF, DMA>), dim3((unsigned)grid), dim3(CG_NT), lds, s, p, stg);
}

template <bool DMA>
static void cg_dispatch(const Conv1x1GapF32& p, hipStream_t s) {
  switch ((p.P + 15) / 16) {
    case 1: cg_launch<1, DMA>(p, s); break;
    case 2: cg_launch<2, DMA>(p, s); break;
    case 3: cg_launch<3, DMA>(p, s); break;
    case 4: cg_launch<4, DMA>(p, s); break;
    case 5: cg_launch<5, DMA>(p, s); break;
    case 6: cg_launch<6, DMA>(p, s); break;
    case 7: cg_launch<7, DMA>(p, s); break;
    case 8: cg_launch<8, DMA>(p, s); break;
    case 9: cg_launch<9, DMA>(p, s); break;
    case 10: cg_launch<10, DMA>(p, s); break;
    case 11: cg_launch<11, DMA>(p, s); break;
    case 12: cg_launch<12, DMA>(p, s); break;
    case 13: cg_launch<13, DMA>(p, s); break;
    case 14: cg_launch<14, DMA>(p, s); break;
    case 15: cg_launch<15, DMA>(p, s); break;
    default: cg_launch<16, DMA>(p, s); break;
  }
}

}  // namespace

namespace {
__global__ __launch_bounds__(256) void pack_cg_f32_kernel(const float* __restrict__ w, int M, int K, int Mp32,
                                                          float* __restrict__ out) {
  const long long total = (long long)((K + 15) / 16) * Mp32 * 16;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int s = (int)(i & 3), kq = (int)((i >> 2) & 3);
    const long long rq = i >> 4;
    const int row = (int)(rq % Mp32), q = (int)(rq / Mp32);
    const int k = 16 * q + 4 * s + kq;
    out[i] = (row < M && k < K) ? w[(long long)row * K + k] : 0.0f;
  }
}
}  // namespace

size_t cg_f32_pack_bytes(int M, int K) { return size_t((K + 15) / 16) * size_t((M + 31) / 32 * 32) * 64; }

void launch_pack_cg_f32(const float* w, int M, int K, float* out, hipStream_t s) {
  const int Mp32 = (M + 31) / 32 * 32;
  long long blocks = ((long long)((K + 15) / 16) * Mp32 * 16 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pack_cg_f32_kernel, dim3((unsigned)blocks), dim3(256), 0, s, w, M, K, Mp32, out);
}

bool conv1x1_gap_f32_eligible(const Conv1x1GapF32& p) {
  return p.x && p.wc && p.y && p.N >= 1 && p.C >= CG_KC && p.C % CG_KC == 0 && p.P >= 1 && p.P <= 256 &&
         p.M >= 1 && p.x_ps >= p.P && (reinterpret_cast<uintptr_t>(p.x) & 3) == 0 &&
         (long long)p.C * p.x_ps * 4 < (1LL << 31) && (2 * CG_KC * p.x_ps + 512) * 4 <= 150 * 1024 &&
         (long long)p.N * ((p.M + CG_MB - 1) / CG_MB) < (1LL << 31);
}

void launch_conv1x1_gap_f32(const Conv1x1GapF32& p, hipStream_t s) {
  const bool dma = p.x_ps % 4 == 0 && (reinterpret_cast<uintptr_t>(p.x) & 15) == 0 && (p.x_nstride & 3) == 0;
  if (dma)
    cg_dispatch<true>(p, s);
  else
    cg_dispatch<false>(p, s);
}

}  // namespace ore
