// Host-ASan / UBSan driver for the planner (csrc/ore_model.cpp: ore_model_load_ex, plan(), the fusion
// passes, the arena and the walker's host side), run on the GPU box (the planner needs a HIP device;
// device code is built normally).  Through the C ABI only (include/ore.h):
//   model_fuzz MNIST.onnx SQUEEZENET.onnx ITERATIONS
// 1. MNIST-8 and SqueezeNet-1.0 load (f32 at batch 1, 4 and 700 -- 700 > run_batch of the default
//    plan is not needed here, so 300 -- and f16 at 4), plan under every fusion setting tests use, run
//    once on zeros, and are destroyed;
// 2. ITERATIONS random byte mutations of MNIST-8 are LOADED (parse + shape rules + planner + weight
//    packing) and destroyed; each must load or fail with a status, never fault.  Mutated models are
//    not run.
// Any sanitizer report aborts (-fno-sanitize-recover=all), so exit 0 means clean.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <vector>

#include <hip/hip_runtime.h>

#include "ore.h"

static std::vector<char> slurp(const char* path) {
  std::ifstream f(path, std::ios::binary);
  return std::vector<char>(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
}

static int run_model(ore_ctx* ctx, const std::vector<char>& bytes, int64_t batch, int32_t flags) {
  ore_model* m = nullptr;
  if (ore_model_load_ex(ctx, bytes.data(), bytes.size(), batch, flags, &m)) {
    std::fprintf(stderr, "load failed: %s\n", ore_last_error(ctx));
    return 1;
  }
  int64_t dims[4], out_elems = 0;
  ore_model_input_dims(m, dims);
  ore_model_output_elems(m, &out_elems);
  const size_t in_bytes = size_t(batch * dims[1] * dims[2] * dims[3]) * 4, out_bytes = size_t(batch * out_elems) * 4;
  void *x = nullptr, *y = nullptr;
  if (ore_malloc(ctx, in_bytes, &x) || ore_malloc(ctx, out_bytes, &y)) return 1;
  (void)hipMemset(x, 0, in_bytes);
  const int32_t fusions[] = {ORE_FUSE_ALL, 0, 7, ORE_FUSE_ALL | ORE_FUSE_EAGER, ORE_FUSE_ALL | ORE_KEEP_VALUES};
  for (int32_t f : fusions) {
    if (ore_model_set_fusion(m, f) || ore_model_run(m, static_cast<float*>(x), batch, static_cast<float*>(y)) ||
        ore_sync(ctx)) {
      std::fprintf(stderr, "fusion %d: %s\n", f, ore_last_error(ctx));
      return 1;
    }
  }
  ore_model_destroy(m);
  ore_free(ctx, x);
  ore_free(ctx, y);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s MNIST.onnx SQUEEZENET.onnx ITERATIONS\n", argv[0]);
    return 2;
  }
  const std::vector<char> mnist = slurp(argv[1]), sq = slurp(argv[2]);
  ore_ctx* ctx = nullptr;
  if (ore_ctx_create(0, &ctx)) {
    std::fprintf(stderr, "ctx: %s\n", ore_last_error(nullptr));
    return 1;
  }
  int bad = 0;
  bad |= run_model(ctx, mnist, 1, 0);
  bad |= run_model(ctx, mnist, 4, 0);
  bad |= run_model(ctx, sq, 1, 0);
  bad |= run_model(ctx, sq, 4, 0);
  bad |= run_model(ctx, sq, 300, 0);
  bad |= run_model(ctx, sq, 4, ORE_LOAD_NO_WINOGRAD);
  bad |= run_model(ctx, sq, 4, ORE_LOAD_F16);
  if (bad) return 1;
  const long iters = std::atol(argv[3]);
  uint64_t s = 4321;
  auto rnd = [&]() {  // xorshift64*
    s ^= s >> 12; s ^= s << 25; s ^= s >> 27;
    return (s * 0x2545F4914F6CDD1DULL) >> 11;
  };
  long loaded = 0, refused = 0;
  for (long it = 0; it < iters; ++it) {
    std::vector<char> b = mnist;
    const int nmut = 1 + int(rnd() % 4);
    for (int k = 0; k < nmut; ++k) {
      const size_t i = (rnd() % 10 < 8) ? rnd() % std::min<size_t>(b.size(), 4096) : rnd() % b.size();
      b[i] = char(rnd());
    }
    if (rnd() % 5 == 0) b.resize(rnd() % b.size());
    ore_model* m = nullptr;
    if (ore_model_load_ex(ctx, b.data(), b.size(), 1 + int64_t(rnd() % 8), 0, &m) == ORE_OK) {
      ++loaded;
      ore_model_destroy(m);
    } else {
      ++refused;
    }
  }
  if (ore_sync(ctx)) return 1;
  ore_ctx_destroy(ctx);
  std::printf("model_fuzz: 7 model plans run clean; %ld mutated models loaded, %ld refused; no sanitizer report\n",
              loaded, refused);
  return 0;
}
