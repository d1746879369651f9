// Host-only ASan / UBSan driver for the ONNX wire-format parser (csrc/ore_onnx.cpp, which replaces the
// reference's ModelProto::parse_from_bytes, main.rs:30, and the initializer decode of get_stored_tensor,
// utils.rs:113-185).  Built by tools/asan/build.sh with -fsanitize=address,undefined on the host side.
//   parse_fuzz MODEL.onnx ITERATIONS [CASE_FILE ...]
// Parses MODEL (must succeed), each CASE_FILE (tests/test_abi.py's wire-type mismatch cases: must be
// rejected), then ITERATIONS random byte mutations / truncations of MODEL (the scheme of
// test_abi.py::test_parse_fuzz_mutated_mnist): each must parse or be rejected, never fault.  Any
// sanitizer report aborts the process (halt_on_error), so exit 0 means clean.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "ore_internal.h"

static std::vector<uint8_t> slurp(const char* path) {
  std::ifstream f(path, std::ios::binary);
  return std::vector<uint8_t>(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
}

static bool parse(const std::vector<uint8_t>& b) {
  ore::Graph g;
  std::string err;
  // a heap copy of exactly the payload, so ASan sees every read past its end
  uint8_t* p = static_cast<uint8_t*>(std::malloc(b.size() ? b.size() : 1));
  if (!b.empty()) std::memcpy(p, b.data(), b.size());
  const bool ok = ore::parse_model(p, b.size(), &g, &err);
  std::free(p);
  return ok;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s MODEL.onnx ITERATIONS [CASE_FILE ...]\n", argv[0]);
    return 2;
  }
  const std::vector<uint8_t> model = slurp(argv[1]);
  if (model.empty() || !parse(model)) {
    std::fprintf(stderr, "the unmutated model does not parse\n");
    return 1;
  }
  int rejected_cases = 0;
  for (int i = 3; i < argc; ++i) {
    if (parse(slurp(argv[i]))) {
      std::fprintf(stderr, "case %s parsed but should be rejected\n", argv[i]);
      return 1;
    }
    ++rejected_cases;
  }
  const long iters = std::atol(argv[2]);
  uint64_t s = 1234;
  auto rnd = [&]() {  // xorshift64*
    s ^= s >> 12; s ^= s << 25; s ^= s >> 27;
    return (s * 0x2545F4914F6CDD1DULL) >> 11;
  };
  long ok = 0, bad = 0;
  for (long it = 0; it < iters; ++it) {
    std::vector<uint8_t> b = model;
    const int nmut = 1 + int(rnd() % 4);
    for (int k = 0; k < nmut; ++k) {
      const size_t i = (rnd() % 10 < 8) ? rnd() % std::min<size_t>(b.size(), 4096) : rnd() % b.size();
      b[i] = uint8_t(rnd());
    }
    if (rnd() % 5 == 0) b.resize(rnd() % b.size());
    (parse(b) ? ok : bad)++;
  }
  std::printf("parse_fuzz: %d rejected cases, %ld mutations parsed, %ld rejected, no sanitizer report\n",
              rejected_cases, ok, bad);
  return 0;
}
