// Malformed-input fuzz of the native wire/file parsers under ASan+UBSan
// (tests/test_sanitizers.py): PredictRequest / ModelSpec protobuf views, the
// snappy decoder and the LevelDB-SSTable reader must either parse or throw, never
// read out of bounds. Inputs: random bytes, truncations and bit flips of a valid
// PredictRequest (built here by hand, field numbers of tensorflow.serving).
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "../runtime/sstable.h"
#include "../runtime/tfproto.h"

using namespace kdl;

static void varint(std::string& s, uint64_t v) {
  while (v >= 0x80) { s.push_back((char)(v | 0x80)); v >>= 7; }
  s.push_back((char)v);
}
static void field(std::string& s, int num, const std::string& payload) {
  varint(s, ((uint64_t)num << 3) | 2);
  varint(s, payload.size());
  s += payload;
}

static std::string valid_request() {
  std::string spec, tensor, shape, dim, entry, req;
  field(spec, 1, "clothing-model");
  field(spec, 3, "serving_default");
  varint(tensor, (1 << 3) | 0); varint(tensor, 1);            // dtype DT_FLOAT
  for (int d : {1, 2, 2, 3}) { std::string x; varint(x, (1 << 3) | 0); varint(x, d); field(shape, 2, x); }
  field(tensor, 2, shape);
  field(tensor, 4, std::string(48, '\x01'));                  // tensor_content
  field(entry, 1, "input_8");
  field(entry, 2, tensor);
  field(req, 1, spec);
  field(req, 2, entry);
  return req;
}

template <class F>
static void expect_no_crash(F f) {
  try { f(); } catch (const std::exception&) {}
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  std::mt19937 rng(7);
  const std::string good = valid_request();
  {
    auto v = parse_predict_request((const uint8_t*)good.data(), good.size());
    if (v.inputs.size() != 1) { printf("valid request not parsed\n"); return 1; }
  }
  for (int it = 0; it < iters; ++it) {
    std::string s;
    switch (it % 4) {
      case 0: s = good.substr(0, rng() % (good.size() + 1)); break;       // truncation
      case 1: s = good; for (int k = 0; k < 3; ++k) s[rng() % s.size()] ^= (char)(1 << (rng() % 8)); break;
      case 2: s.resize(rng() % 256); for (auto& c : s) c = (char)rng(); break;
      default: s = good; s.insert(rng() % s.size(), std::string(1 + rng() % 8, (char)0xff)); break;
    }
    const uint8_t* p = (const uint8_t*)s.data();
    expect_no_crash([&] { parse_predict_request(p, s.size()); });
    expect_no_crash([&] { parse_model_spec_request(p, s.size()); });
    expect_no_crash([&] { snappy_uncompress(p, s.size()); });
    expect_no_crash([&] { read_sstable(s, true); });
    expect_no_crash([&] { read_sstable(s, false); });
  }
  printf("fuzzed %d inputs\n", iters);
  return 0;
}
