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

// unpacked = true: the 12 values as unpacked float_val (field 5, wire type I32, one tag
// per value) instead of tensor_content
static std::string valid_request(bool unpacked = false) {
  std::string spec, tensor, shape, dim, entry, req;
  field(spec, 1, "clothing-model");
  field(spec, 3, "serving_default");
  varint(tensor, (1 << 3) | 0); varint(tensor, 1);            // dtype DT_FLOAT
  for (int d : {1, 2, 2, 3}) { std::string x; varint(x, (1 << 3) | 0); varint(x, d); field(shape, 2, x); }
  field(tensor, 2, shape);
  if (unpacked) {
    for (int i = 0; i < 12; ++i) { varint(tensor, (5 << 3) | 5); tensor += std::string("\x00\x00\x80\x3f", 4); }
  } else {
    field(tensor, 4, std::string(48, '\x01'));                // tensor_content
  }
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

// Every parse runs on an exact-size heap copy, so ASan sees a read one byte past the
// input (a std::string's inline/capacity slack would hide it).
static void fuzz_one(const std::string& s) {
  std::vector<uint8_t> buf(s.begin(), s.end());
  if (buf.empty()) buf.reserve(1);
  const uint8_t* p = buf.data();
  expect_no_crash([&] { parse_predict_request(p, buf.size()); });
  expect_no_crash([&] { parse_model_spec_request(p, buf.size()); });
  expect_no_crash([&] { snappy_uncompress(p, buf.size()); });
  expect_no_crash([&] { read_sstable(s, true); });
  expect_no_crash([&] { read_sstable(s, false); });
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  std::mt19937 rng(7);
  const std::string seeds[2] = {valid_request(false), valid_request(true)};
  for (const auto& good : seeds) {
    auto v = parse_predict_request((const uint8_t*)good.data(), good.size());
    if (v.inputs.size() != 1) { printf("valid request not parsed\n"); return 1; }
  }
  // regression: an inputs entry whose tensor ends in a float_val tag with no 4-byte
  // payload behind it (12 03 12 01 2d) must throw, not read past the buffer
  fuzz_one(std::string("\x12\x03\x12\x01\x2d", 5));
  // regression: an SSTable footer whose index handle wraps offset + size + 5 around
  // 2^64 (offset = 2^64 - 6, size = 1) must be rejected, not read before the buffer
  {
    std::string footer;
    varint(footer, 0); varint(footer, 0);                     // metaindex handle
    varint(footer, ~0ull - 5); varint(footer, 1);             // index handle
    footer.resize(40, '\0');
    const uint64_t magic = 0xdb4775248b80fb57ull;
    footer.append(reinterpret_cast<const char*>(&magic), 8);
    bool threw = false;
    try { read_sstable(footer, false); } catch (const std::exception&) { threw = true; }
    if (!threw) { printf("wrapping sstable handle accepted\n"); return 1; }
    fuzz_one(footer);
  }
  for (int it = 0; it < iters; ++it) {
    const std::string& good = seeds[(it >> 2) & 1];
    std::string s;
    switch (it % 4) {
      case 0: s = good.substr(0, rng() % (good.size() + 1)); break;       // truncation
      case 1: s = good; for (int k = 0; k < 3; ++k) s[rng() % s.size()] ^= (char)(1 << (rng() % 8)); break;
      case 2: s.resize(rng() % 256); for (auto& c : s) c = (char)rng(); break;
      default: s = good; s.insert(rng() % s.size(), std::string(1 + rng() % 8, (char)0xff)); break;
    }
    fuzz_one(s);
  }
  printf("fuzzed %d inputs\n", iters);
  return 0;
}
