#include "sstable.h"

#include <cstring>
#include <stdexcept>

namespace kdl {
namespace {

struct Tables {
  uint32_t t[256];
  Tables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82f63b78u : (c >> 1);
      t[i] = c;
    }
  }
};
const Tables& tables() {
  static Tables tb;
  return tb;
}

uint64_t get_varint(const uint8_t*& p, const uint8_t* end) {
  uint64_t v = 0;
  for (int s = 0; s < 64; s += 7) {
    if (p >= end) throw std::runtime_error("sstable: truncated varint");
    const uint8_t b = *p++;
    v |= uint64_t(b & 0x7f) << s;
    if (!(b & 0x80)) return v;
  }
  throw std::runtime_error("sstable: bad varint");
}

uint32_t le32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
uint64_t le64(const uint8_t* p) { uint64_t v; std::memcpy(&v, p, 8); return v; }

struct Handle { uint64_t offset, size; };
Handle get_handle(const uint8_t*& p, const uint8_t* end) {
  Handle h;
  h.offset = get_varint(p, end);
  h.size = get_varint(p, end);
  return h;
}

// Block contents (decompressed) for a handle, checking the 5-byte trailer.
std::string read_block(const std::string& file, Handle h, bool verify) {
  // overflow-safe form of offset + size + 5 <= file.size() (the handle is untrusted)
  const uint64_t fs = file.size();
  if (h.size > fs || h.offset > fs - h.size || fs - h.offset - h.size < 5)
    throw std::runtime_error("sstable: block out of range");
  const uint8_t* b = reinterpret_cast<const uint8_t*>(file.data()) + h.offset;
  const uint8_t type = b[h.size];
  if (verify) {
    const uint32_t expect = crc32c_unmask(le32(b + h.size + 1));
    const uint32_t got = crc32c(b, h.size + 1);   // covers data + type byte
    if (expect != got) throw std::runtime_error("sstable: block checksum mismatch");
  }
  if (type == 0) return std::string(reinterpret_cast<const char*>(b), h.size);
  if (type == 1) return snappy_uncompress(b, h.size);
  throw std::runtime_error("sstable: unknown block compression " + std::to_string(type));
}

void parse_block(const std::string& blk, std::vector<std::pair<std::string, std::string>>* out) {
  if (blk.size() < 4) throw std::runtime_error("sstable: short block");
  const uint8_t* base = reinterpret_cast<const uint8_t*>(blk.data());
  const uint32_t nrestarts = le32(base + blk.size() - 4);
  const size_t limit = blk.size() - 4 - size_t(nrestarts) * 4;
  if (limit > blk.size()) throw std::runtime_error("sstable: bad restart count");
  const uint8_t* p = base;
  const uint8_t* end = base + limit;
  std::string key;
  while (p < end) {
    const uint64_t shared = get_varint(p, end);
    const uint64_t nonshared = get_varint(p, end);
    const uint64_t vlen = get_varint(p, end);
    const uint64_t avail = uint64_t(end - p);
    if (shared > key.size() || nonshared > avail || vlen > avail - nonshared)
      throw std::runtime_error("sstable: bad entry");
    key.resize(shared);
    key.append(reinterpret_cast<const char*>(p), nonshared);
    p += nonshared;
    out->emplace_back(key, std::string(reinterpret_cast<const char*>(p), vlen));
    p += vlen;
  }
}

}  // namespace

uint32_t crc32c(const uint8_t* data, size_t n, uint32_t init) {
  const auto& t = tables().t;
  uint32_t c = ~init;
  for (size_t i = 0; i < n; ++i) c = t[(c ^ data[i]) & 0xff] ^ (c >> 8);
  return ~c;
}

std::string snappy_uncompress(const uint8_t* data, size_t n) {
  const uint8_t* p = data;
  const uint8_t* end = data + n;
  const uint64_t len = get_varint(p, end);
  // untrusted header: a snappy element expands at most 64x (a 3-byte copy of 64
  // bytes), so a larger claim is corrupt -- and must not reach reserve()
  if (len > uint64_t(n) * 64 + 64) throw std::runtime_error("snappy: implausible uncompressed length");
  std::string out;
  out.reserve(len);
  while (p < end) {
    const uint8_t tag = *p++;
    const int kind = tag & 3;
    if (kind == 0) {                                   // literal
      uint64_t l = tag >> 2;
      if (l >= 60) {
        const int nb = int(l - 59);
        if (end - p < nb) throw std::runtime_error("snappy: truncated literal length");
        l = 0;
        for (int i = 0; i < nb; ++i) l |= uint64_t(p[i]) << (8 * i);
        p += nb;
      }
      l += 1;
      if (uint64_t(end - p) < l) throw std::runtime_error("snappy: truncated literal");
      if (out.size() + l > len) throw std::runtime_error("snappy: output overrun");
      out.append(reinterpret_cast<const char*>(p), l);
      p += l;
    } else {
      uint64_t l, off;
      if (kind == 1) {
        if (end - p < 1) throw std::runtime_error("snappy: truncated copy1");
        l = ((tag >> 2) & 7) + 4;
        off = (uint64_t(tag >> 5) << 8) | *p++;
      } else if (kind == 2) {
        if (end - p < 2) throw std::runtime_error("snappy: truncated copy2");
        l = (tag >> 2) + 1;
        off = uint64_t(p[0]) | (uint64_t(p[1]) << 8);
        p += 2;
      } else {
        if (end - p < 4) throw std::runtime_error("snappy: truncated copy4");
        l = (tag >> 2) + 1;
        off = le32(p);
        p += 4;
      }
      if (off == 0 || off > out.size()) throw std::runtime_error("snappy: bad offset");
      if (out.size() + l > len) throw std::runtime_error("snappy: output overrun");
      const size_t from = out.size() - off;
      for (uint64_t i = 0; i < l; ++i) out.push_back(out[from + i]);  // may overlap
    }
  }
  if (out.size() != len) throw std::runtime_error("snappy: length mismatch");
  return out;
}

std::vector<std::pair<std::string, std::string>> read_sstable(const std::string& file, bool verify) {
  constexpr uint64_t kMagic = 0xdb4775248b80fb57ull;
  constexpr size_t kFooter = 48;
  if (file.size() < kFooter) throw std::runtime_error("sstable: file too small");
  const uint8_t* f = reinterpret_cast<const uint8_t*>(file.data()) + file.size() - kFooter;
  if (le64(f + 40) != kMagic) throw std::runtime_error("sstable: bad magic (not a TensorBundle index?)");
  const uint8_t* p = f;
  (void)get_handle(p, f + 40);                     // metaindex (unused by TensorBundle)
  const Handle index = get_handle(p, f + 40);
  std::vector<std::pair<std::string, std::string>> idx, out;
  parse_block(read_block(file, index, verify), &idx);
  for (const auto& kv : idx) {
    const uint8_t* q = reinterpret_cast<const uint8_t*>(kv.second.data());
    const Handle h = get_handle(q, q + kv.second.size());
    parse_block(read_block(file, h, verify), &out);
  }
  return out;
}

}  // namespace kdl
