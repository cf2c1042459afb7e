// Reader for the LevelDB-format SSTable that TensorFlow uses as the TensorBundle
// index (`variables/variables.index` of a SavedModel): footer
// with magic 0xdb4775248b80fb57, index block of BlockHandles, prefix-compressed
// data blocks with restart arrays, 5-byte block trailers (compression type +
// masked CRC32C). Snappy-compressed blocks are decoded by a built-in decoder.
#pragma once
#include <stdint.h>

#include <string>
#include <utility>
#include <vector>

namespace kdl {

uint32_t crc32c(const uint8_t* data, size_t n, uint32_t init = 0);
inline uint32_t crc32c_unmask(uint32_t masked) {
  const uint32_t rot = masked - 0xa282ead8u;
  return (rot >> 17) | (rot << 15);
}
std::string snappy_uncompress(const uint8_t* data, size_t n);

// All (key, value) entries of the table in key order. Throws on corruption.
std::vector<std::pair<std::string, std::string>> read_sstable(const std::string& bytes, bool verify_crc = true);

}  // namespace kdl
