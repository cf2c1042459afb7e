// Native closed-loop gRPC load generator (tools/serve_bench.py --client native): `conns`
// HTTP/2 connections, one thread each, every connection keeps `streams` unary calls of the
// same request in flight. Python clients top out near 1-2k req/s per process on a 1-image
// Predict (profiles/serve_native_front_r5.txt), below what a front-end must be measured at.
#pragma once
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

namespace kdl {

struct LoadResult {
  int64_t ok = 0, failed = 0;            // calls completed after the warm-up
  double seconds = 0;                    // measured span (after the warm-up)
  std::vector<double> lat_ms;            // per OK call, after the warm-up
  std::map<int, int64_t> codes;          // grpc-status -> count (after the warm-up; -1: no status)
  std::string error;                     // first connection-level failure, if any
};

// raw_frame: `message` already carries its 5-byte gRPC prefix (sent as is, to test a server's
// handling of prefixes that do not match the bytes that follow)
LoadResult grpc_load(const std::string& host, int port, const std::string& path, const std::string& message,
                     int conns, int streams, double seconds, double warm_s, double timeout_s = 30,
                     bool raw_frame = false);

}  // namespace kdl
