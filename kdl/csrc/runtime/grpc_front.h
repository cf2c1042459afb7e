// Native gRPC front-end of the model server (the reference's
// TF-Serving is C++ gRPC end to end: /root/reference/tf-serving-clothing-model-deployment.yaml:20-27,
// clients at /root/reference/model_server.py:15-16,38-55).
//
// The grpcio server spends ~0.4-0.8 ms of Python/Cython CPU per 1-image request
// (profiles/serve_native_front_r5.txt): one process cannot feed even one MI355X at the
// reference's request shape (one image per Predict). Here:
//   * io_threads epoll workers, each with its own SO_REUSEPORT listener (the kernel spreads
//     connections; --procs processes share the port the same way), HTTP/2 by libnghttp2 (h2.h)
//     with 1 MiB frames and 8 MiB stream windows (a 1 MB f32 image needs no WINDOW_UPDATE
//     round trip);
//   * Predict FAST PATH, no Python and no GIL: the request message is walked in place by the
//     tfproto codec, the image view goes to the signature's DynamicBatcher::submit_async, the
//     executor thread that finishes the batch builds the PredictResponse and hands it back to
//     the connection's worker through an eventfd mailbox;
//   * everything else -- other methods, other versions / labels, any request the fast path
//     would reject (so every error message stays the Python servicer's TF-Serving text) --
//     goes to the SLOW PATH: a small pool of threads that call the Python servicer with the GIL.
// Routes are registered by the Python side (serving/native_front.py) per (model, signature)
// and dropped on every version change; a route whose batcher has shut down falls back to the
// slow path, which answers (or re-learns the new version's route).
#pragma once
#include <stdint.h>

#include <functional>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "batcher.h"

namespace kdl {

struct FrontRoute {
  std::string model, signature;        // model_spec.name, resolved signature name
  int64_t version = 0;                 // the served version (requests naming another go slow)
  std::string input_key, output_key;
  int dtype = 0;                       // TF DataType of the input: 1 DT_FLOAT, 4 DT_UINT8
  int image = 0;                       // fixed input H = W
  int out_cols = 0;
  std::shared_ptr<DynamicBatcher> batcher;
  std::shared_ptr<DynamicBatcher> u8;  // DT_FLOAT route: exact 8-bit payloads ride this one
};

struct SlowReply {
  int code = 0;                        // grpc status code
  std::string message, body;           // body: the response message (code 0)
  std::vector<std::pair<std::string, std::string>> meta;   // extra initial metadata
};
// (method path, request message, deadline in now_us() time or 0) -> reply; slow-pool threads
using SlowFn = std::function<SlowReply(const std::string& path, const std::string& msg, int64_t deadline_us)>;

constexpr int kFrontLatBuckets = 19;   // serving/metrics.py LAT_BUCKETS_MS
struct FrontStats {
  int64_t fast_ok = 0, fast_err = 0, slow = 0, exact_u8 = 0, connections = 0, open_connections = 0;
  int64_t by_code[17] = {};            // fast-path answers per grpc status
  int64_t lat[kFrontLatBuckets + 1] = {};   // fast-path latency histogram (ms), +Inf last
  double lat_sum_ms = 0;
  static constexpr int kMaxWorkers = 64;
  int64_t worker_calls[kMaxWorkers] = {};   // requests received per I/O worker (SO_REUSEPORT spread)
};

class GrpcFront {
 public:
  // binds host:port (0: any free port) once per io thread; throws on failure.
  // max_recv_bytes: largest request message (grpcio's max_receive_message_length; larger ones
  // get RESOURCE_EXHAUSTED before their bytes are buffered); the bodies held at once are capped
  // at max(16 x that, 256 MiB). reuse_port: the port may be shared with other processes
  // (--procs); false makes the bind fail when another server holds it.
  GrpcFront(const std::string& host, int port, int io_threads, int slow_threads, SlowFn slow,
            size_t max_recv_bytes = size_t(64) << 20, bool reuse_port = true);
  ~GrpcFront();
  GrpcFront(const GrpcFront&) = delete;
  GrpcFront& operator=(const GrpcFront&) = delete;

  int port() const;
  void set_route(FrontRoute r);
  void clear_routes();
  // close listeners and connections, join every thread; answers nothing more (in-flight
  // batcher callbacks arriving later are dropped). Idempotent.
  void stop();
  FrontStats stats() const;

  struct Impl;                         // opaque (grpc_front.cpp)

 private:
  std::unique_ptr<Impl> p_;
};

// f32 payload -> uint8 pixels when it is EXACTLY float32(u) / 127.5 - 1 for 8-bit u (the
// reference gateway's keras Xception preprocessing, model_server.py:18): false at the first
// block holding a value that is not (dst then undefined)
bool f32_to_u8_exact(const float* __restrict x, uint8_t* __restrict u, size_t n);

// percent-encoding of a grpc-message value (gRPC HTTP/2 protocol: bytes outside 0x20-0x7e and '%')
std::string grpc_percent_encode(const std::string& s);

}  // namespace kdl
