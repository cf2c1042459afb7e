// Native gRPC front-end (runtime/grpc_front.h) under TSAN / ASan+UBSan, no Python: a GrpcFront
// (epoll workers, slow pool, eventfd mailbox) in front of a DynamicBatcher drained by a fake
// executor thread, hammered by the native load generator (runtime/grpc_load.h) on the fast path
// and on the slow path at once, while another thread keeps replacing and clearing the route;
// then the batcher is shut down and the front stopped with calls in flight.
//   front_stress [conns=4] [streams=4] [seconds=2]
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "runtime/batcher.h"
#include "runtime/grpc_front.h"
#include "runtime/grpc_load.h"
#include "runtime/h2.h"

using namespace kdl;

namespace {

void varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back(char(v | 0x80));
    v >>= 7;
  }
  o.push_back(char(v));
}
void field(std::string& o, int num, const std::string& bytes) {   // length-delimited
  varint(o, uint64_t(num) << 3 | 2);
  varint(o, bytes.size());
  o += bytes;
}

// PredictRequest{model_spec{name}, inputs{key: TensorProto{DT_UINT8, [1, S, S, 3], content}}}
std::string predict_request(const std::string& model, const std::string& key, int S, uint8_t fill) {
  std::string spec, shape, tensor, entry, req;
  field(spec, 1, model);
  for (int d : {1, S, S, 3}) {
    std::string dim;
    varint(dim, 1 << 3);
    varint(dim, uint64_t(d));
    field(shape, 2, dim);
  }
  varint(tensor, 1 << 3);
  varint(tensor, 4);                    // DT_UINT8
  field(tensor, 2, shape);
  field(tensor, 4, std::string(size_t(S) * S * 3, char(fill)));
  field(entry, 1, key);
  field(entry, 2, tensor);
  field(req, 1, spec);
  field(req, 2, entry);
  return req;
}

long rss_kib() {
  FILE* f = std::fopen("/proc/self/statm", "r");
  long pages = 0, res = 0;
  if (f) {
    if (std::fscanf(f, "%ld %ld", &pages, &res) != 2) res = 0;
    std::fclose(f);
  }
  return res * 4;
}

// Requests that claim or carry more than the cap (advisor r5 / VERDICT r5 item 8): 1,024 streams
// on each connection announcing 2 GiB - 1 behind a 4 KiB body, plus streams whose honest prefix
// and bytes exceed a 1 MiB cap. Every stream must get RESOURCE_EXHAUSTED, none may reach the
// slow path, and the process must not grow by the announced sizes.
bool oversize_phase(int conns) {
  std::atomic<int> slow_calls{0};
  GrpcFront front("127.0.0.1", 0, 2, 2, [&](const std::string&, const std::string&, int64_t) {
    slow_calls.fetch_add(1);
    return SlowReply{};
  }, size_t(1) << 20, false);
  const long rss0 = rss_kib();
  const std::string path = "/tensorflow.serving.PredictionService/Predict";
  std::string liar(5, '\0');            // prefix: 0x7fffffff bytes follow; only 4 KiB do
  liar[1] = char(0x7f), liar[2] = char(0xff), liar[3] = char(0xff), liar[4] = char(0xff);
  liar += std::string(size_t(4) << 10, 'x');
  const std::string big(size_t(3) << 20, 'y');   // honest prefix, 3 MiB > 1 MiB
  LoadResult a, b;
  std::thread ta([&] { a = grpc_load("127.0.0.1", front.port(), path, liar, conns, 1024, 1.0, 0.0, 10.0, true); });
  std::thread tb([&] { b = grpc_load("127.0.0.1", front.port(), path, big, 2, 16, 1.0, 0.0, 10.0); });
  ta.join();
  tb.join();
  const long grow = rss_kib() - rss0;
  front.stop();
  bool ok = a.error.empty() && b.error.empty() && slow_calls.load() == 0;
  for (const LoadResult* r : {&a, &b})
    for (const auto& kv : r->codes)
      if (kv.first != 8) {
        std::printf("oversize: unexpected grpc-status %d x%lld\n", kv.first, (long long)kv.second);
        ok = false;
      }
  const int64_t n = a.failed + b.failed;
  if (a.failed < 100 || b.failed < 4) ok = false;
  if (grow > (long(512) << 10)) ok = false;   // 1,024 x 2 GiB announced per connection; < 512 MiB grown
  std::printf("oversize: %lld + %lld streams RESOURCE_EXHAUSTED (%lld total), errors '%s' '%s', slow calls %d, "
              "rss +%ld KiB: %s\n", (long long)a.failed, (long long)b.failed, (long long)n, a.error.c_str(),
              b.error.c_str(), slow_calls.load(), grow, ok ? "OK" : "FAIL");
  return ok;
}

}  // namespace

int main(int argc, char** argv) {
  const int conns = argc > 1 ? std::atoi(argv[1]) : 4;
  const int streams = argc > 2 ? std::atoi(argv[2]) : 4;
  const double secs = argc > 3 ? std::atof(argv[3]) : 2.0;
  std::string why;
  if (!h2::api(&why)) {
    std::printf("SKIP %s\n", why.c_str());
    return 0;
  }
  constexpr int S = 16, COLS = 10;
  BatcherOptions o;
  o.max_batch_size = 8;
  o.batch_timeout_us = 200;
  o.allowed_batch_sizes = {1, 2, 4, 8};
  o.item_bytes = size_t(S) * S * 3;
  o.out_cols = COLS;
  o.copy_threads = 2;
  auto batcher = std::make_shared<DynamicBatcher>(o);
  std::atomic<bool> stop_exec{false};
  std::thread exec([&] {                // fake device: row = first byte + class index
    std::vector<uint8_t> staging(o.item_bytes * 8);
    std::vector<float> out(size_t(COLS) * 8);
    Batch b;
    while (!stop_exec.load()) {
      if (!batcher->next_batch(staging.data(), 2000, &b, true)) continue;
      for (int i = 0; i < b.n_real; ++i)
        for (int k = 0; k < COLS; ++k) out[size_t(i) * COLS + k] = float(staging[size_t(i) * o.item_bytes] + k);
      batcher->finish(b, out.data(), ST_OK);
    }
  });
  std::atomic<int> slow_calls{0};
  GrpcFront front("127.0.0.1", 0, 2, 2, [&](const std::string& path, const std::string&, int64_t) {
    slow_calls.fetch_add(1);
    SlowReply r;
    r.code = 5;
    r.message = "slow path: " + path;
    return r;
  });
  FrontRoute route;
  route.model = "m";
  route.signature = "serving_default";
  route.version = 1;
  route.input_key = "x";
  route.output_key = "y";
  route.dtype = 4;
  route.image = S;
  route.out_cols = COLS;
  route.batcher = batcher;
  std::atomic<bool> stop_flip{false};
  std::thread flip([&] {
    while (!stop_flip.load()) {
      front.set_route(route);
      std::this_thread::sleep_for(std::chrono::milliseconds(3));
      front.clear_routes();
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    front.set_route(route);
  });
  const std::string req = predict_request("m", "x", S, 7);
  const std::string path = "/tensorflow.serving.PredictionService/Predict";
  LoadResult fast, slow;
  std::thread tf([&] { fast = grpc_load("127.0.0.1", front.port(), path, req, conns, streams, secs, 0.1); });
  std::thread ts([&] { slow = grpc_load("127.0.0.1", front.port(), "/no.such/Method", "", 1, 2, secs, 0.1); });
  tf.join();
  ts.join();
  stop_flip.store(true);
  flip.join();
  int bad = 0;
  for (const LoadResult* r : {&fast, &slow}) {
    if (!r->error.empty()) {
      std::printf("load error: %s\n", r->error.c_str());
      ++bad;
    }
    for (const auto& kv : r->codes)
      if (kv.first != 0 && kv.first != 5) {
        std::printf("unexpected grpc-status %d x%lld\n", kv.first, (long long)kv.second);
        ++bad;
      }
  }
  const FrontStats st = front.stats();
  if (fast.ok < 50 || st.fast_ok < 50 || slow.codes.count(5) == 0 || slow_calls.load() == 0) {
    std::printf("too little traffic: fast ok %lld, front fast_ok %lld, slow calls %d\n", (long long)fast.ok,
                (long long)st.fast_ok, slow_calls.load());
    ++bad;
  }
  // teardown with calls in flight: the batcher shuts down under load, then the front stops
  LoadResult tail;
  std::thread tt([&] { tail = grpc_load("127.0.0.1", front.port(), path, req, conns, streams, 1.0, 0.0, 3.0); });
  std::this_thread::sleep_for(std::chrono::milliseconds(300));
  batcher->shutdown();
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  front.stop();
  tt.join();
  stop_exec.store(true);
  exec.join();
  std::printf("fast ok %lld (front %lld), slow answers %d, open connections at stop %lld: %s\n",
              (long long)fast.ok, (long long)st.fast_ok, slow_calls.load(), (long long)st.open_connections,
              bad ? "FAIL" : "OK");
  bad += oversize_phase(conns) ? 0 : 1;
  return bad ? 1 : 0;
}
