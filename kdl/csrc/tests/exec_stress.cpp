// Stress test of the native batch executor (executor.cpp) with fake device backends,
// run under ThreadSanitizer and AddressSanitizer+UBSan by tests/test_sanitizers.py:
// three executors (one failing every batch, so it is isolated after max_failures)
// share one batcher fed by many producer threads; each completed request must get back
// exactly its own rows, every request must end (no waiter left blocked), and stop()
// must drain the batches in flight.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <memory>
#include <random>
#include <thread>
#include <vector>

#include "../runtime/executor.h"

using namespace kdl;

int main(int argc, char** argv) {
  const int producers = argc > 1 ? atoi(argv[1]) : 8;
  const int per_producer = argc > 2 ? atoi(argv[2]) : 200;
  BatcherOptions o;
  o.max_batch_size = 8;
  o.batch_timeout_us = 300;
  o.max_enqueued_batches = 64;
  o.allowed_batch_sizes = {1, 2, 4, 8};
  o.item_bytes = 48;
  o.out_cols = 3;
  DynamicBatcher b(o);
  ExecGroup g;
  std::vector<std::unique_ptr<FakeBackend>> fakes;
  fakes.emplace_back(new FakeBackend(2, o.item_bytes, o.max_batch_size, o.out_cols, 200));
  fakes.emplace_back(new FakeBackend(3, o.item_bytes, o.max_batch_size, o.out_cols, 50));
  fakes.emplace_back(new FakeBackend(2, o.item_bytes, o.max_batch_size, o.out_cols, 100, 1));
  std::vector<std::unique_ptr<Executor>> exs;
  for (size_t i = 0; i < fakes.size(); ++i) {
    ExecOptions eo;
    eo.name = "fake" + std::to_string(i);
    eo.max_failures = 2;
    eo.poll_us = 2000;
    exs.emplace_back(new Executor(&b, &fakes[i]->api, &g, eo));
    exs.back()->start();
  }
  std::atomic<int> ok{0}, failed{0}, bad{0};
  std::vector<std::thread> prods;
  for (int p = 0; p < producers; ++p) {
    prods.emplace_back([&, p] {
      std::mt19937 rng(p);
      for (int r = 0; r < per_producer; ++r) {
        const int n = 1 + rng() % 4;
        std::vector<uint8_t> data(n * o.item_bytes);
        for (int i = 0; i < n; ++i) memset(&data[i * o.item_bytes], (p * 13 + r * 5 + i) & 0x7f, o.item_bytes);
        const int64_t t = b.submit(data.data(), n, rng() % 10 == 0 ? now_us() + rng() % 400 : 0);
        if (t < 0) { failed++; continue; }
        std::vector<float> out(n * o.out_cols);
        if (b.wait(t, out.data(), out.size()) != ST_OK) { failed++; continue; }
        for (int i = 0; i < n; ++i)
          for (int k = 0; k < o.out_cols; ++k)
            if (out[i * o.out_cols + k] != (float)((p * 13 + r * 5 + i) & 0x7f) + k) bad++;
        ok++;
      }
    });
  }
  for (auto& t : prods) t.join();
  for (auto& e : exs) e->stop();
  b.shutdown();
  int64_t batches = 0;
  for (auto& e : exs) batches += e->stats().batches;
  printf("ok=%d failed=%d bad=%d batches=%lld healthy=%d\n", ok.load(), failed.load(), bad.load(),
         (long long)batches, g.healthy());
  if (bad.load() != 0 || ok.load() == 0) return 1;
  if (ok.load() + failed.load() != producers * per_producer) return 2;
  if (g.healthy() != 2 || exs[2]->healthy()) return 3;   // the failing backend was isolated
  return 0;
}
