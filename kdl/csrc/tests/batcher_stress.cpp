// Multi-threaded stress test of the native DynamicBatcher, built and run under
// ThreadSanitizer and AddressSanitizer+UBSan by tests/test_sanitizers.py
// (SURVEY.md §5 "Race detection / sanitizers": TSAN/ASAN on a CPU build of the
// batcher). Producers submit requests of random sizes with random deadlines
// (some already expired, some abandoned mid-flight), several consumer threads
// form batches, copy payloads, "run" them (result row = item's first byte) and
// finish; a late shutdown races in-flight waits. Every completed request must
// get back exactly its own rows. argv[3] = item bytes: large items (e.g. 262144)
// make every full batch go through the persistent CopyPool from 3 consumers at once,
// and every byte of each item is checked in the staging copy.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <random>
#include <thread>
#include <vector>

#include "../runtime/batcher.h"

using namespace kdl;

int main(int argc, char** argv) {
  const int producers = argc > 1 ? atoi(argv[1]) : 8;
  const int per_producer = argc > 2 ? atoi(argv[2]) : 300;
  BatcherOptions o;
  o.max_batch_size = 16;
  o.batch_timeout_us = 200;
  o.max_enqueued_batches = 64;
  o.allowed_batch_sizes = {1, 2, 4, 8, 16};
  o.item_bytes = argc > 3 ? size_t(atol(argv[3])) : 64;
  o.copy_threads = 4;
  o.out_cols = 3;
  DynamicBatcher b(o);
  std::atomic<int> ok{0}, expired{0}, rejected{0}, bad{0};
  std::atomic<bool> stop{false};

  std::vector<std::thread> consumers;
  for (int c = 0; c < 3; ++c) {
    consumers.emplace_back([&, c] {
      std::vector<uint8_t> staging(o.item_bytes * o.max_batch_size);
      std::vector<float> results(o.out_cols * o.max_batch_size);
      std::mt19937 rng(1000 + c);
      while (!stop.load()) {
        Batch bt;
        if (!b.next_batch(staging.data(), 2000, &bt)) continue;
        for (int i = 0; i < bt.bucket; ++i) {
          // every byte of a real item must carry its fill value (pooled piece copies)
          bool whole = true;
          if (i < bt.n_real)
            for (size_t q = 1; q < o.item_bytes; q += 4093) whole &= staging[i * o.item_bytes + q] == staging[i * o.item_bytes];
          for (int k = 0; k < o.out_cols; ++k)
            results[i * o.out_cols + k] = i < bt.n_real ? (whole ? (float)staging[i * o.item_bytes] + k : -7.f) : -1.f;
        }
        if (rng() % 8 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 300));
        b.finish(bt, results.data(), ST_OK);
      }
    });
  }
  std::vector<std::thread> prods;
  for (int p = 0; p < producers; ++p) {
    prods.emplace_back([&, p] {
      std::mt19937 rng(p);
      for (int r = 0; r < per_producer; ++r) {
        const int n = 1 + rng() % 5;
        std::vector<uint8_t> data(n * o.item_bytes);
        for (int i = 0; i < n; ++i) memset(&data[i * o.item_bytes], (p * 31 + r * 7 + i) & 0x7f, o.item_bytes);
        const int mode = rng() % 10;
        int64_t deadline = 0;
        if (mode == 0) deadline = now_us() - 1;                 // already expired
        else if (mode == 1) deadline = now_us() + rng() % 500;  // may expire while queued
        const int64_t t = b.submit(data.data(), n, deadline);
        if (t < 0) { rejected++; continue; }
        std::vector<float> out(n * o.out_cols);
        const int st = b.wait(t, out.data(), out.size());
        if (st == ST_OK) {
          for (int i = 0; i < n; ++i)
            for (int k = 0; k < o.out_cols; ++k)
              if (out[i * o.out_cols + k] != (float)((p * 31 + r * 7 + i) & 0x7f) + k) bad++;
          ok++;
        } else if (st == ST_DEADLINE) {
          expired++;
        } else {
          rejected++;
        }
      }
    });
  }
  for (auto& t : prods) t.join();
  // shutdown while consumers may be inside next_batch
  b.shutdown();
  stop = true;
  for (auto& t : consumers) t.join();
  const BatcherStats s = b.stats();
  printf("ok=%d expired=%d rejected=%d bad=%d batches=%lld items=%lld\n", ok.load(), expired.load(),
         rejected.load(), bad.load(), (long long)s.batches, (long long)s.items);
  if (bad.load() != 0 || ok.load() == 0) return 1;
  if (ok.load() + expired.load() + rejected.load() != producers * per_producer) return 2;
  return 0;
}
