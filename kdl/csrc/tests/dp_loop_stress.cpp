// Stress of the data-parallel state machine (runtime/dp_core.h) on the loopback platform
// (runtime/dp_loop.h), run under ThreadSanitizer and ASan+UBSan by tests/test_sanitizers.py:
// rank 0's DpLeader (heartbeat on) under the real DynamicBatcher + Executor, world-1 follower
// threads, producer threads submitting random request sizes; every request must get exactly
// its own rows; a DP_RELOAD to a new model version mid-run (new communicators, followers
// rebuild) and a second phase under it; DP_STOP; then a dead-follower phase in which the
// leader must fail within its timeout and every follower thread must end.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <memory>
#include <random>
#include <thread>
#include <vector>

#include "../runtime/dp_loop.h"
#include "../runtime/executor.h"

using namespace kdl;

namespace {
constexpr size_t ITEM = 32;
constexpr int COLS = 3, NSLOTS = 2;
const std::vector<int> BUCKETS = {1, 2, 4};

struct Ids {
  std::string s, g;
};

// follower rank r: serve epochs until STOP (1) or an error (-1)
int follower(int world, int r, const std::vector<Ids>& ids, double liveness, std::atomic<int>* forwards) {
  int epoch = 0, version = 0;
  for (;;) {
    loop::Device dev(r, NSLOTS, ITEM, 4, COLS, BUCKETS, version, 50);
    loop::Comm s(ids[epoch].s, world, r), g(ids[epoch].g, world, r);
    DpCtrl c{};
    try {
      LoopDpFollower f(&dev, &s, &g);
      c = f.run(liveness);
    } catch (const std::exception&) {
      forwards->fetch_add((int)dev.forwards());
      return -1;
    }
    forwards->fetch_add((int)dev.forwards());
    if (c.cmd == DP_RELOAD) {
      ++epoch;
      version = c.version;
      continue;
    }
    return 1;
  }
}

// producers against one batcher; returns bad rows (wrong logits)
int produce(DynamicBatcher& b, int producers, int per, int version, int world, std::atomic<int>* ok, std::atomic<int>* failed) {
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int p = 0; p < producers; ++p)
    th.emplace_back([&, p] {
      std::mt19937 rng(p + 17 * version);
      for (int q = 0; q < per; ++q) {
        const int n = 1 + rng() % (4 * world);
        std::vector<uint8_t> data(n * ITEM);
        std::vector<uint32_t> id(n);
        for (int i = 0; i < n; ++i) {
          id[i] = uint32_t(p * 10000 + q * 16 + i);
          memcpy(&data[i * ITEM], &id[i], 4);
          for (size_t k = 4; k < ITEM; ++k) data[i * ITEM + k] = uint8_t(rng());
        }
        const int64_t t = b.submit(data.data(), n, 0);
        std::vector<float> out(n * COLS);
        if (t < 0 || b.wait(t, out.data(), out.size()) != ST_OK) {
          failed->fetch_add(1);
          continue;
        }
        for (int i = 0; i < n; ++i)
          for (int k = 0; k < COLS; ++k)
            if (out[i * COLS + k] != loop::Device::logit(id[i], k, version)) bad++;
        ok->fetch_add(1);
      }
    });
  for (auto& t : th) t.join();
  return bad.load();
}

BatcherOptions bopts(int world) {
  BatcherOptions o;
  o.max_batch_size = 4 * world;
  o.batch_timeout_us = 300;
  o.max_enqueued_batches = 256;
  o.allowed_batch_sizes = {world, 2 * world, 4 * world};
  o.item_bytes = ITEM;
  o.out_cols = COLS;
  return o;
}
}  // namespace

int main(int argc, char** argv) {
  const int world = argc > 1 ? atoi(argv[1]) : 4;
  const int producers = argc > 2 ? atoi(argv[2]) : 4;
  const int per = argc > 3 ? atoi(argv[3]) : 40;
  std::vector<Ids> ids;
  for (int e = 0; e < 3; ++e) ids.push_back({loop::unique_id(), loop::unique_id()});
  std::atomic<int> forwards{0}, ok{0}, failed{0};
  std::vector<std::thread> fth;
  std::vector<int> frc(world, 0);
  for (int r = 1; r < world; ++r)
    fth.emplace_back([&, r] { frc[r] = follower(world, r, ids, 5.0, &forwards); });

  int bad = 0;
  for (int epoch = 0; epoch < 2; ++epoch) {
    const int version = epoch == 0 ? 0 : 7;
    loop::Device dev0(0, NSLOTS, ITEM, 4 * world, COLS, BUCKETS, version, 50);
    loop::Comm s(ids[epoch].s, world, 0), g(ids[epoch].g, world, 0);
    LoopDpLeader leader(&dev0, &s, &g, BUCKETS, 5.0, 0.02);
    DynamicBatcher b(bopts(world));
    ExecGroup grp;
    ExecOptions eo;
    eo.name = "dp";
    eo.poll_us = 2000;
    Executor ex(&b, leader.api(), &grp, eo);
    ex.start();
    bad += produce(b, producers, per, version, world, &ok, &failed);
    std::this_thread::sleep_for(std::chrono::milliseconds(100));   // idle: heartbeat pings
    ex.stop();
    if (leader.send_ctrl(epoch == 0 ? DP_RELOAD : DP_STOP, 7) != 0) {
      printf("send_ctrl failed\n");
      return 4;
    }
    b.shutdown();
  }
  for (auto& t : fth) t.join();
  for (int r = 1; r < world; ++r)
    if (frc[r] != 1) {
      printf("follower %d did not stop cleanly\n", r);
      return 5;
    }

  // dead follower: the leader fails within its timeout, the rest of the followers end on silence
  {
    const auto id = Ids{loop::unique_id(), loop::unique_id()};
    std::vector<Ids> one = {id};
    std::vector<std::thread> th;
    std::vector<int> rc(world, 0);
    for (int r = 1; r < world; ++r) th.emplace_back([&, r] { rc[r] = follower(world, r, one, 1.0, &forwards); });
    loop::Device dev0(0, NSLOTS, ITEM, 4 * world, COLS, BUCKETS, 0, 50);
    loop::Comm s(id.s, world, 0), g(id.g, world, 0);
    LoopDpLeader leader(&dev0, &s, &g, BUCKETS, 0.5, 0.0);
    DynamicBatcher b(bopts(world));
    ExecGroup grp;
    ExecOptions eo;
    eo.max_failures = 2;
    eo.poll_us = 2000;
    Executor ex(&b, leader.api(), &grp, eo);
    ex.start();
    std::atomic<int> ok2{0}, failed2{0};
    bad += produce(b, 2, 5, 0, world, &ok2, &failed2);
    {
      loop::Comm ks(id.s, world, world - 1), kg(id.g, world, world - 1);   // same worlds: mark the last rank dead
      ks.kill();
      kg.kill();
    }
    bad += produce(b, 2, 5, 0, world, &ok2, &failed2);
    ex.stop();
    b.shutdown();
    for (auto& t : th) t.join();
    if (!leader.broken() || ex.healthy() || failed2.load() == 0) {
      printf("dead follower not detected (broken=%d healthy=%d failed=%d)\n", leader.broken(), ex.healthy(), failed2.load());
      return 6;
    }
  }
  printf("world=%d ok=%d failed=%d bad=%d forwards=%d\n", world, ok.load(), failed.load(), bad, forwards.load());
  if (bad != 0 || ok.load() != 2 * producers * per || failed.load() != 0) return 1;
  return 0;
}
