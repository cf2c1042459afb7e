// Data-parallel serving protocol over point-to-point links, as a
// pure schedule: which messages each rank posts for one step, in which order, with which
// sizes. Header-only and device-free, so the SAME code drives the RCCL backend (comm.cpp:
// leader = rank 0's HipExecBackend, followers = DpFollower) and the CPU test that checks
// every rank's sends against its peers' receives (tests/test_dp_native.py via kdl._rt).
//
// Two channels (two communicators, so a step's gather never queues behind the next step's
// scatter): SCATTER carries rank 0 -> rank r the control word, then the uint8 shard;
// GATHER carries rank r -> rank 0 the fp32 logits of that shard.
//
//   leader, step with global bucket G = world x shard:
//     SCATTER  send ctrl (32 B) to r = 1..world-1     (one group)
//              send shard r (shard x item_bytes) to r (one group)   [cmd BATCH only]
//     GATHER   recv logits (shard x out_cols x 4 B) from r = 1..world-1 (one group)
//   follower r, per step:
//     SCATTER  recv ctrl from 0; (BATCH) recv shard from 0
//     GATHER   (BATCH) send logits to 0
//   The follower posts the NEXT step's ctrl receive right behind this step's shard receive,
//   so per-pair message order on each channel is identical on both ends.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace kdl {

// DP_PING: a control word with no batch (the leader's heartbeat while idle); followers re-post
// the control receive in the same slot. A follower that sees no control word for its liveness
// window treats the leader as dead (dp_core.h).
enum DpCmd : int32_t { DP_STOP = 0, DP_BATCH = 1, DP_RELOAD = 2, DP_PING = 3 };

struct DpCtrl {              // 32 bytes on the wire (device-side control word)
  int32_t cmd;
  int32_t shard;             // images per rank (a captured per-rank bucket)
  int32_t n_real;            // real images in the global batch
  int32_t seq;               // step number (checked by followers)
  int32_t version;           // DP_RELOAD: the model version to load
  int32_t pad[3];
};
static_assert(sizeof(DpCtrl) == 32, "wire size");

enum DpChannel : int { DP_SCATTER = 0, DP_GATHER = 1 };

struct DpMsg {
  int channel;               // DpChannel
  bool send;                 // true: this rank sends to `peer`
  int peer;
  size_t bytes;
  int what;                  // 0 ctrl, 1 shard, 2 logits
  int group;                 // messages of one group are posted between one GroupStart / GroupEnd
};

struct DpGeometry {
  int world;
  size_t item_bytes;         // bytes per image (uint8 299x299x3 = 268,203)
  int out_cols;              // logits per image
};

// smallest captured per-rank bucket that holds ceil(n_real / world) images (0: none fits)
inline int dp_plan_shard(int n_real, int world, const std::vector<int>& rank_buckets) {
  const int need = n_real <= 0 ? 1 : (n_real + world - 1) / world;
  int best = 0;
  for (int b : rank_buckets)
    if (b >= need && (best == 0 || b < best)) best = b;
  return best;
}

// leader (rank 0) messages of one step
inline std::vector<DpMsg> dp_leader_step(const DpGeometry& g, int cmd, int shard) {
  std::vector<DpMsg> m;
  for (int r = 1; r < g.world; ++r) m.push_back({DP_SCATTER, true, r, sizeof(DpCtrl), 0, 0});
  if (cmd != DP_BATCH) return m;
  for (int r = 1; r < g.world; ++r) m.push_back({DP_SCATTER, true, r, (size_t)shard * g.item_bytes, 1, 1});
  for (int r = 1; r < g.world; ++r)
    m.push_back({DP_GATHER, false, r, (size_t)shard * g.out_cols * sizeof(float), 2, 2});
  return m;
}

// follower messages of one step (the ctrl receive of THIS step was posted by the previous
// step, or by the loop prologue for step 0); `next` = also post the next step's ctrl receive
inline std::vector<DpMsg> dp_follower_step(const DpGeometry& g, int cmd, int shard, bool next) {
  std::vector<DpMsg> m;
  if (cmd == DP_BATCH) m.push_back({DP_SCATTER, false, 0, (size_t)shard * g.item_bytes, 1, 0});
  if (next) m.push_back({DP_SCATTER, false, 0, sizeof(DpCtrl), 0, 1});
  if (cmd == DP_BATCH) m.push_back({DP_GATHER, true, 0, (size_t)shard * g.out_cols * sizeof(float), 2, 2});
  return m;
}

inline DpMsg dp_follower_prologue() { return {DP_SCATTER, false, 0, sizeof(DpCtrl), 0, 0}; }

}  // namespace kdl
