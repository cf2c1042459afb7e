"""Native RCCL data-parallel serving (kdl/csrc/runtime/comm.cpp) -- CPU half.

The leader (rank 0's DpLeader) and followers (DpFollower) post exactly the message lists of
kdl/csrc/runtime/dp_schedule.h. Here every rank's lists are generated for a random sequence of
steps (varying shard sizes, then STOP) and matched pairwise per channel: each (sender, receiver)
pair must see the same sequence of message sizes on both ends, or RCCL would deadlock or
mis-deliver. Reference topology being replaced: Deployment replicas behind a ClusterIP Service
(/root/reference/tf-serving-clothing-model-deployment.yaml:8)."""
import random

import pytest

from kdl.ops import _lib

pytestmark = pytest.mark.skipif(not _lib.rt_available(), reason="kdl._rt not built")
ITEM, COLS = 299 * 299 * 3, 10


def _simulate(world, steps):
    R = _lib.rt()
    sent = {}     # (channel, src, dst) -> [bytes...]
    recv = {}
    def add(rank, ops):
        for ch, is_send, peer, nbytes, _what, _grp in ops:
            key = (ch, rank, peer) if is_send else (ch, peer, rank)
            (sent if is_send else recv).setdefault(key, []).append(nbytes)
    for r in range(1, world):       # follower prologue: the first control receive
        add(r, [(0, False, 0, R.DP_CTRL_BYTES, 0, 0)])
    for cmd, shard in steps:
        add(0, R.dp_leader_step(world, ITEM, COLS, cmd, shard))
        for r in range(1, world):
            add(r, R.dp_follower_step(world, ITEM, COLS, cmd, shard, cmd == 1))
    return sent, recv


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_every_send_has_a_matching_receive(world):
    R = _lib.rt()
    rng = random.Random(world)
    buckets = [1, 2, 4, 8, 16, 32]
    steps = []
    for _ in range(50):
        n = rng.randint(1, 32 * world)
        steps.append((1, R.dp_plan_shard(n, world, buckets)))
    steps.append((0, 0))            # STOP
    sent, recv = _simulate(world, steps)
    assert sent == recv
    if world > 1:
        # per follower: 51 control words, 50 shards in, 50 logits out
        assert len(sent[(0, 0, 1)]) == 101 and len(sent[(1, 1, 0)]) == 50
        assert sent[(1, 1, 0)][0] == steps[0][1] * COLS * 4


def test_reload_control_word_then_batches_match():
    """A DP_RELOAD ends the followers' loop; after the rebuild both ends restart the schedule
    (follower prologue again) and still match."""
    R = _lib.rt()
    s1, r1 = _simulate(4, [(1, 8), (1, 32), (2, 0)])
    s2, r2 = _simulate(4, [(1, 4), (0, 0)])
    assert s1 == r1 and s2 == r2


def test_plan_shard_picks_the_smallest_bucket():
    R = _lib.rt()
    b = [1, 2, 4, 8, 16, 32]
    assert R.dp_plan_shard(1, 8, b) == 1 and R.dp_plan_shard(9, 8, b) == 2
    assert R.dp_plan_shard(256, 8, b) == 32 and R.dp_plan_shard(257, 8, b) == 0   # too big: none
