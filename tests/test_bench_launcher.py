"""bench.py's own rank launcher (VERDICT r3 "next round" item 1): ``python bench.py --gpus N``
without torch.distributed.run must measure N ranks, not silently one. CPU rehearsal through the
gloo ``--dry-run`` hook: every rank starts with the env a launcher would give it, joins one group
on 127.0.0.1, and rank 0 alone prints one JSON line with ``n_gpus: N``."""
import json
import os
import re
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def _run(args, env, timeout=300):
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], cwd=str(ROOT), env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 4])
def test_self_launch_starts_every_rank(n):
    r = _run(["--gpus", str(n), "--dry-run", "--steps", "3", "--warmup", "1"], _env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout                    # rank 0 alone prints
    res = json.loads(lines[0])
    assert res["n_gpus"] == n and res["config"]["parallelism"] == f"dp{n}" and res["steps"] == 3
    seen = re.findall(r"dry-run rank=(\d+) local_rank=(\d+) world=(\d+) master=([\d.]+):(\d+)", r.stderr)
    assert sorted(int(s[0]) for s in seen) == list(range(n)), r.stderr
    assert all(s[0] == s[1] and int(s[2]) == n and s[3] == "127.0.0.1" for s in seen)
    assert len({s[4] for s in seen}) == 1                 # one rendezvous port


def test_more_ranks_than_visible_gpus_is_refused():
    # refused in the launcher parent, before any rank (or any GPU call) starts
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], _env(HIP_VISIBLE_DEVICES="0"), timeout=120)
    assert r.returncode != 0 and "only 1 GPU(s) visible" in r.stderr, r.stderr[-2000:]


def test_launcher_world_must_match_gpus():
    r = _run(["--gpus", "4", "--dry-run"], _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr
