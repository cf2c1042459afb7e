"""Whole-graph tuner logic (kdl/engine/graph_tune.py) on a fake engine whose 'graph time' is
a pure function of its table: challengers win only by more than the margin, --steps-re limits
the tuned steps, --tie moves matching steps together, the time budget stops a pass and the
save callback sees every accepted table."""
from types import SimpleNamespace

import pytest

from kdl.engine import graph_tune as GT


class FakeEngine:
    def __init__(self, names, variants):
        self.steps = [SimpleNamespace(name=n) for n in names]
        self.variants = variants
        self.table = {n: [0, 0] for n in names}

    def tuning(self):
        return dict(self.table)

    def apply_tuning(self, t):
        self.table = {k: list(v) for k, v in t.items()}

    def conv_steps(self):
        return self.steps

    def _variants(self, step):
        return self.variants


def _cost(best):
    """graph time: 1 ms + 0.1 ms per step not on its best cfg."""
    def graph_time(eng, b, reps=30, warm=3):
        return 1.0 + 0.1 * sum(1 for n, v in eng.table.items() if v[1] != best.get(n, 0))
    return graph_time


@pytest.fixture
def patched(monkeypatch):
    def install(best):
        monkeypatch.setattr(GT, "graph_time", _cost(best))
    return install


def test_accepts_wins_and_saves(patched):
    eng = FakeEngine(["a", "b", "c"], [(False, 0), (False, 1), (True, 2)])
    patched({"a": 1, "c": 2})
    saved = []
    t = GT.graph_tune(eng, 32, log=lambda m: None, save=lambda tb: saved.append(dict(tb)))
    assert t == {"a": [0, 1], "b": [0, 0], "c": [1, 2]}
    assert eng.table == t
    assert len(saved) == 2 and saved[-1] == t


def test_steps_re_only_tunes_matching(patched):
    eng = FakeEngine(["conv2d_2", "block5_sepconv1", "conv2d_3"], [(False, 0), (False, 1)])
    patched({"conv2d_2": 1, "block5_sepconv1": 1, "conv2d_3": 1})
    t = GT.graph_tune(eng, 32, log=lambda m: None, steps_re=r"conv2d_[23]")
    assert t["conv2d_2"] == [0, 1] and t["conv2d_3"] == [0, 1] and t["block5_sepconv1"] == [0, 0]


def test_tie_moves_layers_together(patched):
    names = [f"encoder_layer_{i}.qkv" for i in range(3)]
    eng = FakeEngine(names, [(False, 0), (False, 5)])
    patched({n: 5 for n in names})
    logs = []
    t = GT.graph_tune(eng, 32, log=logs.append, tie=r"encoder_layer_\d+")
    assert all(v == [0, 5] for v in t.values())
    assert sum("x3" in m for m in logs) == 1          # one group of three


def test_budget_stops_before_the_next_step(patched, monkeypatch):
    eng = FakeEngine(["a", "b"], [(False, 0), (False, 1)])
    patched({"a": 1, "b": 1})
    clock = iter([0.0] + [100.0] * 50)                 # t0, then every check is past the budget
    monkeypatch.setattr(GT.time, "time", lambda: next(clock))
    logs = []
    t = GT.graph_tune(eng, 32, log=logs.append, budget_s=10)
    assert t == {"a": [0, 0], "b": [0, 0]}
    assert any("time budget" in m for m in logs)


def test_margin_rejects_small_wins(monkeypatch):
    eng = FakeEngine(["a"], [(False, 0), (False, 1)])
    monkeypatch.setattr(GT, "graph_time", lambda e, b, reps=30, warm=3: 1.0 - 0.001 * e.table["a"][1])
    t = GT.graph_tune(eng, 32, log=lambda m: None, margin=0.002)
    assert t == {"a": [0, 0]}
