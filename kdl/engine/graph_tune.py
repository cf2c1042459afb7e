"""Whole-graph tile tuning: coordinate descent on the replay time of the captured
forward (all lanes running), instead of timing each layer alone.

Why: the per-layer autotuner (``EngineBase.autotune``) times a layer's variants
in isolation on an idle chip. In the real step, two lanes replay concurrently
(``lanes.py``) and every kernel shares the chip with the other lane's current
layer, so the solo-fastest tile is only a proxy. Measured on MI355X: at 16
images per lane the middle-flow fused separable conv is 18 % faster alone with
the 64-row tile than with the 96-row tile the b32 table uses, but the 64-row
tile launches 50 % more workgroups, which is exactly what the other lane then
competes with. Only the graph time settles it.

Procedure: start from the committed table; for each tunable layer in graph
order, try every valid (split, cfg) variant on all lanes at once, re-capture the
hipGraphs and time ``reps`` replays of the full forward; a challenger replaces
the incumbent only if it wins an interleaved A/B re-measurement (``confirm``
rounds, median) by more than ``margin``. One pass is ~N_variants graph captures.

    python -m kdl.engine.graph_tune --model xception --batch 32 --lanes 2 \
        --out /tmp/xception_b32_tuned.json
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

import torch


def _steps_of(eng):
    return eng.engines[0].conv_steps() if hasattr(eng, "engines") else eng.conv_steps()


def _variants_of(eng, step):
    e0 = eng.engines[0] if hasattr(eng, "engines") else eng
    return e0._variants(step)


def graph_time(eng, b: int, reps: int = 30, warm: int = 3) -> float:
    """ms per forward replay (all lanes), after (re)capturing the graphs. Stage-pipelined
    engines (``stages.StagePipe``) are timed free-running over two input slots, so
    consecutive batches overlap as they do in bench.py."""
    if getattr(eng, "pipelined", False):
        done = [torch.cuda.Event(), torch.cuda.Event()]
        for r in range(warm + 2):
            eng.launch_async(b, [], [done[r % 2]], slot=r % 2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for r in range(reps):
            eng.launch_async(b, [], [done[r % 2]], slot=r % 2)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / reps
    s = eng.stream
    eng.launch(b, s, capture=True)            # builds + captures any invalidated program
    for _ in range(warm):
        eng.launch(b, s, capture=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        eng.launch(b, s, capture=True)
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def graph_tune(eng, b: int, passes: int = 1, reps: int = 30, confirm: int = 3, margin: float = 0.002,
               log=print, only: set | None = None, tie: str | None = None, verbose: bool = False,
               steps_re: str | None = None, budget_s: float | None = None, save=None) -> dict:
    """``only``: challenge the incumbents with these tile configs only (e.g. newly added ids).
    ``tie``: regex; steps whose names are equal once it is replaced by '*' move together (the
    12 identical encoder layers of a ViT: one layer's few-us win sits inside the margin, the
    same tile on all twelve does not). ``steps_re``: regex; only matching steps are tuned.
    ``budget_s``: stop after this many seconds (the table so far is kept); ``save(table)`` is
    called after every accepted change, so a long pass leaves its progress behind."""
    import re
    table = dict(eng.tuning())
    eng.apply_tuning(table)
    base = statistics.median(graph_time(eng, b, reps) for _ in range(3))
    log(f"start: {base * 1e3:.1f} us/forward")
    t_start = base
    t0 = time.time()
    for p in range(passes):
        changed = 0
        steps = _steps_of(eng)
        groups: dict[str, list] = {}
        for st in steps:
            if steps_re and not re.search(steps_re, st.name):
                continue
            groups.setdefault(re.sub(tie, "*", st.name) if tie else st.name, []).append(st)
        for i, (gname, members) in enumerate(groups.items()):
            if budget_s and time.time() - t0 > budget_s:
                log(f"  time budget ({budget_s:.0f} s) reached at {gname}: stopping")
                break
            step, name = members[0], gname
            cur = table[step.name]
            variants = [v for v in _variants_of(eng, step) if only is None or v[1] in only]
            log(f"  [{i + 1}/{len(groups)}] {name} x{len(members)} ({len(variants)} variants) at {base * 1e3:.1f} us")
            for split, cfg in variants:
                cand = [int(split), int(cfg)]
                if cand == cur:
                    continue
                trial = dict(table, **{m.name: cand for m in members})
                # screen against a FRESH incumbent time taken right before the challenger: a
                # baseline measured minutes earlier drifts with the chip's clock under sustained
                # load (measured: every challenger 4-10 % slower than a stale start, including a
                # hipBLASLt mlp.3 that wins 5 % in bench.py), so a one-sided screen rejected all
                eng.apply_tuning(table)
                t_inc = graph_time(eng, b, reps)
                eng.apply_tuning(trial)
                t = graph_time(eng, b, reps)
                if verbose:
                    log(f"    {cand}: {t * 1e3:.1f} us (incumbent {t_inc * 1e3:.1f})")
                if t >= t_inc * (1 - margin):
                    continue
                # interleaved A/B: incumbent vs challenger, median of `confirm` rounds each
                ta, tb = [], []
                for _ in range(confirm):
                    eng.apply_tuning(table)
                    ta.append(graph_time(eng, b, reps))
                    eng.apply_tuning(trial)
                    tb.append(graph_time(eng, b, reps))
                ma, mb = statistics.median(ta), statistics.median(tb)
                if mb < ma * (1 - margin):
                    log(f"  {name:22s} {cur} -> {cand}: {ma * 1e3:8.1f} -> {mb * 1e3:8.1f} us")
                    table, base, cur = trial, mb, cand
                    changed += 1
                    if save:
                        save(table)
                else:
                    base = ma
            eng.apply_tuning(table)
        log(f"pass {p}: {changed} change(s), {base * 1e3:.1f} us/forward")
        if not changed or (budget_s and time.time() - t0 > budget_s):
            break
    eng.apply_tuning(table)
    log(f"graph tune: {t_start * 1e3:.1f} -> {base * 1e3:.1f} us/forward")
    return table


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="xception")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--lanes", type=int, default=2)
    ap.add_argument("--stages", default=None, metavar="STEP", help="tune a stage-pipelined engine cut after STEP")
    ap.add_argument("--passes", type=int, default=1)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--start", default=None, help="starting table (default: the committed table)")
    ap.add_argument("--out", required=True)
    ap.add_argument("--cfgs", default=None, help="comma list: only these configs challenge the table")
    ap.add_argument("--verbose", action="store_true", help="log every challenger's graph time")
    ap.add_argument("--margin", type=float, default=0.002, help="relative win a challenger must show (screen and A/B)")
    ap.add_argument("--tie", default=None, help=r"regex, e.g. 'encoder_layer_\d+': tune matching layers together")
    ap.add_argument("--steps-re", default=None, help="regex: tune only the matching steps")
    ap.add_argument("--budget-s", type=float, default=None, help="stop after this many seconds")
    a = ap.parse_args(argv)
    from . import registry
    from .tuning import tuning_path
    dev = torch.device("cuda", 0)
    info = registry.get(a.model)
    params = info.init_params(0)
    if a.stages:
        from .stages import StagePipe
        eng = StagePipe(info.engine(params, a.batch, dev), a.stages)
        eng.add_input_slots(2)
    elif a.lanes > 1:
        from .lanes import LaneGroup
        eng = LaneGroup(info, params, a.batch, dev, a.lanes)
    else:
        eng = info.engine(params, a.batch, dev)
    tname = info.tuning or a.model
    start = Path(a.start) if a.start else tuning_path(tname, a.batch, 1 if a.stages else a.lanes)
    if not start.exists():
        start = tuning_path(tname, a.batch)
    eng.load_tuning(start)
    # random input (DVFS / MFMA clock behaviour differs on zeros)
    g = torch.Generator().manual_seed(0)
    inp = eng.inp
    if inp.dtype == torch.uint8:
        inp.copy_(torch.randint(0, 256, tuple(inp.shape), generator=g, dtype=torch.uint8))
    else:
        inp.copy_(torch.rand(tuple(inp.shape), generator=g) * 2 - 1)
    t0 = time.time()
    only = {int(c) for c in a.cfgs.split(",")} if a.cfgs else None
    table = graph_tune(eng, a.batch, passes=a.passes, reps=a.reps, log=lambda m: print(m, flush=True), only=only,
                       tie=a.tie, verbose=a.verbose, margin=a.margin, steps_re=a.steps_re,
                       budget_s=a.budget_s, save=lambda t: Path(a.out).write_text(json.dumps(t, indent=1)))
    Path(a.out).write_text(json.dumps(table, indent=1))
    print(f"wrote {a.out} ({time.time() - t0:.0f} s, started from {start})", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
