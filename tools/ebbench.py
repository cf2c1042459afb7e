"""Fused entry block vs the unfused lowering, per-op device times at batch B (one MI355X).

    python tools/ebbench.py [--batch 32] [--iters 20]
"""
import argparse
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--blocks", default="2,3")
    a = ap.parse_args()
    import torch
    from kdl.engine.tuning import tuning_path
    from kdl.engine.xception import XceptionEngine
    from kdl.models import xception as X
    p = X.init_params(seed=0)
    res = {}
    for fused in ("0", a.blocks):
        os.environ["KDL_ENTRY_BLOCK"] = fused
        e = XceptionEngine(p, max_batch=a.batch, buckets=[a.batch])
        e.load_tuning(tuning_path("xception", a.batch))
        x = torch.randint(0, 256, (a.batch, 299, 299, 3), dtype=torch.uint8, device="cuda")
        e.forward(x)
        prof = e.profile(a.batch, a.iters)
        res[fused] = prof
        tot = sum(t for _, t in prof)
        print(f"== KDL_ENTRY_BLOCK={fused}: {len(prof)} launches, eager sum {tot * 1e3:.1f} us", flush=True)
        for name, t in prof:
            if name.startswith(("block2", "conv2d", "block3", "conv2d_1", "block4", "conv2d_2")):
                print(f"   {name:24s} {t * 1e3:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
