"""Fused entry block vs the unfused lowering, per-op device times at batch B (one MI355X);
``--stamps``: per-phase s_memtime profile of the fused kernel (stamping build, config 100 + id).

    python tools/ebbench.py [--batch 32] [--iters 20] [--blocks 2,3] [--stamps]
"""
import argparse
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def stamps(p, blocks, B):
    import torch
    from kdl.engine.xception import XceptionEngine as XE
    from kdl.models import xception as X
    from kdl.ops.entry_block import CONFIGS, EntryBlock
    geom = {2: (147, 64), 3: (74, 128)}
    for blk in blocks:
        b = X.SPEC[blk - 1]
        s1, s2, r = XE._sep(p, b.main[0], "cuda"), XE._sep(p, b.main[1], "cuda"), XE._pw(p, b.res_conv, "cuda")
        H, C0 = geom[blk]
        cfgs = [2, 13, 15] if blk == 2 else [1]
        for cfg in [c for b in cfgs for c in (b, 100 + b)]:
            eb = EntryBlock(f"block{blk}", s1, s2, r, cfg=cfg)
            x = torch.randn(B, H, H, C0, device="cuda").to(torch.bfloat16)
            y = torch.empty(B, (H - 1) // 2 + 1, (H - 1) // 2 + 1, s1.n, dtype=torch.bfloat16, device="cuda")
            st = torch.zeros(8 * 64 * 5, dtype=torch.int64, device="cuda")
            a = eb.args(x.data_ptr(), y.data_ptr(), B, H, H)
            a["stamps"] = st.data_ptr()
            C = __import__("kdl.ops._lib", fromlist=["lib"]).lib()
            for _ in range(3):
                C.entry_block(cfg, a, torch.cuda.current_stream().cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                C.entry_block(cfg, a, torch.cuda.current_stream().cuda_stream)
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 10 * 1e3
            print(f"block{blk} cfg {cfg}: {t:.1f} us per launch", flush=True)
            if cfg < 100:
                continue
            v = st.view(8, 64, 5).cpu().tolist()
            if cfg in (113, 115):      # warp-specialized: [consumer start, consumer end, producer start, producer end]
                ph = {n: [] for n in ("iteration", "consumers busy", "producers busy")}
                for wg in range(8):
                    for k in range(3, 62):
                        a0, a1 = v[wg][k], v[wg][k + 1]
                        if 0 in a0[:4] or a1[0] == 0:
                            continue
                        ph["iteration"].append(a1[0] - a0[0])
                        ph["consumers busy"].append(a0[1] - a0[0])
                        ph["producers busy"].append(a0[3] - a0[2])
                print("  per iteration (= one step; median shader cycles, 8 workgroups):", flush=True)
                for n, xs in ph.items():
                    if xs:
                        print(f"    {n:20s} {statistics.median(xs):8.0f}", flush=True)
                continue
            ph = {n: [] for n in ("P1 dw1", "P2 gemm1", "P3 dw2", "P4 gemm2+pool", "out+B0")}
            steps_ = 0
            for wg in range(8):
                for k in range(63):
                    s0, s_next = v[wg][k], v[wg][k + 1]
                    if 0 in s0 or s_next[0] == 0 or s0[4] == 0:
                        continue      # warm-up steps (no P3/P4 stamp) or beyond the run
                    steps_ += 1
                    ph["P1 dw1"].append(s0[1] - s0[0])
                    ph["P2 gemm1"].append(s0[2] - s0[1])
                    ph["P3 dw2"].append(s0[3] - s0[2])
                    ph["P4 gemm2+pool"].append(s0[4] - s0[3])
                    ph["out+B0"].append(s_next[0] - s0[4])
            print(f"  per output step (median shader cycles over {steps_} steps, 8 workgroups):", flush=True)
            for n, xs in ph.items():
                if xs:
                    print(f"    {n:16s} {statistics.median(xs):8.0f}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--blocks", default="2,3")
    ap.add_argument("--stamps", action="store_true")
    a = ap.parse_args()
    import torch
    from kdl.engine.tuning import tuning_path
    from kdl.engine.xception import XceptionEngine
    from kdl.models import xception as X
    p = X.init_params(seed=0)
    if a.stamps:
        stamps(p, [int(b) for b in a.blocks.split(",")], a.batch)
        return
    for fused in ("0", a.blocks):
        os.environ["KDL_ENTRY_BLOCK"] = fused
        e = XceptionEngine(p, max_batch=a.batch, buckets=[a.batch])
        e.load_tuning(tuning_path("xception", a.batch))
        x = torch.randint(0, 256, (a.batch, 299, 299, 3), dtype=torch.uint8, device="cuda")
        e.forward(x)
        prof = e.profile(a.batch, a.iters)
        tot = sum(t for _, t in prof)
        print(f"== KDL_ENTRY_BLOCK={fused}: {len(prof)} launches, eager sum {tot * 1e3:.1f} us", flush=True)
        for name, t in prof:
            if name.startswith(("block2", "conv2d", "block3", "block4")):
                print(f"   {name:24s} {t * 1e3:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
