#!/usr/bin/env python
"""Depthwise KxK (EfficientNet-B7 MBConv) kernel sweep at batch 32: numerics of every
timed config vs a torch fp32 oracle, time of the host heuristic at several LDS
budgets, and an explicit (cg, rb, tw, seg) tile grid. Prints the best configs per
shape. Shapes are the B7 600x600 depthwise layers (count = layers of that shape)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from kdl.ops import _lib  # noqa: E402

# name: (H, W, C, K, S, layers)
SHAPES = {
    "s1a": (300, 300, 64, 3, 1, 1), "s1": (300, 300, 32, 3, 1, 3), "s2a": (300, 300, 192, 3, 2, 1),
    "s2": (150, 150, 288, 3, 1, 6), "s3a": (150, 150, 288, 5, 2, 1), "s3": (75, 75, 480, 5, 1, 6),
    "s4a": (75, 75, 480, 3, 2, 1), "s4": (38, 38, 960, 3, 1, 9), "s5a": (38, 38, 960, 5, 1, 1),
    "s5": (38, 38, 1344, 5, 1, 9), "s6a": (38, 38, 1344, 5, 2, 1), "s6": (19, 19, 2304, 5, 1, 12),
    "s7a": (19, 19, 2304, 3, 1, 1), "s7": (19, 19, 3840, 3, 1, 3),
}


def smem(K, S, cg, rb, tw):
    patch = ((rb - 1) * S + K) * ((tw - 1) * S + K) * cg * 16
    return max(K * K * cg * 8 * 4 + patch, (256 * 8 + 64) * 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--grid", action="store_true", help="also sweep explicit (cg, rb, tw, seg) tiles")
    ap.add_argument("--max-lds", type=int, default=96)
    ap.add_argument("--direct", action="store_true", help="sweep the direct streaming kernel (algo 2) only")
    a = ap.parse_args()
    C_ = _lib.lib()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev).manual_seed(0)
    tot_auto = tot_best = 0.0
    for name in a.shapes.split(","):
        H, W, C, K, S, nl = SHAPES[name]
        B, pad = a.batch, (K - 1) // 2
        OH, OW = (H + 2 * pad - K) // S + 1, (W + 2 * pad - K) // S + 1
        Cs = max(8, C // 24)
        x = torch.randn(B, H, W, C, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(K * K, C, device=dev, generator=g) * 0.2).float().contiguous()
        bias = (torch.randn(C, device=dev, generator=g) * 0.1).float().contiguous()
        w1 = (torch.randn(Cs, C, device=dev, generator=g) * 0.05).float().contiguous()
        y = torch.empty(B, OH, OW, C, device=dev, dtype=torch.bfloat16)
        base = dict(x=x.data_ptr(), w=w.data_ptr(), bias=bias.data_ptr(), y=y.data_ptr(), w1=w1.data_ptr(),
                    B=B, H=H, W=W, C=C, OH=OH, OW=OW, K=K, S=S, pad=pad, act=2, Cs=Cs)
        pool = torch.empty(B * 4 * 1024 * 1024 // 4 // B, device=dev)   # 4 MB of partials
        base["pool"] = pool.data_ptr()
        xf = x.float().permute(0, 3, 1, 2)
        ref = F.conv2d(xf, w.t().reshape(C, 1, K, K), bias, stride=S, padding=pad, groups=C)
        ref = F.silu(ref).permute(0, 2, 3, 1)
        scale = ref.abs().max().item()

        def ok(kw):
            cg, rb, tw, nt, seg = C_.dwk_tiles({**base, **kw})
            return nt * Cs <= pool.numel() // B

        def tm(kw, n=20):
            for _ in range(3):
                C_.dwk({**base, **kw}, s)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                C_.dwk({**base, **kw}, s)
            e1.record()
            e1.synchronize()
            err = ((y.float() - ref).abs().max() / scale).item()
            return e0.elapsed_time(e1) / n * 1e3, err

        gb = (B * H * W * C + B * OH * OW * C) * 2 / 1e9
        res = []
        t0, e = tm({})
        print(f"{name:4s} {H}x{W}x{C} k{K}s{S} x{nl}: auto {t0:7.1f} us {gb / t0 * 1e3:5.2f} TB/s err {e:.1e} "
              f"tiles {C_.dwk_tiles(base)}", flush=True)
        assert e < 2e-2, e
        for alg in (1, 2):
            t, e = tm(dict(algo=alg))
            assert e < 2e-2, (alg, e)
            print(f"      algo {alg} (default tiles {C_.dwk_tiles({**base, 'algo': alg})}): {t:7.1f} us "
                  f"{gb / t * 1e3:5.2f} TB/s", flush=True)
        if a.direct:
            for seg, rb, pd in [(sg, r, p) for sg in (2, 4) for r in (0, 4, 8, 12, 16, 24, 38, 75) for p in (1, 3)]:
                    if rb > OH:
                        continue
                    kw = dict(algo=2, seg=seg, rb=rb, pd=pd)
                    if not ok(kw):
                        continue
                    t, e = tm(kw)
                    assert e < 2e-2, (kw, e)
                    res.append((t, kw, C_.dwk_tiles({**base, **kw})[:3]))
        for kb in (() if a.direct else (16, 24, 32, 40, 48, 64, 80, 96)):
            for seg in (3, 4, 5, 7):
                kw = dict(lds_kb=kb, seg=seg, algo=1)
                if not ok(kw):
                    continue
                t, e = tm(kw)
                assert e < 2e-2, (kw, e)
                res.append((t, kw, C_.dwk_tiles({**base, **kw})[:3]))
        if a.grid and not a.direct:
            C8 = C // 8
            tws = sorted({(OW + k - 1) // k for k in range(1, 9)} - {0})
            for cg in [d for d in (1, 2, 4, 8) if C8 % d == 0]:
                for tw in tws:
                    if tw > 64:
                        continue
                    for rb in (1, 2, 3, 4, 6, 8, 12, 16):
                        if rb > OH or smem(K, S, cg, rb, tw) > a.max_lds * 1024:
                            continue
                        for seg in (3, 5, 7):
                            kw = dict(cg=cg, rb=rb, tw=tw, seg=seg)
                            if not ok(kw):
                                continue
                            t, e = tm(kw, 10)
                            assert e < 2e-2, (kw, e)
                            res.append((t, kw, (cg, rb, tw)))
        if not res:
            res.append((t0, {}, None))
        res.sort(key=lambda r: r[0])
        for t, kw, tiles in res[:6]:
            lds = f"smem {smem(K, S, *tiles) // 1024} KiB" if kw.get("algo") == 1 else ""
            print(f"      {t:7.1f} us {gb / t * 1e3:5.2f} TB/s  {kw} tiles={tiles} {lds}", flush=True)
        tot_auto += t0 * nl
        tot_best += res[0][0] * nl
    print(f"B7 depthwise total over the listed shapes (x layers): auto {tot_auto:.0f} us, best {tot_best:.0f} us")


if __name__ == "__main__":
    main()
