#!/usr/bin/env python
"""ViT-B/16 linears: our HIP GEMMs vs the vendor libraries on the same box.

For every distinct linear of an encoder layer (QKV, out_proj, mlp.0, mlp.3) and the
patch embedding, at the bench shape (batch 32 -> M = 32 * 197 token rows), times

  ours      the engine's tuned launch (kdl/ops/conv.py LDS-DMA MFMA GEMM, bf16; or
            gemm_f8.hip, e4m3 with block scales) WITH its fused epilogue (bias, GELU,
            residual add, e4m3 output scaling) -- exactly what the captured graph runs
  hipblaslt torch.nn.functional.linear in bf16 (hipBLASLt), GEMM + bias only, and
            GEMM + the same epilogue as separate torch ops
  scaled_mm torch._scaled_mm e4m3 x e4m3 -> bf16 with per-tensor scales (fp8 rows)

each as the median of ``--reps`` runs of ``--iters`` back-to-back launches (CUDA events).
One JSON line per (GEMM, dtype):

    python tools/gemm_vs_vendor.py [--batch 32] > profiles/vit_gemm_vs_vendor.jsonl
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def _time(fn, iters: int, reps: int) -> float:
    for _ in range(3):
        fn()
    out = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        out.append(e0.elapsed_time(e1) * 1e3 / iters)
    return statistics.median(out)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sweep", action="store_true", help="also time every candidate tile config of each GEMM")
    a = ap.parse_args(argv)
    from kdl.engine import registry
    from kdl.engine.tuning import tuning_path
    from kdl.models import vit as V
    B = a.batch
    dev = torch.device("cuda")
    params = V.init_params(seed=0)
    print(f"# tools/gemm_vs_vendor.py --batch {B}: us per launch (median of {a.reps} x {a.iters}); "
          "tflops = 2MNK / ours", flush=True)
    for fam in ("vit_b16", "vit_b16_fp8"):
        info = registry.get(fam)
        eng = info.engine(params, B, dev)
        tp = tuning_path(info.tuning or fam, B)
        if tp.exists():
            eng.load_tuning(tp)
        seen = set()
        for st in eng.conv_steps():
            key = st.name.split(".")[-1] if "encoder_layer" in st.name else st.name
            if key in seen or ("encoder_layer" in st.name and "encoder_layer_0." not in st.name):
                continue
            seen.add(key)
            lay = st.layer
            N = lay.n
            K = lay.K if hasattr(lay, "K") else lay.k
            M = B * (V.TOKENS - 1) if st.name == "conv_proj" else B * V.TOKENS
            with torch.cuda.stream(eng.stream):
                ours = _time(lambda: eng._emit_conv(None, st, B), a.iters, a.reps)
            torch.cuda.synchronize()
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
            bias = torch.randn(N, device=dev, dtype=torch.bfloat16)
            res = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
            gelu = key in ("mlp.0",)
            resid = key in ("out_proj", "mlp.3")
            lin = _time(lambda: torch.nn.functional.linear(x, w, bias), a.iters, a.reps)

            def full():
                y = torch.nn.functional.linear(x, w, bias)
                if gelu:
                    y = torch.nn.functional.gelu(y)
                if resid:
                    y = y + res
                return y
            lin_ep = _time(full, a.iters, a.reps)
            row = {"family": fam, "gemm": key, "M": M, "N": N, "K": K, "ours_us": round(ours, 2),
                   "ours_tflops": round(2 * M * N * K / ours / 1e6, 1), "hipblaslt_bf16_us": round(lin, 2),
                   "hipblaslt_bf16_plus_epilogue_us": round(lin_ep, 2)}
            if fam.endswith("fp8"):
                try:
                    x8 = x.to(torch.float8_e4m3fn)
                    w8 = w.to(torch.float8_e4m3fn)
                    one = torch.ones((), device=dev)
                    sm = _time(lambda: torch._scaled_mm(x8, w8.t(), scale_a=one, scale_b=one, bias=bias,
                                                        out_dtype=torch.bfloat16), a.iters, a.reps)
                    row["scaled_mm_e4m3_us"] = round(sm, 2)
                except Exception as e:  # noqa: BLE001 - report, do not fail the sweep
                    row["scaled_mm_e4m3_us"] = None
                    row["scaled_mm_error"] = str(e)[:200]
            if a.sweep:
                sw = {}
                with torch.cuda.stream(eng.stream):
                    for split, cfg in st.layer.variants(None):
                        sw[cfg] = round(_time(lambda: eng._emit_conv(None, st, B, split=split, cfg=cfg),
                                              a.iters, a.reps), 2)
                torch.cuda.synchronize()
                row["tuned_cfg"] = st.layer.cfg
                row["sweep_us"] = dict(sorted(sw.items(), key=lambda kv: kv[1]))
            print(json.dumps(row), flush=True)
        del eng
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
