"""Numerics gate for every benchmarked configuration.

Builds EXACTLY what ``bench.py --model <m>`` times -- the family's engine at batch 32,
its committed tuning table (kdl/tuning/<family>_b32.json), the default stage-pipeline
cut, hipGraph replays with several batches in flight on two input slots -- and compares
every batch's logits with the plain-PyTorch fp32 oracle of the same random-init weights
(run on the GPU in fp32; gfx950 has no reduced-precision fp32 GEMM mode to fall into):

* relative max logit error (max |engine - oracle| / max |oracle|),
* cosine similarity per image,
* top-1 agreement on at least 30 of the 32 images of every batch: strict (engine argmax ==
  oracle argmax) for bf16 / fp16 families; for EfficientNet-B7 and the fp8 ViT "up to ties":
  the engine's top-1 class must score within that image's own max logit error of the
  oracle's best class (random-init 1000-class heads have near-tied logits: B7's smallest
  oracle top-1/top-2 margin is 0.0000-0.0010 of the logit range, so strict argmax there
  measures the tie, not the engine). Strict counts are printed for every family.

Tolerances are per family and dtype: bf16 Xception (36 fused layers) is held to 5 %,
fp16 ResNet-50 to 5 %, bf16 ViT to 5 %, fp8-e4m3 ViT and bf16 EfficientNet-B7 (55 MBConv
blocks at 600x600) looser, with the measured values printed so the margins are visible
in the GPU log.
"""
import pytest
import torch
import torch.nn.functional as F

from kdl.engine import registry
from kdl.engine.stages import StagePipe
from kdl.engine.tuning import tuning_path

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
B = 32

# family -> (max rel logit err, min per-image cosine, min top-1 agreements of 32, tie-aware, batches)
GATES = {
    "xception": (0.05, 0.995, 30, False, 4),
    "resnet50": (0.05, 0.995, 30, False, 3),
    "vit_b16": (0.05, 0.995, 30, False, 3),
    # round 4 measured (profiles/numerics_gate_r4.txt): fp8 ViT 0.094-0.113, B7 0.150-0.174
    "vit_b16_fp8": (0.13, 0.99, 30, True, 3),
    "efficientnet_b7": (0.20, 0.99, 30, True, 2),
}


# second gate for EfficientNet-B7: against the bf16-ROUNDING oracle
# (tools/b7_trace.py: fp32 math, rounded to bf16 exactly where the engine stores bf16), which the
# engine tracks far more closely than the fp32 oracle (0.074 measured, profiles/b7_numerics_r5.txt),
# so a 2x numerics regression no longer hides inside the 20 % fp32 gate
BF16_ORACLE_GATES = {"efficientnet_b7": 0.10}


def _bf16_oracle(params, x_u8):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    from tools import b7_trace as T
    with torch.no_grad():
        logits, _ = T.run(T.Folded(params, DEV), x_u8.to(DEV), "bf16")
    return logits.float().cpu()


def _oracle(info, params, x_u8):
    p = {k: v.to(DEV) for k, v in params.items()}
    with torch.no_grad():
        return info.oracle(p, x_u8.to(DEV)).float().cpu()


def _pipelined_logits(info, params, imgs):
    """bench.py's engine: StagePipe(engine(b32), default cut) + committed table, graph replays,
    two slots, batch i+1's stage 1 overlapping batch i's stage 2."""
    eng = StagePipe(info.engine(params, B, DEV), info.stage_cut)
    tp = tuning_path(info.tuning or info.name, B)
    assert tp.exists(), f"no committed tuning table {tp}"
    eng.load_tuning(tp)
    slots = eng.add_input_slots(2)
    for j in range(2):
        eng.program(B, True, j)
    done = [torch.cuda.Event() for _ in range(2)]
    outs = []
    for i, x in enumerate(imgs):
        j = i % 2
        if i >= 2:
            done[j].synchronize()
            outs.append(eng.slot_logits(j).cpu().clone())
        slots[j].copy_(x.to(DEV))
        ready = torch.cuda.Event()
        ready.record()
        eng.launch_async(B, [ready], [done[j]], capture=True, slot=j)
    for i in range(max(0, len(imgs) - 2), len(imgs)):
        done[i % 2].synchronize()
        outs.append(eng.slot_logits(i % 2).cpu().clone())
    return eng, outs


@pytest.mark.parametrize("model", list(GATES))
def test_benchmarked_config_matches_fp32_oracle(model):
    tol, cos_min, top1_min, ties, nb = GATES[model]
    info = registry.get(model)
    params = info.init_params(0)
    S = info.input_size
    gen = torch.Generator().manual_seed(2024)
    imgs = [torch.randint(0, 256, (B, S, S, 3), generator=gen, dtype=torch.uint8) for _ in range(nb)]
    eng, outs = _pipelined_logits(info, params, imgs)
    assert len(outs) == nb
    for i, (x, out) in enumerate(zip(imgs, outs)):
        ref = _oracle(info, params, x)
        assert out.shape == ref.shape == (B, info.classes)
        assert torch.isfinite(out).all()
        err = ((out - ref).abs().max() / ref.abs().max()).item()
        cos = F.cosine_similarity(out, ref, dim=1)
        strict = int((out.argmax(1) == ref.argmax(1)).sum())
        # up to ties: the engine's pick scores within this image's own max logit error of the best
        row_err = (out - ref).abs().max(dim=1).values
        picked = ref.gather(1, out.argmax(1, keepdim=True))[:, 0]
        tied = int((picked >= ref.max(dim=1).values - row_err).sum())
        top2 = ref.topk(2, dim=1).values
        margin = (top2[:, 0] - top2[:, 1]).min().item() / ref.abs().max().item()
        agree = tied if ties else strict
        print(f"{model} batch {i}: rel err {err:.4f} (gate {tol}), cos min {cos.min():.5f} (gate {cos_min}), "
              f"top-1 strict {strict}/{B}, up to ties {tied}/{B} (gate {top1_min}, {'ties' if ties else 'strict'}), "
              f"smallest oracle top-1 margin {margin:.4f}")
        assert err <= tol, (model, i, err)
        if model in BF16_ORACLE_GATES:
            rb = _bf16_oracle(params, x)
            err_b = ((out - rb).abs().max() / rb.abs().max()).item()
            print(f"{model} batch {i}: rel err vs the bf16-rounding oracle {err_b:.4f} "
                  f"(gate {BF16_ORACLE_GATES[model]})")
            assert err_b <= BF16_ORACLE_GATES[model], (model, i, err_b)
        assert cos.min().item() >= cos_min, (model, i, cos.min().item())
        assert agree >= top1_min, (model, i, strict, tied)


def test_xception_headline_stages_are_deterministic_and_slot_independent():
    """The same batch through either input slot of the bench pipeline gives bit-identical logits
    (no cross-slot / cross-parity buffer aliasing in the stage versioning)."""
    info = registry.get("xception")
    params = info.init_params(0)
    gen = torch.Generator().manual_seed(7)
    x = torch.randint(0, 256, (B, 299, 299, 3), generator=gen, dtype=torch.uint8)
    y = torch.randint(0, 256, (B, 299, 299, 3), generator=gen, dtype=torch.uint8)
    _, outs = _pipelined_logits(info, params, [x, y, x, y, x])
    assert torch.equal(outs[0], outs[2]) and torch.equal(outs[2], outs[4])
    assert torch.equal(outs[1], outs[3])
