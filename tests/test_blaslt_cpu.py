"""hipBLASLt GEMM node plumbing on the host (no GPU): which layers offer it, how the tuning
ids map to heuristic ranks, which epilogues it may take, and how a table picks it up."""
import pytest
import torch

from kdl.engine.base import EngineBase, Step
from kdl.ops.conv import BLT_ALGOS, BLT_BASE, MODE_DW, MODE_PW, ConvGemmLayer, cfg_tile, is_blaslt


def _lin(relu_out=0, blaslt=True, n=128, k=64):
    g = torch.Generator().manual_seed(0)
    return ConvGemmLayer("lin", MODE_PW, torch.randn(n, k, generator=g, dtype=torch.float64),
                         torch.randn(n, generator=g), cin_pad=k, n=n, relu_out=relu_out, device="cpu",
                         blaslt=blaslt)


def test_blaslt_ids_are_offered_only_when_asked():
    assert [c for _, c in _lin(blaslt=False).variants() if is_blaslt(c)] == []
    ids = [c for split, c in _lin().variants() if is_blaslt(c)]
    assert ids == list(range(BLT_BASE, BLT_BASE + BLT_ALGOS))
    assert cfg_tile(BLT_BASE)[1] == 16 and _lin().nf(BLT_BASE) == 128 // 16


def test_blaslt_epilogue_mapping():
    x, y, r = 0x1000, 0x2000, 0x3000
    d = _lin(relu_out=0).blaslt_args(x, y, M=100, res=r, algo=3)
    assert (d["act"], d["res"], d["algo"], d["N"], d["K"], d["ldy"]) == (0, r, 3, 128, 64, 128)
    assert _lin(relu_out=2).blaslt_args(x, y, M=100, res=r)["act"] == 1    # ReLU after the residual: C then act
    assert _lin(relu_out=1).blaslt_args(x, y, M=100)["act"] == 1           # ReLU without a residual
    assert _lin(relu_out=3).blaslt_args(x, y, M=100)["act"] == 2           # GELU
    for ro in (1, 3):                                                      # activation BEFORE the add
        with pytest.raises(AssertionError):
            _lin(relu_out=ro).blaslt_args(x, y, M=100, res=r)


def test_blaslt_refused_for_fused_lowerings():
    g = torch.Generator().manual_seed(1)
    w, b = torch.randn(64, 32, generator=g, dtype=torch.float64), torch.randn(64, generator=g)
    with pytest.raises(AssertionError):
        ConvGemmLayer("sep", MODE_DW, w, b, cin_pad=32, n=64, dww=torch.randn(9, 32), device="cpu", blaslt=True)
    with pytest.raises(AssertionError):
        ConvGemmLayer("s2", MODE_PW, w, b, cin_pad=32, n=64, stride=2, device="cpu", blaslt=True)


class _Eng(EngineBase):
    def __init__(self, layers):
        self.steps = [Step("conv", f"l{i}", lay, "a", "b") for i, lay in enumerate(layers)]
        self.programs = {}


def test_tuning_table_selects_blaslt_only_where_built():
    eng = _Eng([_lin(), _lin(blaslt=False)])
    eng.apply_tuning({"l0": [0, BLT_BASE + 2], "l1": [0, BLT_BASE + 2]})
    assert eng.steps[0].layer.cfg == BLT_BASE + 2
    assert not is_blaslt(eng.steps[1].layer.cfg)          # refused: no unpacked weights on that layer
    assert eng.tuning()["l0"] == [0, BLT_BASE + 2]


def test_splitk_ids_variants_and_tuning():
    from kdl.ops.conv import MODE_CONV, is_splitk, splitk_id, splitk_parts
    g = torch.Generator().manual_seed(2)
    lay = ConvGemmLayer("c2", MODE_CONV, torch.randn(256, 9 * 256, generator=g, dtype=torch.float64),
                        torch.randn(256, generator=g), cin_pad=256, n=256, device="cpu", ksplit=(2, 3))
    sk = [c for _, c in lay.variants(14) if is_splitk(c)]
    assert sk and all(splitk_parts(c)[0] in (2, 3) and cfg_tile(c)[0] <= 160 for c in sk)
    assert splitk_parts(splitk_id(3, 16)) == (3, 16) and not is_blaslt(splitk_id(3, 16))
    plain = _lin()                                             # built without ksplit: refused
    eng = _Eng([lay, plain])
    eng.apply_tuning({"l0": [0, sk[0]], "l1": [0, splitk_id(2, 16)]})
    assert eng.steps[0].layer.cfg == sk[0] and not is_splitk(eng.steps[1].layer.cfg)
