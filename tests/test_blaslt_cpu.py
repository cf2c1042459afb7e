"""No vendor GEMM in the product: the hipBLASLt node of rounds 3-4 left
kdl._C in round 5 (its source is a tools-only probe, tools/probes/blaslt). Every layer's tuning
variants are hand-written kernel ids, a table naming a retired vendor id (1000-1999) is refused
at load, no committed table carries one, and the native library links no hipBLASLt."""
import json
from pathlib import Path

import torch

from kdl.ops.conv import MODE_PW, ConvGemmLayer

ROOT = Path(__file__).resolve().parents[1]


def _lin(n=128, k=64):
    g = torch.Generator().manual_seed(0)
    return ConvGemmLayer("lin", MODE_PW, torch.randn(n, k, generator=g, dtype=torch.float64),
                         torch.randn(n, generator=g), cin_pad=k, n=n, device="cpu")


def test_variants_are_hand_written_ids_only():
    assert all(not (1000 <= c < 2000) for _, c in _lin().variants())


def test_a_table_naming_a_retired_vendor_id_is_refused():
    from kdl.engine.base import EngineBase, Step

    class E(EngineBase):
        def __init__(self):
            self.steps = [Step("conv", "lin", _lin(), "a", "b")]

        def invalidate(self):
            pass
    e = E()
    before = e.steps[0].layer.cfg
    e.apply_tuning({"lin": [0, 1003]})
    assert e.steps[0].layer.cfg == before


def test_no_committed_table_uses_a_vendor_gemm():
    for p in (ROOT / "kdl" / "tuning").glob("*.json"):
        for k, v in json.loads(p.read_text()).items():
            cfg = v if isinstance(v, int) else v[1]
            assert not (1000 <= int(cfg) < 2000), (p.name, k, cfg)


def test_native_library_sources_and_link_line_carry_no_vendor_blas():
    src = (ROOT / "kdl" / "csrc" / "build.py").read_text()
    assert "-lhipblaslt" not in src and "blaslt.cpp" not in src
    for f in (ROOT / "kdl" / "csrc").rglob("*"):
        if f.suffix in (".cpp", ".h", ".hip"):
            assert "hipblaslt" not in f.read_text().lower(), f
