"""Stage-pipelining buffer versioning (kdl/engine/stages.py) on CPU: which buffers
cross a cut, which get stage-private copies, which stage waits for which, and the
write-pointer split of residual GEMMs. Uses synthetic step lists and the real
Xception / ResNet-50 / ViT-B/16 / EfficientNet-B7 lowerings (built on CPU, no
launches); the GPU tests check the pipelined logits against the plain engines."""
import pytest
import torch

from kdl.engine.base import Step
from kdl.engine.stages import _cu_mask, plan_stages


def _analyse(steps, cut, scratch=()):
    return plan_stages(steps, cut, scratch)


def _chain():
    # a -> b -> c (residual from a) -> d ; "t" is reused by both halves
    return [Step("conv", "s0", src="input", dst="a"),
            Step("conv", "s1", src="a", dst="t"),
            Step("conv", "s2", src="t", dst="b"),
            Step("conv", "s3", src="b", dst="c", res="a"),
            Step("conv", "s4", src="c", dst="t"),
            Step("conv", "s5", src="t", dst="logits")]


def test_crossing_versions_are_parity_double_buffered():
    sp = _analyse(_chain(), "s2")
    # b (cut output) and a (residual read by s3) cross the cut
    assert sp.boundary == ["a", "b"]
    assert sp.wait_for == [1, 1]
    s3 = sp.remaps[0][3], sp.remaps[1][3]
    assert s3[0]["b"] == "b#x0p0" and s3[1]["b"] == "b#x0p1"
    assert s3[0]["a"] == "a#x0p0" and s3[1]["a"] == "a#x0p1"
    # the writers of a / b (stage 0) write the parity copy
    assert sp.remaps[1][0]["a"] == "a#x0p1" and sp.remaps[1][2]["b"] == "b#x0p1"


def test_buffer_reused_by_both_stages_gets_private_copy():
    sp = _analyse(_chain(), "s2")
    assert sp.remaps[0][1]["t"] == "t"            # stage 0's version keeps the name
    assert sp.remaps[0][4]["t"] == "t#s1"         # stage 1's own copy
    assert sp.remaps[0][5]["t"] == "t#s1"
    assert sp.aliases["t#s1"] == "t"


def test_scratch_is_per_stage():
    sp = _analyse(_chain(), "s2", scratch=["__tmp"])
    assert "__tmp" not in sp.remaps[0][0]
    assert sp.remaps[0][4]["__tmp"] == "__tmp#s1"


def test_residual_gemm_writes_through_separate_pointer():
    # x is the residual stream: each layer reads x as res and writes x (res == dst)
    steps = [Step("conv", "l0", src="input", dst="x"),
             Step("conv", "l1", src="x", dst="h"),
             Step("conv", "l2", src="h", dst="x", res="x"),
             Step("conv", "l3", src="x", dst="h"),
             Step("conv", "l4", src="h", dst="x", res="x"),
             Step("fc", "head", src="x", dst="logits")]
    sp = _analyse(steps, "l2")
    m = sp.remaps[1][4]                          # first residual GEMM of stage 1
    assert m["x"] == "x#x0p1"                     # reads the crossing version
    assert m["x@w"] == "x#s1"                     # writes its stage-private copy


def test_in_place_step_modifies_the_version_it_reads():
    steps = [Step("conv", "p", src="input", dst="d"),
             Step("scale", "sc", src="d", dst="d"),
             Step("conv", "q", src="d", dst="logits")]
    for cut in ("p", "sc"):
        sp = _analyse(steps, cut)
        assert sp.boundary == ["d"]
        for par in (0, 1):                        # one physical buffer for p, sc and q
            assert sp.remaps[par][0]["d"] == sp.remaps[par][1]["d"] == sp.remaps[par][2]["d"] == f"d#x0p{par}"


def test_three_stages_wait_for_last_reader():
    steps = [Step("conv", "a", src="input", dst="a"),
             Step("conv", "b", src="a", dst="b"),
             Step("conv", "c", src="b", dst="c", res="a"),
             Step("conv", "d", src="c", dst="logits")]
    sp = _analyse(steps, "a,b")
    # a is written in stage 0 and last read in stage 2: stage 0 waits on stage 2
    assert sp.wait_for == [2, 2, 2]
    assert len(sp.ranges) == 3


def test_cu_masks_are_disjoint_and_cover():
    a, b = _cu_mask(0, [0.6, 0.4]), _cu_mask(1, [0.6, 0.4])
    assert all((x & y) == 0 for x, y in zip(a, b))
    assert sum(bin(x).count("1") for x in a + b) == 256


def _xception_engine(fused=()):
    from kdl.engine import xception as XE
    from kdl.models import xception as X

    class Fake(XE.XceptionEngine):
        def __init__(self, p):
            self.device = torch.device("cpu")
            self.max_batch, self.buckets, self.steps, self.in_kind = 1, [1], [], "u8"
            self.head, self.size, self.shapes, self._remap = X.DEFAULT_HEAD, X.INPUT_SIZE, {}, {}
            self.fused_blocks = {b: None for b in fused}

    p = X.init_params(seed=0)
    e = Fake(p)
    e._build(p)
    return e


def _xception_steps():
    return _xception_engine().steps


def test_xception_default_cut_boundaries():
    from kdl.engine import registry
    cut = registry.get("xception").stage_cut
    sp = _analyse(_xception_steps(), cut, scratch=["__dwtmp"])
    # the cut is after middle block 8 (its sepconv3 adds the residual in its epilogue): one
    # boundary buffer, the block output
    assert sp.boundary == ["block8_sepconv3_out"]
    assert sp.wait_for == [1, 1]


def test_resnet_cut_inside_stage_privatises_shared_buffers():
    from kdl.engine.resnet import ResNetEngine
    from kdl.models import resnet as R

    class FR(ResNetEngine):
        def __init__(self, p):
            self.device = torch.device("cpu")
            self.max_batch, self.steps, self.size, self.classes, self.shapes = 1, [], R.INPUT_SIZE, 1000, {}
            self.in_kind, self.dtype, self.dt, self._remap = "u8", torch.float16, 1, {}

    p = R.init_params(seed=0)
    e = FR(p)
    e._build(p)
    from kdl.engine import registry
    sp = _analyse(e.steps, "layer3.1.conv3")
    assert len(sp.boundary) == 1
    # layer3's pad / mid buffers are used on both sides of a layer3.1 cut
    assert "pad14_256#s1" in sp.aliases and "mid14_256#s1" in sp.aliases
    # the default: three stages (cuts after layer2.1 and layer3.3), two parity-buffered boundaries
    sp3 = _analyse(e.steps, registry.get("resnet50").stage_cut)
    assert len(sp3.ranges) == 3 and sorted(sp3.boundary) == ["out14x1024_1", "out28x512_1"]


def test_xception_fused_entry_block_lowering():
    """KDL_ENTRY_BLOCK: block2's residual conv, both separable convs and the pool become ONE
    'block' step reading the block input and writing the block output; the stage cut analysis
    is unchanged (the cut is in the middle flow)."""
    from kdl.engine import registry
    base = _xception_engine()
    e = _xception_engine(fused=[2])
    names = [s.name for s in e.steps]
    assert "block2" in names and not {"conv2d", "block2_sepconv1", "block2_sepconv2", "block2_pool"} & set(names)
    st = e.steps[names.index("block2")]
    assert st.kind == "block" and st.src == "stem2" and st.dst == "block2_out" and st.geom == (147, 147, 74, 74)
    assert len(e.steps) == len(base.steps) - 3
    assert e.shapes["block2_out"] == base.shapes["block2_out"]
    sp = _analyse(e.steps, registry.get("xception").stage_cut, scratch=["__dwtmp"])
    assert sp.boundary == ["block8_sepconv3_out"]


def test_entry_block_plan_covers_every_row_once():
    from kdl.ops.entry_block import OUT, WARM_Y1, WARM_Y2, plan_steps
    for B, grid in ((2, 7), (32, 256), (1, 1), (3, 1000)):
        steps, off = plan_steps(B, 74, 74, 15, grid)
        assert off[0] == 0 and off[-1] == len(steps) and all(a <= b for a, b in zip(off, off[1:]))
        outs = [(b, s, k) for b, s, k, m in steps if m == OUT]
        assert sorted(outs) == [(b, s, k) for b in range(B) for s in range(5) for k in range(74)]
        per_wg = [sum(1 for st in steps[off[g]:off[g + 1]] if st[3] == OUT) for g in range(len(off) - 1)]
        assert max(per_wg) - min(per_wg) <= 1                      # balanced
        for g in range(len(off) - 1):                              # every run starts with its warm-ups
            run = steps[off[g]:off[g + 1]]
            for i, (b, s, k, m) in enumerate(run):
                if m == OUT and (i < 2 or run[i - 1][:2] != (b, s) or run[i - 1][3] == WARM_Y1):
                    raise AssertionError((g, i))
                if m == WARM_Y1:
                    assert run[i + 1] == (b, s, k + 1, WARM_Y2) and run[i + 2][2:] == (k + 2, OUT)
