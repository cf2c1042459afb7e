"""End-to-end Xception on the MI355X engine vs the fp32 Keras-semantics oracle."""
import pytest
import torch

from kdl.models import xception as X

pytestmark = pytest.mark.gpu


def _logit_err(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


@pytest.fixture(scope="module")
def engine(xparams):
    from kdl.engine.xception import XceptionEngine
    return XceptionEngine(xparams, max_batch=4, buckets=[1, 2, 4])


def test_engine_matches_oracle_u8(engine, xparams):
    gen = torch.Generator().manual_seed(11)
    img = torch.randint(0, 256, (3, 299, 299, 3), generator=gen, dtype=torch.uint8)
    ref = X.xception_forward(xparams, img.float() / 127.5 - 1.0)
    out = engine.forward(img.cuda()).cpu()
    torch.cuda.synchronize()
    assert out.shape == (3, 10)
    assert _logit_err(out, ref) < 0.05, (out, ref)


def test_engine_f32_compat_path(xparams):
    from kdl.engine.xception import XceptionEngine
    eng = XceptionEngine(xparams, max_batch=2, in_kind="f32")
    gen = torch.Generator().manual_seed(12)
    x = torch.rand((2, 299, 299, 3), generator=gen) * 2 - 1
    ref = X.xception_forward(xparams, x)
    out = eng.forward(x.cuda()).cpu()
    assert _logit_err(out, ref) < 0.05, (out, ref)


def test_graph_replay_equals_eager(engine):
    gen = torch.Generator().manual_seed(13)
    img = torch.randint(0, 256, (4, 299, 299, 3), generator=gen, dtype=torch.uint8).cuda()
    a = engine.forward(img, capture=True)
    b = engine.forward(img, capture=False)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_bucket_padding_rows_do_not_leak(engine):
    """A 3-image request runs in the 4-bucket; results must not depend on row 4."""
    gen = torch.Generator().manual_seed(14)
    img = torch.randint(0, 256, (4, 299, 299, 3), generator=gen, dtype=torch.uint8).cuda()
    a = engine.forward(img[:3])
    img2 = img.clone()
    img2[3] = 255 - img2[3]
    engine.forward(img2)
    b = engine.forward(img[:3])
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_lane_group_matches_single_engine(xparams):
    """Split-batch lanes (kdl/engine/lanes.py): two batch-2 graphs on two streams over
    row views of one batch-4 slot give the single batch-4 engine's logits."""
    from kdl.engine import registry
    from kdl.engine.lanes import LaneGroup
    from kdl.engine.xception import XceptionEngine
    dev = torch.device("cuda", 0)
    single = XceptionEngine(xparams, max_batch=4)
    lanes = LaneGroup(registry.get("xception"), xparams, 4, dev, 2)
    lanes.apply_tuning(single.tuning())
    slots = lanes.add_input_slots(2)
    gen = torch.Generator().manual_seed(13)
    img = torch.randint(0, 256, (4, 299, 299, 3), generator=gen, dtype=torch.uint8)
    ref = single.forward(img.cuda()).cpu()
    slots[1].copy_(img.cuda())
    torch.cuda.synchronize()
    lanes.launch(4, lanes.stream, slot=1)
    lanes.stream.synchronize()
    out = lanes.slot_logits(1).cpu()
    assert torch.allclose(out, ref, rtol=1e-3, atol=1e-3), (out, ref)
    assert lanes.slot_logits(0).abs().sum().item() == 0.0   # slot 0 untouched


@pytest.mark.parametrize("cut", ["block4_pool", "block7_sepconv1", "block3,block8_sepconv2"])
def test_stage_pipe_matches_single_engine(xparams, cut):
    """Stage pipelining (kdl/engine/stages.py): four batches in flight on two slots,
    stage 1 of batch i+1 overlapping stage 2 of batch i with parity-double-buffered
    boundary buffers (a mid-block cut also double-buffers the block's residual input)
    and per-stage depthwise scratch (split separable convs in both stages), reproduce
    the plain engine's logits batch for batch."""
    from kdl.engine.stages import StagePipe
    from kdl.engine.xception import XceptionEngine
    single = XceptionEngine(xparams, max_batch=4)
    table = single.tuning()
    for name in ("block4_sepconv1", "block13_sepconv2"):    # split lowering in each stage
        table[name] = [1, table[name][1] if table[name][1] < 64 else 16]
    single.apply_tuning(table)
    assert single.tuning()["block4_sepconv1"][0] == 1 and single.tuning()["block13_sepconv2"][0] == 1
    pipe = StagePipe(XceptionEngine(xparams, max_batch=4), cut)
    pipe.apply_tuning(table)
    slots = pipe.add_input_slots(2)
    gen = torch.Generator().manual_seed(21)
    imgs = [torch.randint(0, 256, (4, 299, 299, 3), generator=gen, dtype=torch.uint8) for _ in range(4)]
    refs = [single.forward(x.cuda()).cpu() for x in imgs]
    outs = []
    done = [torch.cuda.Event() for _ in range(2)]
    for i, x in enumerate(imgs):
        j = i % 2
        if i >= 2:                                  # slot j free again: batch i-2 finished
            done[j].synchronize()
            outs.append(pipe.slot_logits(j).cpu())
        slots[j].copy_(x.cuda())                   # current stream; no device-wide sync, so
        ready = torch.cuda.Event()                 # the stages of consecutive batches overlap
        ready.record()
        pipe.launch_async(4, [ready], [done[j]], slot=j)
    for i in (2, 3):
        done[i % 2].synchronize()
        outs.append(pipe.slot_logits(i % 2).cpu())
    for o, r in zip(outs, refs):
        assert torch.allclose(o, r, rtol=1e-3, atol=1e-3), (o, r)
