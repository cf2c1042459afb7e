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
