"""Fused Xception entry block (entry_block.hip, kdl/ops/entry_block.py) against the fp32
Keras-semantics oracle of the same block (SepConv -> ReLU -> SepConv -> 3x3/2 'same' max-pool +
BN(1x1/2 conv)), and the engine lowering (KDL_ENTRY_BLOCK) against the whole-network oracle.
Graph reference: /root/reference/guide.md:222-229 (the served Xception's I/O contract)."""
import os

import pytest
import torch
import torch.nn.functional as F

from kdl.models import xception as X
from kdl.models.layers import maxpool_same

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _block_oracle(p, x_nhwc, blk):
    """fp32 forward of entry block ``blk`` of X.SPEC on an NHWC input."""
    x = x_nhwc.float().permute(0, 3, 1, 2)
    b = X.SPEC[blk - 1]
    res = X._bn(X._conv(x, p, b.res_conv), p, b.res_conv.bn, False)
    y = x
    for op in b.main:
        y = X._bn(X._sep(torch.relu(y) if op.relu_in else y, p, op), p, op.bn, False)
        if op.relu_out:
            y = torch.relu(y)
    return (maxpool_same(y, 3, 2) + res).permute(0, 2, 3, 1)


def _layers(p, blk):
    from kdl.engine.xception import XceptionEngine as XE
    b = X.SPEC[blk - 1]
    return XE._sep(p, b.main[0], DEV), XE._sep(p, b.main[1], DEV), XE._pw(p, b.res_conv, DEV)


GEOM = {2: (147, 64, 74, 128), 3: (74, 128, 37, 256)}


# (block, batch, grid): grids small enough that workgroups run many pooled rows, but whose step
# lists still fit the kernel's LDS step table (EB_MAX_STEPS)
CASES = [(2, 2, None), (2, 2, 9), (2, 3, 97), (2, 1, 8), (3, 2, None), (3, 3, 7), (3, 1, 1)]
# kernel configs per block (entry_block.hip KDL_EB_CONFIGS): VALU / MFMA depthwise, 1 or 2 WGs per CU
# 13 / 15: block2 warp-specialized, 16 waves (8 consumers + 8 producers; 15: the consumers also run one dw2 unit each)
BLOCK_CFGS = {2: [0, 2, 4, 5, 13, 15], 3: [1]}


@pytest.mark.parametrize("blk,B,grid,cfg", [c + (g,) for c in CASES for g in BLOCK_CFGS[c[0]]])
def test_entry_block_matches_oracle(xparams, blk, B, grid, cfg):
    """block2: 147 -> 74 (pool pad 1 on both sides); block3: 74 -> 37 (the asymmetric TF pad: 0
    before, 1 after) with a ReLU on the block input before its first separable conv."""
    from kdl.ops.entry_block import EntryBlock
    H, C0, OH, C1 = GEOM[blk]
    s1, s2, r = _layers(xparams, blk)
    eb = EntryBlock(f"block{blk}", s1, s2, r, device=DEV, grid=grid, cfg=cfg)
    gen = torch.Generator().manual_seed(21 + B + blk)
    # block2 input: block1_conv2 output (post-ReLU); block3 input: block2 output (signed)
    x = torch.randn(B, H, H, C0, generator=gen)
    x = (torch.relu(x) if blk == 2 else x).to(torch.bfloat16)
    ref = _block_oracle(xparams, x.float(), blk)
    y = torch.full((B, OH, OH, C1), float("nan"), dtype=torch.bfloat16, device=DEV)
    eb.emit(None, x.to(DEV).data_ptr(), y.data_ptr(), B, H, H)
    torch.cuda.synchronize()
    got = y.float().cpu()
    assert torch.isfinite(got).all()
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    print(f"entry block{blk} B={B} grid={grid} cfg {cfg}: rel max err {err:.2e}")
    assert err < 2e-2, err


@pytest.mark.parametrize("B,cfg", [(96, 2), (128, 2), (128, 0), (128, 13), (128, 15)])
def test_entry_block2_large_bucket_runs_in_two_waves(xparams, B, cfg):
    """batch >= ~85 overflowed a one-wave plan's step table (EB_MAX_STEPS); the default
    plan now adds whole waves of workgroups. The fp32 oracle runs on the GPU at this size."""
    from kdl.ops.entry_block import EntryBlock
    H, C0, OH, C1 = GEOM[2]
    s1, s2, r = _layers(xparams, 2)
    eb = EntryBlock("block2", s1, s2, r, device=DEV, cfg=cfg)
    _, _, grid = eb.plan(B, OH, OH)
    assert grid > torch.cuda.get_device_properties(0).multi_processor_count
    gen = torch.Generator().manual_seed(5)
    x = torch.relu(torch.randn(B, H, H, C0, generator=gen)).to(torch.bfloat16).to(DEV)
    pg = {k: v.to(DEV) for k, v in xparams.items()}
    ref = _block_oracle(pg, x.float(), 2)
    y = torch.full((B, OH, OH, C1), float("nan"), dtype=torch.bfloat16, device=DEV)
    eb.emit(None, x.data_ptr(), y.data_ptr(), B, H, H)
    torch.cuda.synchronize()
    got = y.float()
    assert torch.isfinite(got).all()
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    print(f"entry block2 B={B} grid={grid}: rel max err {err:.2e}")
    assert err < 2e-2, err


def test_entry_block_refuses_a_step_table_over_the_lds_limit(xparams):
    from kdl.ops.entry_block import EntryBlock
    s1, s2, r = _layers(xparams, 2)
    eb = EntryBlock("block2", s1, s2, r, device=DEV, grid=1)
    with pytest.raises(AssertionError, match="EB_MAX_STEPS"):
        eb.plan(2, 74, 74)


@pytest.mark.parametrize("cfg", [0, 2, 13, 15])
def test_entry_block2_replays_bit_identical(xparams, cfg):
    """Persistent kernel, host step table: two launches give identical bytes (an LDS / DMA ordering
    bug would show as run-to-run noise; VALU and MFMA depthwise configs)."""
    from kdl.ops.entry_block import EntryBlock
    s1, s2, r = _layers(xparams, 2)
    eb = EntryBlock("block2", s1, s2, r, device=DEV, cfg=cfg)
    gen = torch.Generator().manual_seed(5)
    x = torch.relu(torch.randn(4, 147, 147, 64, generator=gen)).to(torch.bfloat16).to(DEV)
    y1 = torch.empty((4, 74, 74, 128), dtype=torch.bfloat16, device=DEV)
    y2 = torch.empty_like(y1)
    eb.emit(None, x.data_ptr(), y1.data_ptr(), 4, 147, 147)
    eb.emit(None, x.data_ptr(), y2.data_ptr(), 4, 147, 147)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)


def test_engine_with_fused_block2_matches_oracle(xparams):
    from kdl.engine.xception import XceptionEngine
    old = os.environ.get("KDL_ENTRY_BLOCK")
    os.environ["KDL_ENTRY_BLOCK"] = "2,3"
    try:
        eng = XceptionEngine(xparams, max_batch=4, buckets=[1, 4])
    finally:
        if old is None:
            os.environ.pop("KDL_ENTRY_BLOCK")
        else:
            os.environ["KDL_ENTRY_BLOCK"] = old
    assert [s.name for s in eng.steps if s.kind == "block"] == ["block2", "block3"]
    gen = torch.Generator().manual_seed(11)
    img = torch.randint(0, 256, (3, 299, 299, 3), generator=gen, dtype=torch.uint8)
    ref = X.xception_forward(xparams, img.float() / 127.5 - 1.0)
    out = eng.forward(img.cuda()).cpu()
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    print(f"engine with fused block2 + block3: logits rel err {err:.2e}")
    assert err < 0.05, (out, ref)
    assert torch.equal(eng.forward(img.cuda(), capture=True).cpu(), eng.forward(img.cuda(), capture=False).cpu())
