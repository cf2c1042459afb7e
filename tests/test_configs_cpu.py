"""Tile-config tables (kdl.ops.conv): what each layer kind may be autotuned over."""
import pytest

from kdl.ops.conv import (C3_BASE, CONFIGS, MODE_CONV, MODE_DW, MODE_PW, S2D_BASE, S2DP, S2DW, SEP_BASE,
                          candidate_configs, cfg_tile, config_applicable, s2dp_smem)


@pytest.mark.parametrize("n", [8, 16, 32, 48, 64, 100, 128, 256, 728, 1024, 2048])
@pytest.mark.parametrize("mode", [MODE_PW, MODE_CONV, MODE_DW])
def test_candidates_valid_for_mode(n, mode):
    c = candidate_configs(n, mode=mode)
    assert c, "every layer needs at least one config"
    assert any(x < SEP_BASE for x in c), "a plain GEMM / split path is always available"
    if mode == MODE_PW:
        assert all(x < SEP_BASE for x in c), "fused separable configs are MODE_DW only"
    if mode == MODE_CONV:
        assert all(x < SEP_BASE or x >= C3_BASE for x in c), "only the 2-D tiled 3x3 conv joins MODE_CONV"
    if mode == MODE_DW:
        assert not any(x >= C3_BASE for x in c)


def test_conv3x3_2d_applicability():
    c3 = [c for c in CONFIGS if c >= C3_BASE]
    assert c3 and all(cfg_tile(c) == (cfg_tile(c)[0], 64) for c in c3)
    # Xception block1_conv2: cin 32 (K = 288), 64 outputs
    assert all(config_applicable(c, 149, 288, 64) for c in c3)
    assert not any(config_applicable(c, 149, 576, 64) for c in c3)      # cin 64: weights exceed registers
    assert not any(config_applicable(c, 149, 288, 128) for c in c3)     # more outputs than one N tile


def test_2d_configs_tile_shapes():
    # sepconv_2d: M tile = TH x TW pixels with TW a multiple of 16
    for cfg in range(S2D_BASE, S2D_BASE + 40):
        if cfg in CONFIGS:
            bm, bn = cfg_tile(cfg)
            assert bm % 16 == 0 and bn % 16 == 0


def test_persistent_lds_budget():
    # the persistent 2-D variant keeps all K x N weights in LDS: K=128 fits, K=736 never does
    for cfg in S2DP:
        assert not config_applicable(cfg, 147, 736, cfg_tile(cfg)[1])
    assert any(config_applicable(cfg, 147, 128, 128) for cfg in S2DP)
    assert all(s2dp_smem(cfg, 64) < s2dp_smem(cfg, 128) for cfg in S2DP)
    # too narrow a map for 16-pixel tile rows
    assert not any(config_applicable(cfg, 37, 128, 128) for cfg in S2DP)
    # the DMA-wave variant keeps no C tile / bias in LDS: strictly smaller than its 2dp twin
    assert s2dp_smem(201, 128) < s2dp_smem(187, 128)
    assert all(config_applicable(cfg, 147, 128, cfg_tile(cfg)[1]) for cfg in S2DW)
    assert not any(config_applicable(cfg, 147, 736, cfg_tile(cfg)[1]) for cfg in S2DW)


def test_lanes_hw_queue_budget(monkeypatch):
    """GPU_MAX_HW_QUEUES parsing used by the lanes diagnostics (profiles/lanes4_vs2.txt)."""
    from kdl.engine.lanes import hw_queues

    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    assert hw_queues() == 4
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "8")
    assert hw_queues() == 8
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "junk")
    assert hw_queues() == 4


@pytest.mark.parametrize("B", [1, 32, 85, 96, 128, 256])
def test_entry_block_plan_fits_the_lds_step_table_at_any_bucket(B):
    """one wave of workgroups overflowed EB_MAX_STEPS above ~85 images; the
    default plan adds whole waves until every workgroup's step table fits."""
    from kdl.ops.entry_block import MAX_STEPS, OUT, fit_plan
    for OH, pc in ((74, 15), (74, 13), (37, 13)):
        steps, off = fit_plan(B, OH, OH, pc, 256)
        assert max(b - a for a, b in zip(off, off[1:])) <= MAX_STEPS
        # every (image, strip, pooled row) output item exactly once
        outs = sorted((b, s, p) for b, s, p, m in steps if m == OUT)
        ns = (OH + pc - 1) // pc
        assert outs == [(b, s, p) for b in range(B) for s in range(ns) for p in range(OH)]
