"""Split-K LDS-DMA GEMM (gemm_pipe.hip ConvGemmArgs.ksplit): fp32 partials per split, the last
split of a tile to arrive sums them and runs the epilogue, per-tile counters reset themselves.
Against fp32 torch at ResNet-50 layer3/4 shapes, eager and over repeated hipGraph replays."""
import pytest
import torch
import torch.nn.functional as F

from kdl.ops import _lib
from kdl.ops.conv import MODE_CONV, MODE_PW, ConvGemmLayer, Geometry, splitk_id

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a.float().cpu() - b.float().cpu()).abs().max() / b.float().abs().max()).item()


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("H,C,stride", [(7, 512, 1), (14, 256, 1), (14, 256, 2)])
def test_splitk_3x3_matches_fp32(H, C, stride, dt):
    gen = torch.Generator().manual_seed(H + C + stride)
    B, N = 8, C
    t = torch.randn(B, H, H, C, generator=gen).to(dt)
    w2 = torch.randn(N, 3, 3, C, generator=gen, dtype=torch.float64) / (9 * C) ** 0.5
    b2 = torch.randn(N, generator=gen) * 0.1
    lay = ConvGemmLayer("c2", MODE_CONV, w2.reshape(N, 9 * C), b2, cin_pad=C, n=N, stride=stride, relu_out=1,
                        device=DEV, dtype=dt, ksplit=(2, 3, 4))
    tpad = torch.zeros(B, H + 2, H + 2, C, dtype=dt)
    tpad[:, 1:-1, 1:-1] = t
    tpad = tpad.to(DEV).contiguous()
    OH = (H + 2 - 3) // stride + 1
    ref = torch.relu(F.conv2d(t.float().permute(0, 3, 1, 2), w2.float().permute(0, 3, 1, 2), b2, stride=stride,
                              padding=1)).permute(0, 2, 3, 1)
    ids = [c for _, c in lay.variants(H) if c >= 2000]
    assert len(ids) >= 6, ids
    for cfg in ids[:: max(1, len(ids) // 8)]:
        y = torch.zeros(B * OH * OH * N, dtype=dt, device=DEV)
        for _ in range(3):                   # counters must be back at 0 after every launch
            y.zero_()
            lay.launch(tpad, y, Geometry(B, H + 2, H + 2, OH, OH), cfg=cfg)
            torch.cuda.synchronize()
            assert _rel(y.cpu().view(B, OH, OH, N), ref) < 2e-2, cfg


def test_splitk_residual_epilogue_in_captured_graph():
    """ResNet layer4 conv3 (K 512 -> N 2048, ReLU after the residual) replayed from a hipGraph."""
    gen = torch.Generator().manual_seed(9)
    B, H, C, N = 32, 7, 512, 2048
    dt = torch.float16
    x = torch.randn(B * H * H, C, generator=gen).to(dt).to(DEV)
    r = torch.randn(B * H * H, N, generator=gen).to(dt).to(DEV)
    w = torch.randn(N, C, generator=gen, dtype=torch.float64) / C ** 0.5
    b = torch.randn(N, generator=gen) * 0.1
    lay = ConvGemmLayer("c3", MODE_PW, w, b, cin_pad=C, n=N, relu_out=2, device=DEV, dtype=dt, ksplit=(2, 4))
    ref = torch.relu(x.float() @ lay.w_ref.to(DEV).t() + b.to(DEV) + r.float())
    y = torch.zeros(B * H * H, N, dtype=dt, device=DEV)
    prog = _lib.lib().Program()
    lay.emit(prog, x.data_ptr(), y.data_ptr(), Geometry(B, H, H, H, H), res=r.data_ptr(), cfg=splitk_id(4, 16))
    s = torch.cuda.Stream()
    prog.capture(s.cuda_stream)
    first = None
    for _ in range(5):
        y.zero_()
        torch.cuda.synchronize()
        prog.launch(s.cuda_stream)
        s.synchronize()
        assert _rel(y, ref) < 4e-3
        # the last split sums every partial in split order: replays are bit-identical
        if first is None:
            first = y.clone()
        assert torch.equal(y, first)
    assert int(lay._splitk_bufs[1].abs().sum()) == 0      # every tile's counter reset by its last split


def test_splitk_in_the_split_separable_lowering():
    """Xception block14 shapes (10x10 maps): depthwise into scratch, then the split-K GEMM with the
    residual-free BN epilogue; every split-K id the layer offers, twice (counters reset)."""
    from kdl.ops.reference import conv_gemm_ref
    from kdl.ops.conv import MODE_DW, is_splitk
    gen = torch.Generator().manual_seed(14)
    B, H, cin, n = 4, 10, 1024, 1536
    w = torch.randn(n, cin, generator=gen, dtype=torch.float64) / cin ** 0.5
    dww = torch.randn(9, cin, generator=gen) / 3
    b = torch.randn(n, generator=gen) * 0.1
    lay = ConvGemmLayer("b14", MODE_DW, w, b, cin_pad=cin, n=n, dww=dww, relu_in=True, relu_out=1,
                        device=DEV, ksplit=(2, 3, 4))
    g = Geometry(B, H, H, H, H)
    x = torch.randn(B, H, H, cin, generator=gen).to(torch.bfloat16).to(DEV).contiguous()
    ref = conv_gemm_ref(lay, x, g)
    tmp = torch.empty(B * H * H * cin, dtype=torch.bfloat16, device=DEV)
    ids = [c for split, c in lay.variants(H) if split and is_splitk(c)]
    assert ids, "no split-K variant offered"
    for cfg in ids:
        for _ in range(2):
            y = torch.zeros(g.M * lay.ldy, dtype=torch.bfloat16, device=DEV)
            lay.emit(None, x.data_ptr(), y.data_ptr(), g, tmp=tmp.data_ptr(), split=True, cfg=cfg)
            torch.cuda.synchronize()
            assert _rel(y.view(g.M, lay.ldy)[:, :n], ref.reshape(g.M, -1)[:, :n]) < 2e-2, cfg
