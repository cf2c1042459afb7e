"""Numerics of every HIP kernel against fp32 torch references (run on MI355X).

Shapes cover the awkward cases from SURVEY.md §2.5: ragged M (19x19xB), the
N=K=728 tails (padded to 736), stride-2 residual convs, the asymmetric TF pool
pad at 74->37, and every autotuner tile config.
"""
import pytest
import torch

from kdl.ops import _lib
from kdl.ops.conv import MODE_CONV, MODE_DW, MODE_PW, ConvGemmLayer, Geometry, cfg_tile
from kdl.ops.pack import round_up
from kdl.ops.reference import conv_gemm_ref, head_ref, pool_add_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rand_act(shape, ldc, c, gen):
    x = torch.zeros(*shape, ldc)
    x[..., :c] = torch.randn(*shape, c, generator=gen)
    return x.to(torch.bfloat16).to(DEV).contiguous()


def _layer(mode, cin, n, gen, stride=1, relu_in=False, relu_out=False):
    cin_pad = round_up(cin, 32)
    k = 9 * cin_pad if mode == MODE_CONV else cin_pad
    w = torch.zeros(n, k, dtype=torch.float64)
    if mode == MODE_CONV:
        w3 = torch.randn(n, 9, cin, generator=gen, dtype=torch.float64) / (9 * cin) ** 0.5
        w.view(n, 9, cin_pad)[:, :, :cin] = w3
    else:
        w[:, :cin] = torch.randn(n, cin, generator=gen, dtype=torch.float64) / cin ** 0.5
    bias = torch.randn(n, generator=gen) * 0.1
    dww = None
    if mode == MODE_DW:
        dww = torch.zeros(9, cin_pad)
        dww[:, :cin] = torch.randn(9, cin, generator=gen) / 3
    return ConvGemmLayer("t", mode, w, bias, cin_pad=cin_pad, n=n, stride=stride, dww=dww,
                         relu_in=relu_in, relu_out=relu_out, device=DEV)


def _check(y, ref, n, tol=2e-2):
    yf = y.float().view(ref.shape)
    err = (yf - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err <= tol * scale, f"max err {err} vs scale {scale}"
    # padded output channels must stay exactly zero
    if yf.shape[1] > n:
        assert yf[:, n:].abs().max().item() == 0.0


@pytest.mark.parametrize("cin,n,H,stride", [(64, 128, 37, 2), (728, 1024, 19, 2), (256, 728, 37, 2),
                                            (128, 256, 10, 1)])
def test_conv_gemm_pointwise(cin, n, H, stride):
    gen = torch.Generator().manual_seed(1)
    lay = _layer(MODE_PW, cin, n, gen, stride=stride)
    B = 3
    OH = (H - 1) // stride + 1
    g = Geometry(B, H, H, OH, OH)
    x = _rand_act((B, H, H), lay.cin_pad, cin, gen)
    ref = conv_gemm_ref(lay, x, g)
    for _, cfg in lay.variants(H):
        y = torch.full((g.M * lay.ldy,), float("nan"), dtype=torch.bfloat16, device=DEV)
        lay.launch(x, y, g, cfg=cfg)
        torch.cuda.synchronize()
        _check(y, ref, n)


@pytest.mark.parametrize("mode,cin,n,H", [(MODE_PW, 736, 736, 19), (MODE_PW, 768, 3072, 14), (MODE_CONV, 64, 64, 30)])
def test_gemm_pipe_k_rotation(mode, cin, n, H):
    """K-rotated LDS-DMA GEMM (ConvGemmArgs.krot: each M tile starts its K loop at its own
    step) against the fp32 reference on every pipelined config, incl. KSUB > 1 tails."""
    from kdl.ops.conv import PIPE_BASE, SEP_BASE
    gen = torch.Generator().manual_seed(12)
    lay = _layer(mode, cin, n, gen, relu_out=True)
    lay.krot = 1
    B = 3
    OH = H - 2 if mode == MODE_CONV else H
    g = Geometry(B, H, H, OH, OH)
    x = _rand_act((B, H, H), lay.cin_pad, cin, gen)
    ref = conv_gemm_ref(lay, x, g)
    cfgs = [c for _, c in lay.variants(H) if PIPE_BASE <= c < SEP_BASE]
    assert cfgs
    for cfg in cfgs:
        y = torch.full((g.M * lay.ldy,), float("nan"), dtype=torch.bfloat16, device=DEV)
        lay.launch(x, y, g, cfg=cfg)
        torch.cuda.synchronize()
        try:
            _check(y, ref, n)
        except AssertionError as e:
            raise AssertionError(f"cfg={cfg}: {e}") from None


def test_conv_gemm_conv3x3():
    gen = torch.Generator().manual_seed(2)
    lay = _layer(MODE_CONV, 32, 64, gen, relu_out=True)
    B, H = 2, 23
    g = Geometry(B, H, H, H - 2, H - 2)
    x = _rand_act((B, H, H), 32, 32, gen)
    ref = conv_gemm_ref(lay, x, g)
    for _, cfg in lay.variants(H):
        y = torch.zeros(g.M * lay.ldy, dtype=torch.bfloat16, device=DEV)
        lay.launch(x, y, g, cfg=cfg)
        torch.cuda.synchronize()
        _check(y, ref, 64)


@pytest.mark.parametrize("cin,n,H,relu_in,relu_out,with_res", [
    (728, 728, 19, True, True, False),
    (728, 728, 19, False, False, True),
    (64, 128, 29, False, True, False),
    (256, 728, 37, True, True, False),
    (1024, 1536, 10, False, True, False),
    # 2-D spatial tiles (sepconv_2d.hip): partial tiles at both edges, with/without pre-ReLU
    (64, 128, 74, False, True, False),
    (128, 128, 67, True, False, True),
    (256, 256, 70, True, True, False),
    # the headline's 147x147 block2 layers (bench table: sepconv_2dp / sepconv_2dw ids 185 / 204)
    (64, 128, 147, False, True, False),
    (128, 128, 147, True, False, False),
])
def test_conv_gemm_separable(cin, n, H, relu_in, relu_out, with_res):
    gen = torch.Generator().manual_seed(3)
    lay = _layer(MODE_DW, cin, n, gen, relu_in=relu_in, relu_out=relu_out)
    B = 2
    g = Geometry(B, H, H, H, H)
    x = _rand_act((B, H, H), lay.cin_pad, cin, gen)
    res = _rand_act((B, H, H), lay.ldy, n, gen) if with_res else None
    ref = conv_gemm_ref(lay, x, g, res=res)
    for split, cfg in lay.variants(H):
        y = torch.zeros(g.M * lay.ldy, dtype=torch.bfloat16, device=DEV)
        lay.launch(x, y, g, res=res, cfg=cfg, split=split)
        torch.cuda.synchronize()
        try:
            _check(y, ref, n)
        except AssertionError as e:
            raise AssertionError(f"split={split} cfg={cfg}: {e}") from None


@pytest.mark.parametrize("H,C,relu", [(19, 736, True), (37, 256, True), (74, 128, False), (10, 1024, False),
                                      (23, 96, True)])
def test_dw3x3_tiled_and_direct(H, C, relu):
    """Standalone depthwise 3x3 'same' (split separable lowering): LDS-tiled kernel (algo 1)
    and the direct row-streaming kernel (algo 2, several seg / band / prefetch shapes incl.
    partial bands and partial column segments) against torch fp32."""
    import torch.nn.functional as F
    C_ = _lib.lib()
    gen = torch.Generator().manual_seed(11)
    B = 3
    x = torch.randn(B, H, H, C, generator=gen).to(torch.bfloat16).to(DEV)
    w = (torch.randn(9, C, generator=gen) / 3).float().to(DEV).contiguous()
    xf = x.float().permute(0, 3, 1, 2)
    xf = xf.relu() if relu else xf
    ref = F.conv2d(F.pad(xf, (1, 1, 1, 1)), w.t().reshape(C, 1, 3, 3), groups=C).permute(0, 2, 3, 1)
    base = dict(x=x.data_ptr(), w=w.data_ptr(), B=B, H=H, W=H, C=C, relu_in=int(relu))
    s = torch.cuda.current_stream().cuda_stream
    for kw in [dict(algo=1), dict(algo=2), dict(algo=2, seg=2, rb=2, pd=2), dict(algo=2, seg=3, rb=5, pd=1),
               dict(algo=2, seg=4, rb=H, pd=2)]:
        y = torch.full_like(x, float("nan"))
        C_.dw3x3({**base, "y": y.data_ptr(), **kw}, s)
        torch.cuda.synchronize()
        err = (y.float() - ref).abs().max().item()
        assert err <= 1e-2 * ref.abs().max().item(), (kw, err)


def test_sepconv_2d_repeat_race_screen():
    """2-D tiled fused separable conv: run-to-run identical on an early-flow shape."""
    gen = torch.Generator().manual_seed(5)
    lay = _layer(MODE_DW, 128, 128, gen, relu_in=True, relu_out=False)
    B, H = 4, 147
    g = Geometry(B, H, H, H, H)
    x = _rand_act((B, H, H), lay.cin_pad, 128, gen)
    cfgs = [c for split, c in lay.variants(H) if not split and c >= 160]
    assert cfgs, "no 2-D tiled variant offered at 147x147"
    for cfg in cfgs:
        y0 = torch.zeros(g.M * lay.ldy, dtype=torch.bfloat16, device=DEV)
        lay.launch(x, y0, g, cfg=cfg)
        for _ in range(5):
            y = torch.zeros_like(y0)
            lay.launch(x, y, g, cfg=cfg)
            torch.cuda.synchronize()
            assert torch.equal(y, y0), f"cfg {cfg} nondeterministic"


def test_conv_gemm_repeat_race_screen():
    """Same launch many times: LDS/DMA ordering bugs show up as run-to-run diffs."""
    gen = torch.Generator().manual_seed(4)
    lay = _layer(MODE_DW, 728, 728, gen, relu_in=True, relu_out=True)
    B, H = 8, 19
    g = Geometry(B, H, H, H, H)
    x = _rand_act((B, H, H), lay.cin_pad, 728, gen)
    for split, cfg in lay.variants(H):
        y0 = torch.zeros(g.M * lay.ldy, dtype=torch.bfloat16, device=DEV)
        lay.launch(x, y0, g, cfg=cfg, split=split)
        for _ in range(10):
            y = torch.zeros_like(y0)
            lay.launch(x, y, g, cfg=cfg, split=split)
            torch.cuda.synchronize()
            assert torch.equal(y, y0), f"cfg {cfg} nondeterministic"


@pytest.mark.parametrize("in_kind", ["u8", "f32"])
def test_stem(in_kind):
    gen = torch.Generator().manual_seed(5)
    B, H = 2, 299
    OH = (H - 3) // 2 + 1
    w = torch.randn(3, 3, 3, 32, generator=gen, dtype=torch.float64) * 0.2
    bias = torch.randn(32, generator=gen, dtype=torch.float64) * 0.1
    img = torch.randint(0, 256, (B, H, H, 3), generator=gen, dtype=torch.uint8)
    xn = img.double() / 127.5 - 1.0
    ref = torch.relu(torch.nn.functional.conv2d(xn.permute(0, 3, 1, 2), w.permute(3, 2, 0, 1), stride=2)
                     + bias[None, :, None, None]).permute(0, 2, 3, 1).reshape(-1, 32).float()
    wk = w.reshape(27, 32).t()
    if in_kind == "u8":
        b2, wk, x = bias - wk.sum(1), wk / 127.5, img.to(DEV)
    else:
        b2, x = bias, xn.float().to(DEV)
    from kdl.ops.pack import pack_fragments
    wp = pack_fragments(wk, 2, 1).to(DEV)
    bb = b2.float().to(DEV)
    y = torch.zeros(B * OH * OH * 32, dtype=torch.bfloat16, device=DEV)
    _lib.lib().stem_conv(dict(x=_lib.ptr(x), wp=_lib.ptr(wp), bias=_lib.ptr(bb), y=_lib.ptr(y), B=B, H=H, W=H,
                              OH=OH, OW=OH, ldy=32, in_kind=0 if in_kind == "u8" else 1),
                         _lib.stream_ptr())
    torch.cuda.synchronize()
    err = (y.float().cpu().view(-1, 32) - ref).abs().max().item()
    assert err < 0.03 * ref.abs().max().item(), err


@pytest.mark.parametrize("H,C,with_res", [(147, 128, True), (74, 256, True), (37, 736, False), (19, 1024, True)])
def test_pool_add(H, C, with_res):
    from kdl.models.layers import tf_same_pad
    gen = torch.Generator().manual_seed(6)
    B = 2
    OH, pt, _ = tf_same_pad(H, 3, 2)
    x = torch.randn(B * H * H * C, generator=gen).to(torch.bfloat16).to(DEV)
    res = torch.randn(B * OH * OH * C, generator=gen).to(torch.bfloat16).to(DEV) if with_res else None
    y = torch.zeros(B * OH * OH * C, dtype=torch.bfloat16, device=DEV)
    _lib.lib().pool_add(dict(x=_lib.ptr(x), res=_lib.ptr(res), y=_lib.ptr(y), B=B, H=H, W=H, OH=OH, OW=OH,
                             C=C, pad_top=pt, pad_left=pt), _lib.stream_ptr())
    torch.cuda.synchronize()
    ref = pool_add_ref(x, res, B, H, H, OH, OH, C, pt)
    err = (y.float().view(-1, C) - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item(), err
    # both kernels explicitly: pixel-per-thread and row-streaming (partial bands / segments)
    for kw in [dict(algo=1), dict(algo=2), dict(algo=2, seg=1, rb=1), dict(algo=2, seg=4, rb=3),
               dict(algo=2, seg=2, rb=OH)]:
        y.fill_(float("nan"))
        _lib.lib().pool_add(dict(x=_lib.ptr(x), res=_lib.ptr(res), y=_lib.ptr(y), B=B, H=H, W=H, OH=OH, OW=OH,
                                 C=C, pad_top=pt, pad_left=pt, **kw), _lib.stream_ptr())
        torch.cuda.synchronize()
        err = (y.float().view(-1, C) - ref).abs().max().item()
        assert err <= 2e-2 * ref.abs().max().item(), (kw, err)


def test_pool_add_batch_beyond_grid_y_limit():
    """B * OH > 65535 (a server --max_batch_size of thousands): the pixel-per-thread kernel's
    grid.y cannot hold it, so the launcher takes the 1-D row-streaming grid instead of failing."""
    from kdl.models.layers import tf_same_pad
    gen = torch.Generator().manual_seed(9)
    B, H, C = 6600, 19, 8
    OH, pt, _ = tf_same_pad(H, 3, 2)
    assert B * OH > 65535
    x = torch.randn(B * H * H * C, generator=gen).to(torch.bfloat16).to(DEV)
    res = torch.randn(B * OH * OH * C, generator=gen).to(torch.bfloat16).to(DEV)
    y = torch.full((B * OH * OH * C,), float("nan"), dtype=torch.bfloat16, device=DEV)
    _lib.lib().pool_add(dict(x=_lib.ptr(x), res=_lib.ptr(res), y=_lib.ptr(y), B=B, H=H, W=H, OH=OH, OW=OH,
                             C=C, pad_top=pt, pad_left=pt, algo=1), _lib.stream_ptr())
    torch.cuda.synchronize()
    ref = pool_add_ref(x, res, B, H, H, OH, OH, C, pt)
    assert (y.float().view(-1, C) - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()


@pytest.mark.parametrize("HW,K,N", [(37 * 37, 480, 80), (19 * 19, 2304, 384), (150 * 150 // 9, 288, 48)])
def test_ascale_fold_channel_scale(HW, K, N):
    """EfficientNet SE scale on the project GEMM: the LDS-DMA GEMM scales its A operand by
    ConvGemmArgs.ascale (per image and channel, per-image M tiles) between LDS and the MFMAs;
    every pipelined tile config must equal (D * s_b) W^T."""
    from kdl.ops.conv import PIPE_BASE, SEP_BASE
    gen = torch.Generator().manual_seed(9)
    B = 3
    lay = _layer(MODE_PW, K, N, gen)
    g = Geometry(B, HW, 1, HW, 1)
    x = _rand_act((B, HW, 1), lay.cin_pad, K, gen)
    sc = (torch.rand(B, K, generator=gen) + 0.25).to(DEV)
    xs = (x.float().view(B, HW, lay.cin_pad) * sc[:, None, :]).to(torch.bfloat16).contiguous()
    ref = conv_gemm_ref(lay, xs.view(-1), g)
    kw = dict(ascale=(_lib.ptr(sc), K))
    cfgs = [c for _, c in lay.variants(1) if PIPE_BASE <= c < SEP_BASE]
    assert cfgs
    for cfg in cfgs:
        y = torch.full((g.M * lay.ldy,), float("nan"), dtype=torch.bfloat16, device=DEV)
        lay.emit(None, _lib.ptr(x), _lib.ptr(y), g, cfg=cfg, **kw)
        torch.cuda.synchronize()
        try:
            _check(y, ref, N, tol=3e-2)
        except AssertionError as e:
            raise AssertionError(f"cfg={cfg}: {e}") from None


def test_ascale_refused_off_the_pipelined_gemms():
    """A-operand scales on a kernel that would ignore them (the register-B GEMM) fail loudly."""
    gen = torch.Generator().manual_seed(3)
    lay = _layer(MODE_PW, 64, 64, gen)
    g = Geometry(2, 64, 1, 64, 1)
    x = _rand_act((2, 64, 1), lay.cin_pad, 64, gen)
    y = torch.zeros(g.M * lay.ldy, dtype=torch.bfloat16, device=DEV)
    sc = torch.ones(2, 64, device=DEV)
    lay.emit(None, _lib.ptr(x), _lib.ptr(y), g, cfg=0)          # the same launch without scales runs
    torch.cuda.synchronize()
    with pytest.raises(AssertionError):
        lay.emit(None, _lib.ptr(x), _lib.ptr(y), g, cfg=0, ascale=(_lib.ptr(sc), 64))
    ga = lay.args(_lib.ptr(x), _lib.ptr(y), g, None, cfg=0)
    ga.update(ascale=_lib.ptr(sc), ascale_ld=64)
    with pytest.raises(RuntimeError):
        _lib.lib().conv_gemm(MODE_PW, 0, ga, _lib.stream_ptr())


# (K, n) of every streaming-GEMM instance (EfficientNet-B7's large-map expand / project convs)
STREAM_KN = [(32, 32), (64, 32), (32, 192), (192, 48), (64, 288), (288, 48), (288, 80), (96, 480), (480, 80)]


@pytest.mark.parametrize("K,N", STREAM_KN)
@pytest.mark.parametrize("kind", ["silu", "ascale_res"])
@pytest.mark.parametrize("nt", [False, True])
def test_gemm_stream(K, N, kind, nt):
    """Streaming pointwise GEMM (gemm_stream.hip, id STREAM_BASE) against the fp32 reference: the
    expand form (SiLU epilogue) and the project form (per-image SE scales on the A operand,
    residual add), on a ragged 37x37 map (partial 16-row fragments, images crossing workgroups);
    both the plain and the nontemporal-store ids."""
    from kdl.ops.conv import STREAM_BASE, STREAM_NT
    cfg = STREAM_NT if nt else STREAM_BASE
    gen = torch.Generator().manual_seed(K * 7 + N)
    B, H = 3, 37
    lay = _layer(MODE_PW, K, N, gen)
    assert lay.stream_ok() and (False, cfg) in lay.variants(H)
    g = Geometry(B, H, H, H, H)
    x = _rand_act((B, H, H), lay.cin_pad, K, gen)
    y = torch.full((g.M * lay.ldy,), float("nan"), dtype=torch.bfloat16, device=DEV)
    if kind == "silu":
        ref = conv_gemm_ref(lay, x, g)
        ref[:, :N] = torch.nn.functional.silu(ref[:, :N])
        lay.relu_out = 4
        lay.launch(x, y, g, cfg=cfg)
    else:
        # (residual instances stop at ldy 288: wider ones are refused, and the engine never offers them)
        res = _rand_act((B, H, H), lay.ldy, N, gen) if lay.stream_ok(res=True) else None
        sc = (torch.rand(B, K, generator=gen) + 0.25).to(DEV)
        xs = (x.float().view(B, H * H, lay.cin_pad) * sc[:, None, :]).to(torch.bfloat16).contiguous()
        ref = conv_gemm_ref(lay, xs.view(-1), g, res=res)
        kw = dict(ascale=(_lib.ptr(sc), K))
        lay.emit(None, _lib.ptr(x), _lib.ptr(y), g, res=_lib.ptr(res) if res is not None else None, cfg=cfg,
                 **kw)
    torch.cuda.synchronize()
    _check(y, ref, N, tol=3e-2)


@pytest.mark.parametrize("K,N", [(32, 32), (288, 80)])
def test_gemm_stream_persistent(K, N):
    """300x300 maps: more 16-row fragments than the persistent grid's waves, so every wave walks
    several fragments through its register ring (and the per-CU LDS budget sets the grid)."""
    from kdl.ops.conv import STREAM_BASE
    gen = torch.Generator().manual_seed(K + N)
    B, H = 3 if K == 32 else 2, 300
    lay = _layer(MODE_PW, K, N, gen)
    g = Geometry(B, H, H, H, H)
    x = _rand_act((B, H, H), lay.cin_pad, K, gen)
    ref = conv_gemm_ref(lay, x, g)
    ref[:, :N] = torch.nn.functional.silu(ref[:, :N])
    lay.relu_out = 4
    y = torch.full((g.M * lay.ldy,), float("nan"), dtype=torch.bfloat16, device=DEV)
    lay.launch(x, y, g, cfg=STREAM_BASE)
    torch.cuda.synchronize()
    _check(y, ref, N, tol=3e-2)


def test_gemm_stream_refuses_wide_residual():
    """Residual instances stop at ldy 288: a wider one is refused loudly, not run wrong."""
    from kdl.ops.conv import STREAM_BASE
    gen = torch.Generator().manual_seed(3)
    lay = _layer(MODE_PW, 96, 480, gen)
    g = Geometry(1, 8, 8, 8, 8)
    x = _rand_act((1, 8, 8), lay.cin_pad, 96, gen)
    res = _rand_act((1, 8, 8), lay.ldy, 480, gen)
    y = torch.zeros(g.M * lay.ldy, dtype=torch.bfloat16, device=DEV)
    assert not lay.stream_ok(res=True)
    with pytest.raises(RuntimeError):
        lay.launch(x, y, g, res=res, cfg=STREAM_BASE)
        torch.cuda.synchronize()


def test_head():
    gen = torch.Generator().manual_seed(7)
    B, HW, F_, H1, NC = 5, 100, 2048, 100, 10
    x = torch.randn(B * HW * F_, generator=gen).to(torch.bfloat16).to(DEV)
    w1 = (torch.randn(F_, H1, generator=gen) / 45).to(DEV)
    b1 = (torch.randn(H1, generator=gen) * 0.1).to(DEV)
    w2 = (torch.randn(H1, NC, generator=gen) / 10).to(DEV)
    b2 = (torch.randn(NC, generator=gen) * 0.1).to(DEV)
    out = torch.zeros(B, NC, device=DEV)
    w1t = w1.t().contiguous()
    feat = torch.zeros(B, F_, device=DEV)
    hid = torch.zeros(F_ // 64, B, H1, device=DEV)
    _lib.lib().head_dense(dict(x=_lib.ptr(x), w1=_lib.ptr(w1t), b1=_lib.ptr(b1), w2=_lib.ptr(w2),
                               b2=_lib.ptr(b2), out=_lib.ptr(out), feat=_lib.ptr(feat), hid=_lib.ptr(hid), B=B, HW=HW, ldx=F_, F=F_, H1=H1, NC=NC),
                          _lib.stream_ptr())
    torch.cuda.synchronize()
    ref = head_ref(x, B, HW, F_, F_, w1, b1, w2, b2)
    assert torch.allclose(out, ref, atol=1e-4, rtol=1e-3), (out - ref).abs().max()
