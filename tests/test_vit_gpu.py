"""ViT-B/16 on MI355X: LayerNorm, flash-style MFMA attention, patchify + token
embedding, GELU GEMM epilogue against fp32 torch, then the engine vs the oracle."""
import math

import pytest
import torch
import torch.nn.functional as F

from kdl.models import vit as V
from kdl.ops import _lib
from kdl.ops.conv import MODE_PW, ConvGemmLayer, Geometry

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a.float().cpu() - b.float().cpu()).abs().max() / b.float().abs().max()).item()


@pytest.mark.parametrize("D", [768, 200, 2048])   # <= 1024: two rows per wave; 2048: one row per wave
def test_layernorm_rows_and_strided_cls_rows(D):
    gen = torch.Generator().manual_seed(0)
    B, T = 3, 197
    x = (torch.randn(B * T, D, generator=gen) * 2 + 0.5).to(torch.bfloat16).to(DEV)
    g = torch.rand(D, generator=gen).to(DEV) + 0.5
    b = torch.randn(D, generator=gen).to(DEV) * 0.1
    y = torch.zeros_like(x)
    C, s = _lib.lib(), _lib.stream_ptr()
    C.layernorm(dict(x=x.data_ptr(), y=y.data_ptr(), gamma=g.data_ptr(), beta=b.data_ptr(), rows=B * T, D=D,
                     ldx=D, ldy=D, eps=1e-6), s)
    cls = torch.zeros(16, D, dtype=torch.bfloat16, device=DEV)
    C.layernorm(dict(x=x.data_ptr(), y=cls.data_ptr(), gamma=g.data_ptr(), beta=b.data_ptr(), rows=B, D=D,
                     ldx=T * D, ldy=D, eps=1e-6), s)
    torch.cuda.synchronize()
    ref = F.layer_norm(x.float(), (D,), g, b, 1e-6)
    assert _rel(y, ref) < 1e-2
    assert _rel(cls[:B], ref.view(B, T, D)[:, 0]) < 1e-2


@pytest.mark.parametrize("T", [197, 50, 256, 300, 1])   # <= 256: whole-head kernel; 300: query-tiled
def test_attention_matches_softmax_reference(T):
    gen = torch.Generator().manual_seed(T)
    B, H, dh = 2, 12, 64
    qkv = torch.randn(B * T, 3 * H * dh, generator=gen).to(torch.bfloat16).to(DEV)
    out = torch.zeros(B * T, H * dh, dtype=torch.bfloat16, device=DEV)
    _lib.lib().attention(dict(qkv=qkv.data_ptr(), out=out.data_ptr(), B=B, T=T, H=H, dh=dh,
                              scale=1 / math.sqrt(dh)), _lib.stream_ptr())
    torch.cuda.synchronize()
    q, k, v = qkv.float().view(B, T, 3, H, dh).permute(2, 0, 3, 1, 4)
    ref = (torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(dh), -1) @ v).transpose(1, 2).reshape(B * T, H * dh)
    assert _rel(out, ref) < 2e-2


def test_patchify_embed_and_patch_gemm():
    gen = torch.Generator().manual_seed(5)
    p = V.init_params(seed=1)
    B = 2
    x = torch.randint(0, 256, (B, 224, 224, 3), generator=gen, dtype=torch.uint8)
    from kdl.engine.vit import ViTEngine
    eng = ViTEngine(p, max_batch=B, device=DEV)
    eng.inp.copy_(x.to(DEV))
    prog = _lib.lib().Program()
    for st in eng.steps[:3]:            # patchify, conv_proj, embed
        eng._emit(prog, st, B)
    prog.run(int(eng.stream.cuda_stream))
    torch.cuda.synchronize()
    ref = V.embed(p, V.preprocess(x)).reshape(B * V.TOKENS, V.DIM)
    assert _rel(eng.bufs["X"], ref) < 2e-2


def test_gelu_epilogue():
    gen = torch.Generator().manual_seed(6)
    M, K, N = 300, 768, 3072
    x = torch.randn(M, K, generator=gen).to(torch.bfloat16)
    w = torch.randn(N, K, generator=gen, dtype=torch.float64) / K ** 0.5
    b = torch.randn(N, generator=gen) * 0.1
    lay = ConvGemmLayer("fc1", MODE_PW, w, b, cin_pad=K, n=N, relu_out=3, device=DEV)
    y = torch.zeros(M * N, dtype=torch.bfloat16, device=DEV)
    lay.launch(x.to(DEV).contiguous(), y, Geometry(1, 1, M, 1, M))
    torch.cuda.synchronize()
    ref = F.gelu(x.float() @ w.float().t() + b)
    assert _rel(y.view(M, N), ref) < 2e-2


def test_vit_engine_matches_oracle():
    from kdl.engine.vit import ViTEngine
    p = V.init_params(seed=0)
    eng = ViTEngine(p, max_batch=4, device=DEV, buckets=[2, 4])
    gen = torch.Generator().manual_seed(9)
    x = torch.randint(0, 256, (3, 224, 224, 3), generator=gen, dtype=torch.uint8)
    ref = V.vit_forward(p, x)
    for capture in (False, True):
        out = eng.forward(x.to(DEV), capture=capture).cpu()
        cos = F.cosine_similarity(out, ref, dim=1)
        assert cos.min() > 0.99, cos
        assert _rel(out, ref) < 0.1


@pytest.mark.parametrize("fp8", [False, True])
def test_vit_stage_pipe_matches_engine(fp8):
    """Stage pipelining of ViT-B/16 (kdl/engine/stages.py): the residual stream X is
    updated by residual GEMMs (res == dst), so a cut between encoder layers hands X across
    in a parity double-buffer and the first residual GEMM of stage 2 writes a stage-private
    copy through a separate write pointer; four batches on two slots match the engine."""
    from kdl.engine.stages import StagePipe
    from kdl.engine.vit import ViTEngine
    from kdl.models import vit as V
    p = V.init_params(seed=0)
    single = ViTEngine(p, max_batch=2, device="cuda", fp8=fp8)
    pipe = StagePipe(ViTEngine(p, max_batch=2, device="cuda", fp8=fp8), "encoder.layers.encoder_layer_5.mlp.3")
    slots = pipe.add_input_slots(2)
    gen = torch.Generator().manual_seed(14)
    imgs = [torch.randint(0, 256, (2, 224, 224, 3), generator=gen, dtype=torch.uint8) for _ in range(4)]
    refs = [single.forward(x.cuda()).cpu() for x in imgs]
    outs, done = [], [torch.cuda.Event() for _ in range(2)]
    for i, x in enumerate(imgs):
        j = i % 2
        if i >= 2:
            done[j].synchronize()
            outs.append(pipe.slot_logits(j).cpu())
        slots[j].copy_(x.cuda())
        ready = torch.cuda.Event()
        ready.record()
        pipe.launch_async(2, [ready], [done[j]], slot=j)
    for i in (2, 3):
        done[i % 2].synchronize()
        outs.append(pipe.slot_logits(i % 2).cpu())
    for o, r in zip(outs, refs):
        assert torch.allclose(o, r, rtol=1e-3, atol=1e-3), (o - r).abs().max()
