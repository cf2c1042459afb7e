"""hipBLASLt GEMM node (kdl/csrc/runtime/blaslt.cpp) against fp32 torch: bias, ReLU,
residual as the C operand (in place), fp16, every heuristic rank the tuner may pick, and
the ViT engine with every eligible linear on it vs the fp32 oracle."""
import pytest
import torch

from kdl.ops import _lib
from kdl.ops.conv import BLT_ALGOS, BLT_BASE, MODE_PW, ConvGemmLayer, Geometry

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a.float().cpu() - b.float().cpu()).abs().max() / b.float().abs().max()).item()


def _layer(N, K, relu_out=0, dtype=torch.bfloat16, seed=0):
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(N, K, generator=g, dtype=torch.float64) / K ** 0.5
    b = torch.randn(N, generator=g) * 0.5
    return ConvGemmLayer("lin", MODE_PW, w, b, cin_pad=K, n=N, relu_out=relu_out, device=DEV, dtype=dtype,
                         blaslt=True)


@pytest.mark.parametrize("M,N,K,relu_out,res,dtype", [
    (6304, 768, 3072, 0, True, torch.bfloat16),     # ViT mlp.3: bias + residual, in place
    (6304, 2304, 768, 0, False, torch.bfloat16),    # ViT QKV: bias
    (197, 768, 768, 0, True, torch.bfloat16),       # one image of out_proj
    (1000, 256, 64, 1, False, torch.float16),       # ResNet conv1-like: bias + ReLU
    (1000, 256, 64, 2, True, torch.float16),        # ResNet conv3-like: ReLU after the residual add
    (6304, 3072, 768, 3, False, torch.bfloat16),    # ViT mlp.0: bias + GELU (hipBLASLt's form)
])
def test_blaslt_linear_matches_fp32(M, N, K, relu_out, res, dtype):
    lay = _layer(N, K, relu_out, dtype)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(M, K, generator=g).to(dtype).to(DEV)
    r = torch.randn(M, lay.ldy, generator=g).to(dtype).to(DEV) if res else None
    ref = x.float() @ lay.w_ref.to(DEV).T + lay.bias[:N].float()
    if res:
        ref = ref + r[:, :N].float()
    if relu_out == 3:
        ref = torch.nn.functional.gelu(ref)
    elif relu_out:
        ref = ref.clamp_min(0)
    geo = Geometry(1, 1, M, 1, M)
    for algo in range(BLT_ALGOS):
        # in place like the ViT residual stream: y is the residual buffer itself
        y = r.clone() if res else torch.zeros(M, lay.ldy, dtype=dtype, device=DEV)
        lay.emit(None, x.data_ptr(), y.data_ptr(), geo, res=y.data_ptr() if res else None, cfg=BLT_BASE + algo)
        torch.cuda.synchronize()
        err = _rel(y[:, :N], ref)
        assert err < 1e-2, (algo, err)


def test_blaslt_node_in_captured_program():
    lay = _layer(768, 768)
    M = 394
    x = torch.randn(M, 768, device=DEV).to(torch.bfloat16)
    y = torch.zeros(M, lay.ldy, dtype=torch.bfloat16, device=DEV)
    C = _lib.lib()
    prog = C.Program()
    lay.emit(prog, x.data_ptr(), y.data_ptr(), Geometry(1, 1, M, 1, M), cfg=BLT_BASE)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        prog.capture(s.cuda_stream)
        for _ in range(3):
            prog.launch(s.cuda_stream)
    s.synchronize()
    ref = x.float() @ lay.w_ref.to(DEV).T + lay.bias[:768]
    assert _rel(y, ref) < 1e-2


def test_vit_engine_with_blaslt_linears_matches_oracle():
    from kdl.engine.vit import ViTEngine
    from kdl.models import vit as V
    p = V.init_params(seed=0)
    eng = ViTEngine(p, max_batch=2, device=DEV, buckets=[2])
    table = {s.name: [0, BLT_BASE] for s in eng.conv_steps() if s.layer.w_plain is not None}
    assert len(table) == 36, len(table)     # qkv, out_proj, mlp.3 of 12 layers
    eng.apply_tuning(table)
    assert all(s.layer.cfg == BLT_BASE for s in eng.conv_steps() if s.name in table)
    x = torch.randint(0, 256, (2, 224, 224, 3), generator=torch.Generator().manual_seed(3), dtype=torch.uint8)
    out = eng.forward(x.to(DEV))
    torch.cuda.synchronize()
    ref = V.vit_forward(p, x)
    assert _rel(out, ref) < 0.05
    cos = torch.nn.functional.cosine_similarity(out.float().cpu(), ref, dim=1)
    assert cos.min() > 0.99, cos


def test_blaslt_e4m3_linear_matches_dequantized_reference():
    from kdl.ops.f8 import F8Linear, from_e4m3, to_e4m3
    g = torch.Generator().manual_seed(7)
    M, N, K = 6304, 768, 3072                    # ViT mlp.3 with the residual in place
    w = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g) * 0.1
    s_in = 4.0 / 448
    lay = F8Linear("mlp3", w, b, s_in, device=DEV, blaslt=True)
    x8 = to_e4m3(torch.randn(M, K, generator=g) * 2 / s_in).to(DEV)
    r = torch.randn(M, N, generator=g).to(torch.bfloat16).to(DEV)
    ref = (from_e4m3(x8.cpu()) * s_in) @ lay.w_ref.T + b + r.float().cpu()
    for algo in range(BLT_ALGOS):
        y = r.clone()
        lay.emit(None, cfg=BLT_BASE + algo, x8=x8.data_ptr(), M=M, y=y.data_ptr(), res=y.data_ptr(), ldy=N)
        torch.cuda.synchronize()
        assert _rel(y, ref) < 1e-2, algo


