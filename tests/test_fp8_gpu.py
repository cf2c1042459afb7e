"""The gfx950 block-scaled fp8 (OCP e4m3) GEMM path: gemm_f8.hip against a dequantized
fp32 reference (which also pins the MFMA operand lane order the kernel stages in)."""
import pytest
import torch

from kdl.ops import _lib

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("M,K,N,relu,res", [(300, 768, 2304, 0, False), (197 * 2, 3072, 768, 0, True),
                                           (128, 768, 3072, 3, False)])
def test_gemm_f8_matches_dequantized_reference(M, K, N, relu, res):
    from kdl.ops.f8 import F8Linear, from_e4m3, to_e4m3
    gen = torch.Generator().manual_seed(M + K)
    x = torch.randn(M, K, generator=gen) * 2
    sa = x.abs().max().item() / 448
    x8 = to_e4m3(x / sa)
    w = torch.randn(N, K, generator=gen) / K ** 0.5
    b = torch.randn(N, generator=gen) * 0.1
    lay = F8Linear("t", w, b, sa, relu_out=relu, device=DEV)
    r = (torch.randn(M, N, generator=gen)).to(torch.bfloat16)
    y = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    if res:
        y.copy_(r.to(DEV))
    x8d = x8.to(DEV).contiguous()
    ref = (from_e4m3(x8) * sa) @ lay.w_ref.t() + b
    if relu == 3:
        ref = torch.nn.functional.gelu(ref)
    if res:
        ref = ref + r.float()
    for cfg in lay.candidates:
        if res:
            y.copy_(r.to(DEV))
        lay.emit(None, cfg=cfg, x8=x8d.data_ptr(), M=M, y=y.data_ptr(), res=y.data_ptr() if res else None)
        torch.cuda.synchronize()
        err = ((y.float().cpu() - ref).abs().max() / ref.abs().max()).item()
        assert err < 1.5e-2, (cfg, err)


def test_gemm_f8_fp8_output():
    from kdl.ops.f8 import F8Linear, from_e4m3, to_e4m3
    gen = torch.Generator().manual_seed(5)
    M, K, N = 256, 768, 768
    x = torch.randn(M, K, generator=gen)
    sa = x.abs().max().item() / 448
    x8 = to_e4m3(x / sa).to(DEV)
    lay = F8Linear("t", torch.randn(N, K, generator=gen) / K ** 0.5, torch.zeros(N), sa, device=DEV)
    so = 0.02
    ref = (from_e4m3(x8.cpu()) * sa) @ lay.w_ref.t()
    for cfg in lay.candidates:                 # incl. the persistent direct-epilogue configs (32-37)
        y8 = torch.zeros(M, N, dtype=torch.uint8, device=DEV)
        lay.emit(None, cfg=cfg, x8=x8.data_ptr(), M=M, y8=y8.data_ptr(), out_scale=so)
        torch.cuda.synchronize()
        got = from_e4m3(y8.cpu()) * so
        assert ((got - ref).abs().max() / ref.abs().max()).item() < 0.08, cfg   # e4m3 output rounding


def test_vit_fp8_engine_matches_oracle():
    import torch.nn.functional as F

    from kdl.engine.vit import ViTEngine
    from kdl.models import vit as V
    p = V.init_params(seed=0)
    eng = ViTEngine(p, max_batch=4, device=DEV, buckets=[4], fp8=True)
    gen = torch.Generator().manual_seed(9)
    x = torch.randint(0, 256, (3, 224, 224, 3), generator=gen, dtype=torch.uint8)
    ref = V.vit_forward(p, x)
    out = eng.forward(x.to(DEV)).cpu()
    cos = F.cosine_similarity(out, ref, dim=1)
    assert cos.min() > 0.97, cos
