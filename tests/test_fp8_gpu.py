"""gfx950 block-scaled fp8 MFMA (OCP e4m3) lane map, determined with exact
small-integer data, and the fp8 GEMM path built on it."""
import pytest
import torch

from kdl.ops import _lib

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _kmap(name):
    """k index of byte j (0..31) of lane group g (= lane >> 4) under a candidate map."""
    if name == "contig32":
        return lambda g, j: 32 * g + j
    if name == "split16":
        return lambda g, j: 16 * g + j if j < 16 else 64 + 16 * g + (j - 16)
    if name == "interleave8":
        return lambda g, j: 8 * g + (j % 8) + 32 * (j // 8)
    raise KeyError(name)


def _pack(A, B, km):
    """A [16][128], B [128][16] small ints -> lane-ordered e4m3 bytes [64][32] each."""
    a = torch.zeros(64, 32)
    b = torch.zeros(64, 32)
    for lane in range(64):
        g, r = lane >> 4, lane & 15
        for j in range(32):
            a[lane, j] = A[r, km(g, j)]
            b[lane, j] = B[km(g, j), r]
    enc = lambda t: t.to(torch.float8_e4m3fn).view(torch.uint8)  # noqa: E731
    return enc(a).contiguous(), enc(b).contiguous()


def probe_layout():
    gen = torch.Generator().manual_seed(0)
    A = torch.randint(-2, 3, (16, 128), generator=gen).float()
    B = torch.randint(-2, 3, (128, 16), generator=gen).float()
    ref = A @ B
    found = []
    for name in ("contig32", "split16", "interleave8"):
        a, b = _pack(A, B, _kmap(name))
        d = torch.zeros(64, 4, device=DEV)
        ad, bd = a.to(DEV), b.to(DEV)
        _lib.lib().mfma_f8_probe(ad.data_ptr(), bd.data_ptr(), d.data_ptr(), _lib.stream_ptr())
        torch.cuda.synchronize()
        D = torch.zeros(16, 16)
        dc = d.cpu()
        for lane in range(64):
            for r in range(4):
                D[4 * (lane >> 4) + r, lane & 15] = dc[lane, r]
        if torch.equal(D, ref):
            found.append(name)
    return found


def test_fp8_mfma_lane_map():
    """Any k bijection shared by A and B gives the same product, so all candidates
    reproduce A.B; what this pins down is the row/column (lane & 15) and C/D maps and
    that 'contig32' (lane group g holds k = 32g .. 32g+31) -- the order gemm_f8.hip
    stages both operands in -- is a valid operand order."""
    found = probe_layout()
    print("fp8 16x16x128 consistent lane maps:", found)
    assert "contig32" in found, found


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
    y8 = torch.zeros(M, N, dtype=torch.uint8, device=DEV)
    so = 0.02
    lay.emit(None, x8=x8.data_ptr(), M=M, y8=y8.data_ptr(), out_scale=so)
    torch.cuda.synchronize()
    ref = (from_e4m3(x8.cpu()) * sa) @ lay.w_ref.t()
    got = from_e4m3(y8.cpu()) * so
    assert ((got - ref).abs().max() / ref.abs().max()).item() < 0.08     # e4m3 output rounding (3 mantissa bits)


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
