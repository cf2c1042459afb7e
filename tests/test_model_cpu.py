"""Keras-semantics oracle and weight-preparation invariants (CPU)."""
import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st
from PIL import Image

from kdl.gateway import preprocess as pp
from kdl.models import xception as X
from kdl.models.layers import bn_eval, fold_bn, maxpool_same, tf_same_pad
from kdl.ops.pack import pack_fragments, round_up, unpack_fragments


def test_param_counts_match_keras():
    assert X.count_params(include_head=False) == 20_861_480      # Keras Xception(include_top=False)
    assert X.count_params() == 21_067_390                        # + GAP/Dense(100)/Dense(10) head


def test_tf_same_padding_asymmetric_pool():
    assert tf_same_pad(147, 3, 2) == (74, 1, 1)
    assert tf_same_pad(74, 3, 2) == (37, 0, 1)                  # odd pad goes bottom/right
    assert tf_same_pad(37, 3, 2) == (19, 1, 1)
    assert tf_same_pad(19, 3, 2) == (10, 1, 1)
    x = torch.arange(74.).view(1, 1, 1, 74).expand(1, 1, 74, 74).contiguous()
    y = maxpool_same(x)
    assert y.shape[-1] == 37
    assert y[0, 0, 0, 0] == 2 and y[0, 0, 0, -1] == 73         # window [72,73,pad] at the right edge
    wrong = torch.nn.functional.max_pool2d(x, 3, 2, padding=1)  # PyTorch symmetric padding is not TF
    assert wrong.shape[-1] == 37 and wrong[0, 0, 0, 0] != y[0, 0, 0, 0]


def test_bn_fold_equivalence_keras_eps():
    g = torch.Generator().manual_seed(0)
    c = 16
    gamma, beta, mean = torch.rand(c, generator=g) + .5, torch.randn(c, generator=g), torch.randn(c, generator=g)
    var = torch.rand(c, generator=g) * 1e-3      # tiny variances make eps=1e-3 vs 1e-5 matter
    x = torch.randn(2, c, 5, 5, generator=g)
    s, t = fold_bn(gamma, beta, mean, var)
    assert torch.allclose(x * s[None, :, None, None] + t[None, :, None, None],
                          bn_eval(x, gamma, beta, mean, var), atol=1e-5)
    assert not torch.allclose(bn_eval(x, gamma, beta, mean, var, eps=1e-5), bn_eval(x, gamma, beta, mean, var))


def test_fragment_pack_roundtrip_and_lane_map():
    w = torch.randn(50, 70, dtype=torch.float64)
    nf, kt = round_up(50, 16) // 16, round_up(70, 32) // 32
    p = pack_fragments(w, nf, kt)
    assert p.shape == (nf, kt, 64, 8)
    assert torch.allclose(unpack_fragments(p, 50, 70), w.to(torch.bfloat16).float())
    # MFMA 16x16x32 operand map: lane l holds W[16f + (l&15)][32t + 8(l>>4) + j]
    f, t, lane, j = 1, 1, 37, 5
    assert p[f, t, lane, j].item() == pytest.approx(w[16 * f + (lane & 15), 32 * t + 8 * (lane >> 4) + j].item(),
                                                    rel=1e-2)


def test_oracle_is_deterministic_and_batch_independent():
    p = X.init_params(seed=1)
    x = torch.rand(3, 299, 299, 3) * 2 - 1
    a = X.xception_forward(p, x)
    b = X.xception_forward(p, x[1:2])
    assert a.shape == (3, 10) and torch.allclose(a[1:2], b, atol=1e-4)


@settings(max_examples=60, deadline=None)
@given(src=st.integers(1, 900), dst=st.sampled_from([224, 299, 331, 600]))
def test_nearest_indices_match_pil(src, dst):
    row = np.arange(src, dtype=np.int64)
    img = Image.fromarray((row % 251).astype(np.uint8)[None, :].repeat(2, 0))
    got = np.asarray(img.resize((dst, 2), Image.NEAREST))[0]
    assert np.array_equal(got, (row[pp.nearest_indices(src, dst)] % 251).astype(np.uint8))


def test_closed_form_is_not_pil():
    """floor((i+0.5)*s) differs from PIL (534->299 row 149)."""
    s = 534 / 299
    assert int((149 + 0.5) * s) == 267
    assert pp.nearest_indices(534, 299)[149] == 266


def test_resnet50_oracle_shapes_and_cost():
    from kdl.models import resnet as R
    assert R.count_params() == R.TOTAL_PARAMS == 25_557_032   # torchvision resnet50
    assert abs(R.macs_per_image() / 1e9 - 4.09) < 0.01
    p = R.init_params(seed=1, calibrate=False)
    x = torch.randint(0, 256, (1, 224, 224, 3), dtype=torch.uint8)
    y1, y2 = R.resnet_forward(p, x), R.resnet_forward(p, x)
    assert y1.shape == (1, 1000) and torch.equal(y1, y2)
    assert [b.stride for b in R.blocks()].count(2) == 3          # v1.5: stride on conv2 of 3 stages


def test_vit_b16_oracle_shapes_and_cost():
    from kdl.models import vit as V
    assert V.count_params() == V.TOTAL_PARAMS == 86_567_656     # torchvision vit_b_16
    assert abs(V.macs_per_image() / 1e9 - 17.56) < 0.01
    p = V.init_params(seed=1)
    x = torch.randint(0, 256, (1, 224, 224, 3), dtype=torch.uint8)
    assert V.vit_forward(p, x).shape == (1, 1000)


def test_efficientnet_b7_oracle_shapes_and_cost():
    from kdl.models import efficientnet as E
    assert len(E.blocks()) == 55
    assert E.count_params() == E.TOTAL_PARAMS == 66_347_960   # torchvision efficientnet_b7
    assert abs(E.macs_per_image() / 1e9 - 37.75) < 0.01
    assert (E.STEM, E.HEAD) == (64, 2560)
