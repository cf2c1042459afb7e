"""``kdl convert-savedmodel``: BN folded into the conv kernels, kernels stored bf16.

CPU: the folded artifact round-trips through the CLI and the model repo loader, its kernels
are exactly what the engine would pack from the unfolded variables, and the fp32 oracle on
it agrees with the oracle on the original variables to bf16 weight rounding. GPU: the
engine built from either gives bit-identical logits.
"""
import json

import numpy as np
import pytest
import torch

from kdl.ingest.fold import FOLDED_KEY, fold_xception, unpack
from kdl.ingest.keras_map import to_keras_variables
from kdl.ingest.savedmodel import write_savedmodel
from kdl.models import xception as X
from kdl.ops.pack import bn_scale_shift


@pytest.fixture(scope="module")
def params():
    return X.init_params(seed=7)


def test_folded_kernels_are_the_engine_products(params):
    f = unpack(fold_xception(params))
    assert FOLDED_KEY not in f and "block5_sepconv1_bn/gamma" not in f and "block1_conv1_bn/gamma" in f
    s, t = bn_scale_shift(params, "block5_sepconv1_bn")
    want = (params["block5_sepconv1/pointwise_kernel"].double() * s).float().to(torch.bfloat16).float()
    assert torch.equal(f["block5_sepconv1/pointwise_kernel"], want)
    assert torch.equal(f["block5_sepconv1_bn/beta"], t.float())
    s2, t2 = bn_scale_shift(f, "block5_sepconv1_bn")       # folded BN reads as (1, shift)
    assert torch.equal(s2, torch.ones_like(s2)) and torch.equal(t2, t.float().double())
    assert torch.equal(f["block5_sepconv1/depthwise_kernel"], params["block5_sepconv1/depthwise_kernel"])


def test_oracle_on_folded_params_matches(params):
    x = torch.rand((2, 299, 299, 3), generator=torch.Generator().manual_seed(1)) * 2 - 1
    a = X.xception_forward(params, x)
    b = X.xception_forward(unpack(fold_xception(params)), x)
    assert (a - b).abs().max() < 0.02 * a.abs().max()


def test_cli_convert_writes_a_servable_folded_artifact(tmp_path, params):
    from kdl.cli import main
    from kdl.serving.backend import load_version_dir
    src, dst = tmp_path / "sm" / "1", tmp_path / "kdl" / "2"
    write_savedmodel(src, to_keras_variables(params, residual_offset=2))
    assert main(["convert-savedmodel", str(src), str(dst)]) == 0
    meta = json.loads((dst / "kdl_model.json").read_text())
    assert meta["bn_folded"] is True and "serving_default" in meta["signatures"]
    size_folded = (dst / "kdl_params.safetensors").stat().st_size
    assert main(["convert-savedmodel", str(src), str(tmp_path / "raw"), "--keep-bn"]) == 0
    assert size_folded < 0.6 * (tmp_path / "raw" / "kdl_params.safetensors").stat().st_size
    source = load_version_dir(dst)
    assert source.origin == "kdl_safetensors" and "block5_sepconv1_bn/gamma" not in source.params
    x = torch.rand((1, 299, 299, 3), generator=torch.Generator().manual_seed(2)) * 2 - 1
    ref = X.xception_forward(params, x)
    got = X.xception_forward(source.params, x, head=source.head)
    assert (got - ref).abs().max() < 0.02 * ref.abs().max()


@pytest.mark.gpu
def test_engine_from_folded_params_is_bit_identical(params):
    from kdl.engine.xception import XceptionEngine
    img = torch.randint(0, 256, (2, 299, 299, 3), generator=torch.Generator().manual_seed(3), dtype=torch.uint8)
    a = XceptionEngine(params, max_batch=2).forward(img.cuda())
    b = XceptionEngine(unpack(fold_xception(params)), max_batch=2).forward(img.cuda())
    assert torch.equal(a, b), (a - b).abs().max()
    assert np.isfinite(a.cpu().numpy()).all()
