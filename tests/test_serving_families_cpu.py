"""The model server serves every family behind the same TF-Serving API (CPU
oracle backend): ResNet-50 from torchvision-layout safetensors written by
``kdl make-synthetic --model resnet50``, uint8 ``images`` -> 1000 logits."""
import grpc
import numpy as np
import pytest
import torch

from kdl.cli import main as cli_main
from kdl.gateway.client import PredictionStub, make_request
from kdl.models import resnet as R
from kdl.serving import protos as P
from kdl.serving.config import BatchingParams, ServerConfig
from kdl.serving.server import ModelServer

pytest.importorskip("kdl._rt")


@pytest.fixture(scope="module")
def resnet_server(tmp_path_factory):
    base = tmp_path_factory.mktemp("m") / "resnet"
    assert cli_main(["make-synthetic", str(base / "1"), "--model", "resnet50", "--seed", "3"]) == 0
    cfg = ServerConfig(port=0, rest_api_port=0, model_name="resnet", model_base_path=str(base), device="cpu",
                       host="127.0.0.1", file_system_poll_wait_seconds=0,
                       batching=BatchingParams(max_batch_size=2, batch_timeout_micros=1000, allowed_batch_sizes=[1, 2]))
    srv = ModelServer(cfg).start(block_until_loaded=True)
    yield srv
    srv.stop(0)


def test_resnet_predict_and_metadata(resnet_server):
    ch = grpc.insecure_channel(f"127.0.0.1:{resnet_server.grpc_port}")
    stub = PredictionStub(ch)
    x = np.random.default_rng(0).integers(0, 256, (2, 224, 224, 3), dtype=np.uint8)
    r = stub.Predict(make_request(x, model_name="resnet", input_key="images"), timeout=60)
    got = np.asarray(r.outputs["logits"].float_val, np.float32).reshape(2, 1000)
    ref = R.resnet_forward(R.init_params(seed=3), torch.from_numpy(x)).numpy()
    assert np.allclose(got, ref, atol=1e-3)
    req = P.GetModelMetadataRequest()
    req.model_spec.name = "resnet"
    req.metadata_field.append("signature_def")
    md = stub.GetModelMetadata(req, timeout=5)
    sdm = P.SignatureDefMap()
    md.metadata["signature_def"].Unpack(sdm)
    sd = sdm.signature_def["serving_default"]
    assert [d.size for d in sd.inputs["images"].tensor_shape.dim] == [-1, 224, 224, 3]
    assert [d.size for d in sd.outputs["logits"].tensor_shape.dim] == [-1, 1000]
    with pytest.raises(grpc.RpcError) as e:   # a 299x299 Xception-shaped request is rejected
        stub.Predict(make_request(np.zeros((1, 299, 299, 3), np.uint8), model_name="resnet", input_key="images"),
                     timeout=5)
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
