"""Wire codec: runtime protos vs the native zero-copy parser/builder (kdl._rt)."""
import numpy as np
import pytest

from kdl.ops import _lib
from kdl.serving import protos as P

rt = pytest.importorskip("kdl._rt")


def _req(x, key="input_8", name="clothing-model", sig="serving_default", version=None, filt=()):
    r = P.PredictRequest()
    r.model_spec.name = name
    r.model_spec.signature_name = sig
    if version is not None:
        r.model_spec.version.value = version
    r.inputs[key].CopyFrom(P.np_to_tensor_proto(x))
    r.output_filter.extend(filt)
    return r.SerializeToString()


def test_tensor_proto_roundtrip_dtypes():
    for dt in (np.float32, np.uint8, np.int32, np.int64, np.float64):
        x = (np.arange(24).reshape(2, 3, 4) % 7).astype(dt)
        t = P.np_to_tensor_proto(x)
        assert t.tensor_content
        y = P.tensor_proto_to_np(P.TensorProto.FromString(t.SerializeToString()))
        assert y.dtype == x.dtype and np.array_equal(x, y)


def test_typed_float_val_and_broadcast():
    t = P.TensorProto(dtype=P.DT_FLOAT)
    t.tensor_shape.dim.add(size=2)
    t.tensor_shape.dim.add(size=2)
    t.float_val.extend([1.5])
    assert np.array_equal(P.tensor_proto_to_np(t), np.full((2, 2), 1.5, np.float32))


def test_native_parse_matches_python():
    x = np.random.default_rng(0).random((2, 299, 299, 3), dtype=np.float32)
    raw = _req(x, version=3, filt=["dense_7"])
    v = rt.parse_predict_request(raw)
    assert v["model_spec"] == {"name": "clothing-model", "signature_name": "serving_default",
                               "version_label": "", "version": 3}
    assert v["output_filter"] == ["dense_7"]
    (t,) = v["inputs"]
    assert t["key"] == "input_8" and t["dtype"] == P.DT_FLOAT and t["dims"] == [2, 299, 299, 3]
    assert t["has_content"] and t["size"] == x.nbytes
    view = np.frombuffer(raw, dtype=np.float32, count=x.size, offset=t["offset"]).reshape(x.shape)
    assert np.array_equal(view, x)


def test_native_parse_rejects_garbage():
    with pytest.raises(ValueError):
        rt.parse_predict_request(b"\x12\xff\xff\xff\xff\x0f")  # length past end


def test_build_response_parses_with_python_protobuf():
    logits = np.random.default_rng(1).standard_normal((3, 10)).astype(np.float32)
    raw = rt.build_predict_response([("dense_7", logits)], "clothing-model", 1, "serving_default")
    r = P.PredictResponse.FromString(raw)
    assert r.model_spec.name == "clothing-model" and r.model_spec.version.value == 1
    out = r.outputs["dense_7"]
    assert out.dtype == P.DT_FLOAT and [d.size for d in out.tensor_shape.dim] == [3, 10]
    assert np.array_equal(np.asarray(out.float_val, np.float32).reshape(3, 10), logits)


def test_request_size_matches_reference_wire():
    """a 1x299x299x3 f32 TensorProto is 1,072,838 bytes on the wire."""
    x = np.zeros((1, 299, 299, 3), np.float32)
    assert len(P.np_to_tensor_proto(x).SerializeToString()) == 1_072_838


def test_model_spec_request_parse():
    req = P.GetModelStatusRequest()
    req.model_spec.name = "m"
    req.model_spec.version.value = 7
    assert rt.parse_model_spec_request(req.SerializeToString())["version"] == 7


def test_f32_to_u8_exact_detects_reference_preprocessing():
    """kdl._rt.f32_to_u8_exact: the reference gateway's x = u8 / 127.5 - 1 (float32, keras_image_helper,
    model_server.py:18) maps back to the exact pixels; any other float fails the check."""
    import numpy as np
    from kdl.ops import _lib
    rt = _lib.rt()
    u = np.random.default_rng(0).integers(0, 256, (2, 299, 299, 3), dtype=np.uint8)
    u[0, 0, 0] = (0, 255, 128)
    x = u.astype(np.float32) / 127.5 - 1
    out = np.empty(u.size, np.uint8)
    assert rt.f32_to_u8_exact(x, out) and np.array_equal(out.reshape(u.shape), u)
    for bad in (0.5, 1.0000001, -1.5, float("nan")):
        y = x.copy()
        y[1, 7, 9, 2] = bad
        assert not rt.f32_to_u8_exact(y, out), bad
