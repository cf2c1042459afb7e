"""SavedModel / TensorBundle ingest without TensorFlow (fixtures are synthesised:
no real Keras export is reachable offline, so parity with real TF output is
'unpinned' beyond the format spec; SURVEY.md §7.4 hard part 4)."""
import numpy as np
import pytest
import torch

from kdl.ingest import tensorbundle as TB
from kdl.ingest.keras_map import to_keras_variables, to_xception_params
from kdl.ingest.savedmodel import SavedModelDir, write_savedmodel
from kdl.models import xception as X


@pytest.fixture(scope="module")
def params():
    return X.init_params(seed=3, calibrate=False)


@pytest.mark.parametrize("compress", [False, True])
def test_sstable_native_matches_python(compress):
    rng = np.random.default_rng(0)
    kv = [(f"key/{i:05d}/{'x' * (i % 7)}".encode(), rng.bytes(int(rng.integers(0, 300)))) for i in range(500)]
    raw = TB.write_sstable(kv, compress=compress, block_size=1024)
    a = TB.read_sstable_py(raw)
    assert a == sorted(kv)
    if TB.read_sstable is not None:
        assert TB.read_sstable(raw) == a


def test_sstable_detects_corruption():
    raw = bytearray(TB.write_sstable([(b"a", b"1" * 100), (b"b", b"2" * 100)]))
    raw[10] ^= 0xFF
    with pytest.raises(Exception):
        TB.read_sstable(bytes(raw))
    with pytest.raises(ValueError):
        TB.read_sstable_py(b"x" * 100)


def test_snappy_decoder_copies():
    # hand-built stream: literal "abcd" + copy(len 8, offset 4) -> "abcdabcdabcd"
    stream = bytes([12]) + bytes([(4 - 1) << 2]) + b"abcd" + bytes([((8 - 4) << 2) | 1, 4])
    assert TB._snappy_py(stream) == b"abcdabcdabcd"
    from kdl.ops import _lib
    if _lib.rt_available():
        assert _lib.rt().snappy_uncompress(stream) == b"abcdabcdabcd"


def test_bundle_roundtrip(tmp_path):
    t = {"a/kernel": np.arange(12, dtype=np.float32).reshape(3, 4), "b": np.array([1, 2, 3], np.int64)}
    TB.write_bundle(tmp_path / "v", t)
    b = TB.TensorBundle(tmp_path / "v")
    assert b.keys() == ["a/kernel", "b"]
    for k, v in t.items():
        assert np.array_equal(b.get(k), v) and b.get(k).dtype == v.dtype


@pytest.mark.parametrize("offset,compress", [(0, False), (7, True)])
def test_savedmodel_roundtrip_to_xception(tmp_path, params, offset, compress):
    d = write_savedmodel(tmp_path / "1", to_keras_variables(params, residual_offset=offset), compress=compress)
    sm = SavedModelDir(d)
    sig = sm.signatures["serving_default"]
    assert list(sig.inputs) == ["input_8"] and list(sig.outputs) == ["dense_7"]
    assert sig.inputs["input_8"].shape == (-1, 299, 299, 3)
    assert "inputs['input_8'] tensor_info" in sm.show()
    p2, head = to_xception_params(sm.variables())
    assert head.hidden == "dense_6" and head.out == "dense_7"
    assert set(p2) == set(params)
    for k in params:
        assert torch.equal(params[k], p2[k]), k


def test_savedmodel_without_object_graph_uses_keys(tmp_path, params):
    d = write_savedmodel(tmp_path / "1", to_keras_variables(params), with_object_graph=False)
    names = SavedModelDir(d).variable_names()
    assert all(k.startswith("layer_with_weights-") for k in names)


def test_missing_variables_is_an_error(tmp_path, params):
    v = to_keras_variables(params)
    v.pop("block5_sepconv1/pointwise_kernel")
    d = write_savedmodel(tmp_path / "1", v)
    with pytest.raises(ValueError, match="missing"):
        to_xception_params(SavedModelDir(d).variables())


def test_shape_mismatch_is_an_error(tmp_path, params):
    v = to_keras_variables(params)
    v["block1_conv1/kernel"] = np.zeros((3, 3, 3, 16), np.float32)
    with pytest.raises(ValueError, match="shape"):
        to_xception_params(SavedModelDir(write_savedmodel(tmp_path / "1", v)).variables())
