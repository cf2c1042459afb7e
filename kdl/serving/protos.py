"""TensorFlow / TF-Serving wire types built at runtime from ``descriptor_pb2``.

The reference talks to TF-Serving with ``tensorflow_serving.apis`` generated
classes (`model_server.py:3-6,38-49`). Neither ``protoc``, ``grpc_tools`` nor
TensorFlow exist here, so the exact same messages (same package names, field
numbers and types, so the bytes are wire-identical) are declared with
``descriptor_pb2`` and materialised with ``message_factory``. Only the fields the
framework reads or writes are declared; protobuf skips unknown fields, so real
TF-produced bytes (e.g. a full ``saved_model.pb``) still parse.

Covered: tensorflow.{DataType, TensorShapeProto, TensorProto, TensorInfo,
SignatureDef, MetaGraphDef, SavedModel, SavedObjectGraph, TrackableObjectGraph,
BundleHeaderProto, BundleEntryProto, VersionDef}; tensorflow.serving.{ModelSpec,
PredictRequest/Response, GetModelMetadataRequest/Response, SignatureDefMap,
GetModelStatusRequest/Response, ModelVersionStatus, StatusProto,
ReloadConfigRequest/Response}; services PredictionService and ModelService.
"""
from __future__ import annotations

from google.protobuf import any_pb2, descriptor_pb2, descriptor_pool, message_factory, wrappers_pb2

F = descriptor_pb2.FieldDescriptorProto
OPT, REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED

# tensorflow.DataType (tensorflow/core/framework/types.proto)
DT_INVALID, DT_FLOAT, DT_DOUBLE, DT_INT32, DT_UINT8 = 0, 1, 2, 3, 4
DT_INT16, DT_INT8, DT_STRING, DT_INT64, DT_BOOL = 5, 6, 7, 9, 10
DT_BFLOAT16, DT_HALF, DT_UINT16 = 14, 19, 17
DTYPE_NAMES = {0: "DT_INVALID", 1: "DT_FLOAT", 2: "DT_DOUBLE", 3: "DT_INT32", 4: "DT_UINT8", 5: "DT_INT16",
               6: "DT_INT8", 7: "DT_STRING", 9: "DT_INT64", 10: "DT_BOOL", 14: "DT_BFLOAT16", 17: "DT_UINT16",
               19: "DT_HALF"}


def _field(msg, name, num, ftype, label=OPT, type_name=None, packed=None, oneof=None):
    f = msg.field.add(name=name, number=num, type=ftype, label=label)
    if type_name:
        f.type_name = type_name
    if packed is not None:
        f.options.packed = packed
    if oneof is not None:
        f.oneof_index = oneof
    return f


def _map(file, msg, name, num, key_type, val_type, val_type_name=None):
    entry = msg.nested_type.add(name="".join(p.capitalize() for p in name.split("_")) + "Entry")
    entry.options.map_entry = True
    _field(entry, "key", 1, key_type)
    _field(entry, "value", 2, val_type, type_name=val_type_name)
    _field(msg, name, num, F.TYPE_MESSAGE, REP, type_name=f".{file.package}.{msg.name}.{entry.name}")


def _build_pool() -> descriptor_pool.DescriptorPool:
    pool = descriptor_pool.DescriptorPool()
    pool.AddSerializedFile(wrappers_pb2.DESCRIPTOR.serialized_pb)
    pool.AddSerializedFile(any_pb2.DESCRIPTOR.serialized_pb)

    # ---------------------------------------------------------------- tensorflow core
    tf = descriptor_pb2.FileDescriptorProto(name="kdl/tensorflow_core.proto", package="tensorflow",
                                            syntax="proto3")
    dt = tf.enum_type.add(name="DataType")
    for num, name in sorted(DTYPE_NAMES.items()):
        dt.value.add(name=name, number=num)

    shape = tf.message_type.add(name="TensorShapeProto")
    dim = shape.nested_type.add(name="Dim")
    _field(dim, "size", 1, F.TYPE_INT64)
    _field(dim, "name", 2, F.TYPE_STRING)
    _field(shape, "dim", 2, F.TYPE_MESSAGE, REP, ".tensorflow.TensorShapeProto.Dim")
    _field(shape, "unknown_rank", 3, F.TYPE_BOOL)

    t = tf.message_type.add(name="TensorProto")
    _field(t, "dtype", 1, F.TYPE_ENUM, type_name=".tensorflow.DataType")
    _field(t, "tensor_shape", 2, F.TYPE_MESSAGE, type_name=".tensorflow.TensorShapeProto")
    _field(t, "version_number", 3, F.TYPE_INT32)
    _field(t, "tensor_content", 4, F.TYPE_BYTES)
    _field(t, "float_val", 5, F.TYPE_FLOAT, REP, packed=True)
    _field(t, "double_val", 6, F.TYPE_DOUBLE, REP, packed=True)
    _field(t, "int_val", 7, F.TYPE_INT32, REP, packed=True)
    _field(t, "string_val", 8, F.TYPE_BYTES, REP)
    _field(t, "int64_val", 10, F.TYPE_INT64, REP, packed=True)
    _field(t, "bool_val", 11, F.TYPE_BOOL, REP, packed=True)
    _field(t, "half_val", 13, F.TYPE_INT32, REP, packed=True)

    ti = tf.message_type.add(name="TensorInfo")
    ti.oneof_decl.add(name="encoding")
    _field(ti, "name", 1, F.TYPE_STRING, oneof=0)
    _field(ti, "dtype", 2, F.TYPE_ENUM, type_name=".tensorflow.DataType")
    _field(ti, "tensor_shape", 3, F.TYPE_MESSAGE, type_name=".tensorflow.TensorShapeProto")

    sd = tf.message_type.add(name="SignatureDef")
    _map(tf, sd, "inputs", 1, F.TYPE_STRING, F.TYPE_MESSAGE, ".tensorflow.TensorInfo")
    _map(tf, sd, "outputs", 2, F.TYPE_STRING, F.TYPE_MESSAGE, ".tensorflow.TensorInfo")
    _field(sd, "method_name", 3, F.TYPE_STRING)

    mi = tf.message_type.add(name="MetaInfoDef")
    _field(mi, "meta_graph_version", 1, F.TYPE_STRING)
    _field(mi, "tags", 4, F.TYPE_STRING, REP)
    _field(mi, "tensorflow_version", 5, F.TYPE_STRING)
    _field(mi, "tensorflow_git_version", 6, F.TYPE_STRING)

    # SavedObjectGraph (subset): node children + user_object metadata + variable info
    soref = tf.message_type.add(name="SavedObjectReference")  # TrackableObjectGraph.ObjectReference
    _field(soref, "node_id", 1, F.TYPE_INT32)
    _field(soref, "local_name", 2, F.TYPE_STRING)
    suo = tf.message_type.add(name="SavedUserObject")
    _field(suo, "identifier", 1, F.TYPE_STRING)
    _field(suo, "metadata", 3, F.TYPE_STRING)
    svar = tf.message_type.add(name="SavedVariable")
    _field(svar, "dtype", 1, F.TYPE_ENUM, type_name=".tensorflow.DataType")
    _field(svar, "shape", 2, F.TYPE_MESSAGE, type_name=".tensorflow.TensorShapeProto")
    _field(svar, "trainable", 3, F.TYPE_BOOL)
    _field(svar, "name", 6, F.TYPE_STRING)
    so = tf.message_type.add(name="SavedObject")
    so.oneof_decl.add(name="kind")
    _field(so, "children", 1, F.TYPE_MESSAGE, REP, ".tensorflow.SavedObjectReference")
    _field(so, "user_object", 4, F.TYPE_MESSAGE, type_name=".tensorflow.SavedUserObject", oneof=0)
    _field(so, "variable", 7, F.TYPE_MESSAGE, type_name=".tensorflow.SavedVariable", oneof=0)
    sog = tf.message_type.add(name="SavedObjectGraph")
    _field(sog, "nodes", 1, F.TYPE_MESSAGE, REP, ".tensorflow.SavedObject")

    mg = tf.message_type.add(name="MetaGraphDef")
    _field(mg, "meta_info_def", 1, F.TYPE_MESSAGE, type_name=".tensorflow.MetaInfoDef")
    _map(tf, mg, "signature_def", 5, F.TYPE_STRING, F.TYPE_MESSAGE, ".tensorflow.SignatureDef")
    _field(mg, "object_graph_def", 7, F.TYPE_MESSAGE, type_name=".tensorflow.SavedObjectGraph")

    sm = tf.message_type.add(name="SavedModel")
    _field(sm, "saved_model_schema_version", 1, F.TYPE_INT64)
    _field(sm, "meta_graphs", 2, F.TYPE_MESSAGE, REP, ".tensorflow.MetaGraphDef")

    # TrackableObjectGraph (tensorflow/core/protobuf/trackable_object_graph.proto)
    tog = tf.message_type.add(name="TrackableObjectGraph")
    tobj = tog.nested_type.add(name="TrackableObject")
    oref = tobj.nested_type.add(name="ObjectReference")
    _field(oref, "node_id", 1, F.TYPE_INT32)
    _field(oref, "local_name", 2, F.TYPE_STRING)
    ser = tobj.nested_type.add(name="SerializedTensor")
    _field(ser, "name", 1, F.TYPE_STRING)
    _field(ser, "full_name", 2, F.TYPE_STRING)
    _field(ser, "checkpoint_key", 3, F.TYPE_STRING)
    _field(tobj, "children", 1, F.TYPE_MESSAGE, REP, ".tensorflow.TrackableObjectGraph.TrackableObject.ObjectReference")
    _field(tobj, "attributes", 2, F.TYPE_MESSAGE, REP,
           ".tensorflow.TrackableObjectGraph.TrackableObject.SerializedTensor")
    _field(tog, "nodes", 1, F.TYPE_MESSAGE, REP, ".tensorflow.TrackableObjectGraph.TrackableObject")

    # TensorBundle (tensorflow/core/protobuf/tensor_bundle.proto)
    ver = tf.message_type.add(name="VersionDef")
    _field(ver, "producer", 1, F.TYPE_INT32)
    _field(ver, "min_consumer", 2, F.TYPE_INT32)
    _field(ver, "bad_consumers", 3, F.TYPE_INT32, REP, packed=True)
    bh = tf.message_type.add(name="BundleHeaderProto")
    endian = bh.enum_type.add(name="Endianness")
    endian.value.add(name="LITTLE", number=0)
    endian.value.add(name="BIG", number=1)
    _field(bh, "num_shards", 1, F.TYPE_INT32)
    _field(bh, "endianness", 2, F.TYPE_ENUM, type_name=".tensorflow.BundleHeaderProto.Endianness")
    _field(bh, "version", 3, F.TYPE_MESSAGE, type_name=".tensorflow.VersionDef")
    be = tf.message_type.add(name="BundleEntryProto")
    _field(be, "dtype", 1, F.TYPE_ENUM, type_name=".tensorflow.DataType")
    _field(be, "shape", 2, F.TYPE_MESSAGE, type_name=".tensorflow.TensorShapeProto")
    _field(be, "shard_id", 3, F.TYPE_INT32)
    _field(be, "offset", 4, F.TYPE_INT64)
    _field(be, "size", 5, F.TYPE_INT64)
    _field(be, "crc32c", 6, F.TYPE_FIXED32)
    pool.Add(tf)

    # ---------------------------------------------------------------- tensorflow.serving
    sv = descriptor_pb2.FileDescriptorProto(name="kdl/tensorflow_serving.proto", package="tensorflow.serving",
                                            syntax="proto3", dependency=[
                                                "kdl/tensorflow_core.proto", "google/protobuf/wrappers.proto",
                                                "google/protobuf/any.proto"])
    ms = sv.message_type.add(name="ModelSpec")
    ms.oneof_decl.add(name="version_choice")
    _field(ms, "name", 1, F.TYPE_STRING)
    _field(ms, "version", 2, F.TYPE_MESSAGE, type_name=".google.protobuf.Int64Value", oneof=0)
    _field(ms, "signature_name", 3, F.TYPE_STRING)
    _field(ms, "version_label", 4, F.TYPE_STRING, oneof=0)

    pr = sv.message_type.add(name="PredictRequest")
    _field(pr, "model_spec", 1, F.TYPE_MESSAGE, type_name=".tensorflow.serving.ModelSpec")
    _map(sv, pr, "inputs", 2, F.TYPE_STRING, F.TYPE_MESSAGE, ".tensorflow.TensorProto")
    _field(pr, "output_filter", 3, F.TYPE_STRING, REP)
    prs = sv.message_type.add(name="PredictResponse")
    _map(sv, prs, "outputs", 1, F.TYPE_STRING, F.TYPE_MESSAGE, ".tensorflow.TensorProto")
    _field(prs, "model_spec", 2, F.TYPE_MESSAGE, type_name=".tensorflow.serving.ModelSpec")

    gmr = sv.message_type.add(name="GetModelMetadataRequest")
    _field(gmr, "model_spec", 1, F.TYPE_MESSAGE, type_name=".tensorflow.serving.ModelSpec")
    _field(gmr, "metadata_field", 2, F.TYPE_STRING, REP)
    gmp = sv.message_type.add(name="GetModelMetadataResponse")
    _field(gmp, "model_spec", 1, F.TYPE_MESSAGE, type_name=".tensorflow.serving.ModelSpec")
    _map(sv, gmp, "metadata", 2, F.TYPE_STRING, F.TYPE_MESSAGE, ".google.protobuf.Any")
    sdm = sv.message_type.add(name="SignatureDefMap")
    _map(sv, sdm, "signature_def", 1, F.TYPE_STRING, F.TYPE_MESSAGE, ".tensorflow.SignatureDef")

    st = sv.message_type.add(name="StatusProto")
    _field(st, "error_code", 1, F.TYPE_INT32)
    _field(st, "error_message", 2, F.TYPE_STRING)
    mvs = sv.message_type.add(name="ModelVersionStatus")
    state = mvs.enum_type.add(name="State")
    for n, v in (("UNKNOWN", 0), ("START", 10), ("LOADING", 20), ("AVAILABLE", 30), ("UNLOADING", 40),
                 ("END", 50)):
        state.value.add(name=n, number=v)
    _field(mvs, "version", 1, F.TYPE_INT64)
    _field(mvs, "state", 2, F.TYPE_ENUM, type_name=".tensorflow.serving.ModelVersionStatus.State")
    _field(mvs, "status", 3, F.TYPE_MESSAGE, type_name=".tensorflow.serving.StatusProto")
    gsr = sv.message_type.add(name="GetModelStatusRequest")
    _field(gsr, "model_spec", 1, F.TYPE_MESSAGE, type_name=".tensorflow.serving.ModelSpec")
    gsp = sv.message_type.add(name="GetModelStatusResponse")
    _field(gsp, "model_version_status", 1, F.TYPE_MESSAGE, REP, ".tensorflow.serving.ModelVersionStatus")

    rcr = sv.message_type.add(name="ReloadConfigRequest")
    _field(rcr, "config", 1, F.TYPE_BYTES)  # ModelServerConfig, opaque here
    rcp = sv.message_type.add(name="ReloadConfigResponse")
    _field(rcp, "status", 1, F.TYPE_MESSAGE, type_name=".tensorflow.serving.StatusProto")

    svc = sv.service.add(name="PredictionService")
    for mname, i, o in (("Predict", "PredictRequest", "PredictResponse"),
                        ("GetModelMetadata", "GetModelMetadataRequest", "GetModelMetadataResponse")):
        svc.method.add(name=mname, input_type=f".tensorflow.serving.{i}", output_type=f".tensorflow.serving.{o}")
    msvc = sv.service.add(name="ModelService")
    msvc.method.add(name="GetModelStatus", input_type=".tensorflow.serving.GetModelStatusRequest",
                    output_type=".tensorflow.serving.GetModelStatusResponse")
    msvc.method.add(name="HandleReloadConfigRequest", input_type=".tensorflow.serving.ReloadConfigRequest",
                    output_type=".tensorflow.serving.ReloadConfigResponse")
    pool.Add(sv)
    return pool


POOL = _build_pool()


def _cls(full_name: str):
    return message_factory.GetMessageClass(POOL.FindMessageTypeByName(full_name))


TensorShapeProto = _cls("tensorflow.TensorShapeProto")
TensorProto = _cls("tensorflow.TensorProto")
TensorInfo = _cls("tensorflow.TensorInfo")
SignatureDef = _cls("tensorflow.SignatureDef")
MetaGraphDef = _cls("tensorflow.MetaGraphDef")
SavedModel = _cls("tensorflow.SavedModel")
SavedObjectGraph = _cls("tensorflow.SavedObjectGraph")
TrackableObjectGraph = _cls("tensorflow.TrackableObjectGraph")
BundleHeaderProto = _cls("tensorflow.BundleHeaderProto")
BundleEntryProto = _cls("tensorflow.BundleEntryProto")
ModelSpec = _cls("tensorflow.serving.ModelSpec")
PredictRequest = _cls("tensorflow.serving.PredictRequest")
PredictResponse = _cls("tensorflow.serving.PredictResponse")
GetModelMetadataRequest = _cls("tensorflow.serving.GetModelMetadataRequest")
GetModelMetadataResponse = _cls("tensorflow.serving.GetModelMetadataResponse")
SignatureDefMap = _cls("tensorflow.serving.SignatureDefMap")
GetModelStatusRequest = _cls("tensorflow.serving.GetModelStatusRequest")
GetModelStatusResponse = _cls("tensorflow.serving.GetModelStatusResponse")
ModelVersionStatus = _cls("tensorflow.serving.ModelVersionStatus")
ReloadConfigRequest = _cls("tensorflow.serving.ReloadConfigRequest")
ReloadConfigResponse = _cls("tensorflow.serving.ReloadConfigResponse")

PREDICT_METHOD = "/tensorflow.serving.PredictionService/Predict"
METADATA_METHOD = "/tensorflow.serving.PredictionService/GetModelMetadata"
STATUS_METHOD = "/tensorflow.serving.ModelService/GetModelStatus"

_NP = {DT_FLOAT: "<f4", DT_DOUBLE: "<f8", DT_INT32: "<i4", DT_UINT8: "u1", DT_INT64: "<i8", DT_INT16: "<i2",
       DT_INT8: "i1", DT_BOOL: "?", DT_HALF: "<f2", DT_UINT16: "<u2"}


def np_to_tensor_proto(arr) -> "TensorProto":
    """Equivalent of ``tf.make_tensor_proto(data, shape=data.shape)`` for numeric
    arrays (model_server.py:35-36): fills ``tensor_content`` with raw LE bytes."""
    import numpy as np
    a = np.ascontiguousarray(arr)
    inv = {np.dtype(v).str: k for k, v in _NP.items()}
    key = a.dtype.newbyteorder("<").str if a.dtype.byteorder not in ("|",) else a.dtype.str
    if a.dtype == np.float32:
        dtype = DT_FLOAT
    elif a.dtype == np.uint8:
        dtype = DT_UINT8
    else:
        dtype = inv.get(key)
        if dtype is None:
            raise TypeError(f"unsupported dtype {a.dtype}")
    t = TensorProto(dtype=dtype)
    for d in a.shape:
        t.tensor_shape.dim.add(size=int(d))
    t.tensor_content = a.astype(np.dtype(_NP[dtype]), copy=False).tobytes()
    return t


def tensor_proto_to_np(t):
    """Decode a TensorProto (tensor_content or the typed *_val fields)."""
    import numpy as np
    shape = tuple(d.size for d in t.tensor_shape.dim)
    if t.dtype not in _NP:
        raise TypeError(f"unsupported dtype {DTYPE_NAMES.get(t.dtype, t.dtype)}")
    dt = np.dtype(_NP[t.dtype])
    if t.tensor_content:
        return np.frombuffer(t.tensor_content, dtype=dt).reshape(shape)
    vals = {DT_FLOAT: t.float_val, DT_DOUBLE: t.double_val, DT_INT32: t.int_val, DT_UINT8: t.int_val,
            DT_INT16: t.int_val, DT_INT8: t.int_val, DT_INT64: t.int64_val, DT_BOOL: t.bool_val,
            DT_HALF: t.half_val}[t.dtype]
    n = int(np.prod(shape)) if shape else 1
    arr = np.asarray(list(vals), dtype=dt if t.dtype != DT_HALF else np.uint16)
    if t.dtype == DT_HALF:
        arr = arr.astype(np.uint16).view(np.float16)
    if arr.size == 1 and n > 1:
        arr = np.full(n, arr[0], dtype=arr.dtype)
    return arr.reshape(shape)
