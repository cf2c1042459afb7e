"""SavedModel ingest without TensorFlow.

The reference produces ``clothing-model/`` with ``tf.saved_model.save``
(`convert.py:6`) and inspects it with ``saved_model_cli`` (`guide.md:202-235`).
This module reads the same directory:

* ``saved_model.pb`` -> the ``serve`` MetaGraphDef and its ``signature_def``
  map (``serving_default``: ``input_8`` f32[-1,299,299,3] -> ``dense_7`` f32[-1,10]);
* ``variables/variables.{index,data-*}`` -> every variable, named by the
  ``full_name`` recorded in the checkpoint's ``_CHECKPOINTABLE_OBJECT_GRAPH``
  (e.g. ``block1_conv1/kernel``), falling back to the checkpoint key;
* :func:`kdl.ingest.keras_map.to_xception_params` then maps those names onto the
  framework's Keras-layout parameter dict (auto-named residual convs/BNs are
  matched by graph order + shape).

``show()`` prints a ``saved_model_cli show --all``-style summary.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

from ..serving import protos as P
from .tensorbundle import TensorBundle, write_bundle

OBJECT_GRAPH_KEY = "_CHECKPOINTABLE_OBJECT_GRAPH"
VAR_SUFFIX = "/.ATTRIBUTES/VARIABLE_VALUE"


@dataclass
class TensorSpec:
    key: str
    name: str
    dtype: int
    shape: tuple[int, ...]          # -1 for unknown dims


@dataclass
class Signature:
    name: str
    method_name: str
    inputs: dict[str, TensorSpec] = field(default_factory=dict)
    outputs: dict[str, TensorSpec] = field(default_factory=dict)


def _spec(key, ti) -> TensorSpec:
    shape = tuple(int(d.size) for d in ti.tensor_shape.dim) if not ti.tensor_shape.unknown_rank else ()
    return TensorSpec(key=key, name=ti.name, dtype=int(ti.dtype), shape=shape)


class SavedModelDir:
    def __init__(self, path: str | Path, tags: tuple[str, ...] = ("serve",)):
        self.path = Path(path)
        pb = self.path / "saved_model.pb"
        if not pb.exists():
            raise FileNotFoundError(f"{pb} not found")
        sm = P.SavedModel.FromString(pb.read_bytes())
        self.schema_version = sm.saved_model_schema_version
        mg = None
        for m in sm.meta_graphs:
            if set(tags) <= set(m.meta_info_def.tags):
                mg = m
                break
        if mg is None:
            raise ValueError(f"no MetaGraphDef with tags {tags} in {pb}")
        self.meta_graph = mg
        self.signatures: dict[str, Signature] = {}
        for name, sd in mg.signature_def.items():
            sig = Signature(name=name, method_name=sd.method_name)
            for k, ti in sd.inputs.items():
                sig.inputs[k] = _spec(k, ti)
            for k, ti in sd.outputs.items():
                sig.outputs[k] = _spec(k, ti)
            self.signatures[name] = sig
        self._bundle: TensorBundle | None = None

    @property
    def bundle(self) -> TensorBundle:
        if self._bundle is None:
            self._bundle = TensorBundle(self.path / "variables" / "variables")
        return self._bundle

    def variable_names(self) -> dict[str, str]:
        """full variable name -> checkpoint key."""
        b = self.bundle
        names: dict[str, str] = {}
        if OBJECT_GRAPH_KEY in b.entries:
            raw = b.raw(OBJECT_GRAPH_KEY)
            tog = P.TrackableObjectGraph.FromString(_string_tensor_payload(raw))
            for node in tog.nodes:
                for attr in node.attributes:
                    if attr.checkpoint_key in b.entries and attr.full_name:
                        names[attr.full_name.split(":")[0]] = attr.checkpoint_key
        if not names:  # fall back to raw checkpoint keys
            for k in b.keys():
                if k != OBJECT_GRAPH_KEY:
                    names[k[:-len(VAR_SUFFIX)] if k.endswith(VAR_SUFFIX) else k] = k
        return names

    def variables(self) -> dict[str, np.ndarray]:
        b = self.bundle
        return {name: b.get(key) for name, key in self.variable_names().items()}

    def show(self) -> str:
        lines = [f"MetaGraphDef with tag-set: '{','.join(self.meta_graph.meta_info_def.tags)}' "
                 "contains the following SignatureDefs:", ""]
        for name, sig in sorted(self.signatures.items()):
            lines.append(f"signature_def['{name}']:")
            lines.append("  The given SavedModel SignatureDef contains the following input(s):")
            for k, s in sig.inputs.items():
                lines += [f"    inputs['{k}'] tensor_info:", f"        dtype: {P.DTYPE_NAMES.get(s.dtype, s.dtype)}",
                          f"        shape: {_fmt_shape(s.shape)}", f"        name: {s.name}"]
            lines.append("  The given SavedModel SignatureDef contains the following output(s):")
            for k, s in sig.outputs.items():
                lines += [f"    outputs['{k}'] tensor_info:", f"        dtype: {P.DTYPE_NAMES.get(s.dtype, s.dtype)}",
                          f"        shape: {_fmt_shape(s.shape)}", f"        name: {s.name}"]
            lines.append(f"  Method name is: {sig.method_name}")
            lines.append("")
        return "\n".join(lines)


def _fmt_shape(shape) -> str:
    if not shape:
        return "unknown_rank"
    return "(" + ", ".join(str(d) for d in shape) + ("," if len(shape) == 1 else "") + ")"


def _string_tensor_payload(raw: bytes) -> bytes:
    """A scalar DT_STRING tensor in a bundle is stored as [varint len][crc?]..[bytes];
    TF writes: varint lengths for all elements, a masked crc32c of the lengths (4 B),
    then the bytes. Accept both that and a bare payload."""
    n, i = 0, 0
    s = 0
    while True:
        c = raw[i]
        i += 1
        n |= (c & 0x7F) << s
        if not c & 0x80:
            break
        s += 7
    if i + 4 + n == len(raw):
        return raw[i + 4:]
    if i + n == len(raw):
        return raw[i:]
    return raw


def write_savedmodel(path: str | Path, variables: dict[str, np.ndarray], input_key: str = "input_8",
                     output_key: str = "dense_7", input_shape=(-1, 299, 299, 3), output_shape=(-1, 10),
                     compress: bool = False, with_object_graph: bool = True,
                     extra_signatures: dict | None = None) -> Path:
    """Write a minimal TF2-style SavedModel (fixture generator for tests/tools).

    Variables are stored under object-based checkpoint keys
    (``layer_with_weights-i/<var>/.ATTRIBUTES/VARIABLE_VALUE``) with a
    TrackableObjectGraph recording each variable's full name, as TF does."""
    path = Path(path)
    (path / "variables").mkdir(parents=True, exist_ok=True)
    sm = P.SavedModel(saved_model_schema_version=1)
    mg = sm.meta_graphs.add()
    mg.meta_info_def.tags.append("serve")
    mg.meta_info_def.tensorflow_version = "2.3.0"
    sigs = {"serving_default": ({input_key: (P.DT_FLOAT, input_shape)}, {output_key: (P.DT_FLOAT, output_shape)})}
    sigs.update(extra_signatures or {})
    for name, (ins, outs) in sigs.items():
        sd = mg.signature_def[name]
        sd.method_name = "tensorflow/serving/predict"
        for k, (dt, shp) in ins.items():
            ti = sd.inputs[k]
            ti.name = f"{name}_{k}:0"
            ti.dtype = dt
            for d in shp:
                ti.tensor_shape.dim.add(size=d)
        for k, (dt, shp) in outs.items():
            ti = sd.outputs[k]
            ti.name = "StatefulPartitionedCall:0"
            ti.dtype = dt
            for d in shp:
                ti.tensor_shape.dim.add(size=d)
    (path / "saved_model.pb").write_bytes(sm.SerializeToString())
    layers: dict[str, list[str]] = {}
    for full in variables:
        layer, var = full.rsplit("/", 1)
        layers.setdefault(layer, []).append(var)
    tensors, tog = {}, P.TrackableObjectGraph()
    root = tog.nodes.add()
    for i, layer in enumerate(layers):
        lnode_id = len(tog.nodes)
        root.children.add(node_id=lnode_id, local_name=f"layer_with_weights-{i}")
        lnode = tog.nodes.add()
        for var in layers[layer]:
            key = f"layer_with_weights-{i}/{var}{VAR_SUFFIX}"
            tensors[key] = np.asarray(variables[f"{layer}/{var}"], dtype=np.float32)
            vid = len(tog.nodes)
            lnode.children.add(node_id=vid, local_name=var)
            vnode = tog.nodes.add()
            vnode.attributes.add(name="VARIABLE_VALUE", full_name=f"{layer}/{var}", checkpoint_key=key)
    extra = {}
    if with_object_graph:
        payload = tog.SerializeToString()
        from .tensorbundle import _put_varint, _crc32c_py, mask_crc
        lens = _put_varint(len(payload))
        extra[OBJECT_GRAPH_KEY] = lens + mask_crc(_crc32c_py(lens)).to_bytes(4, "little") + payload
    write_bundle(path / "variables" / "variables", tensors, compress=compress, extra_entries=extra)
    return path
