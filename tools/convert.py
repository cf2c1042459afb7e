#!/usr/bin/env python
"""Keras .h5 -> TF SavedModel, same API as the reference (convert.py:1-7).

Requires TensorFlow (not available in this environment; kept for users who have
it). The produced directory is served as-is by `python -m kdl.serving`, or
packed once into BN-folded bf16 safetensors with
`python -m kdl.cli convert-savedmodel clothing-model out/1`.
"""
import sys

try:
    import tensorflow as tf
    from tensorflow import keras
except ImportError:  # pragma: no cover
    sys.exit("tools/convert.py needs TensorFlow; use `python -m kdl.cli` for TF-free steps")

src = sys.argv[1] if len(sys.argv) > 1 else "xception_v4_large_08_0.894.h5"
dst = sys.argv[2] if len(sys.argv) > 2 else "clothing-model"
model = keras.models.load_model(src)
tf.saved_model.save(model, dst)
