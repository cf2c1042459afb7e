"""Class labels of the clothing model in output-unit order (`model_server.py:21-32`,
Keras ``flow_from_directory`` alphabetical order). Torch-free so the gateway
image does not need torch."""
LABELS = ["dress", "hat", "longsleeve", "outwear", "pants",
          "shirt", "shoes", "shorts", "skirt", "t-shirt"]
