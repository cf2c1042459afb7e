# MI355X model server image (replaces `FROM tensorflow/serving:2.3.0`, tf-serving.dockerfile:1-5).
# Base: ROCm 7 + PyTorch-ROCm. Build from the repo root:
#   docker build -f deploy/model-server.dockerfile -t model-serving:kdl-model-server .
FROM rocm/pytorch:latest

ENV PYTHONUNBUFFERED=TRUE \
    HSA_ENABLE_IPC_MODE_LEGACY=0 \
    PYTORCH_ROCM_ARCH=gfx950 \
    MODEL_NAME=clothing-model \
    MODEL_BASE_PATH=/models

RUN pip --no-cache-dir install grpcio protobuf safetensors pillow numpy

WORKDIR /opt/kdl
COPY kdl ./kdl
COPY __graft_entry__.py ./
# compile the gfx950 HIP kernels + native executor (kdl/_C) and CPU runtime (kdl/_rt) in-tree
RUN python -m kdl.csrc.build && python -c "import torch, kdl._C, kdl._rt"

# the SavedModel produced by tools/convert.py (or converted by `kdl convert-savedmodel`)
COPY clothing-model /models/clothing-model/1

EXPOSE 8500 8501
# same flags/env contract as tensorflow_model_server's entrypoint
ENTRYPOINT ["python", "-m", "kdl.serving", "--port=8500", "--rest_api_port=8501"]
