# MI355X model server image (replaces `FROM tensorflow/serving:2.3.0`, tf-serving.dockerfile:1-5).
# Base: ROCm 7 + PyTorch-ROCm. Build from the repo root:
#   docker build -f deploy/model-server.dockerfile -t model-serving:kdl-model-server .
# pinned base (ROCm 7.2 runtime, PyTorch 2.10.0+rocm7.0, Python 3.10) -- the environment every
# test and benchmark in this repo ran in; never a floating tag
FROM rocm/pytorch:rocm7.2_ubuntu22.04_py3.10_pytorch_release_2.10.0

ENV PYTHONUNBUFFERED=TRUE \
    HSA_ENABLE_IPC_MODE_LEGACY=0 \
    PYTORCH_ROCM_ARCH=gfx950 \
    MODEL_NAME=clothing-model \
    MODEL_BASE_PATH=/models

# libnghttp2: HTTP/2 of the native gRPC front-end (kdl/csrc/runtime/h2.cpp dlopens it; without it
# the server falls back to grpcio)
RUN apt-get update && apt-get install -y --no-install-recommends libnghttp2-14 && rm -rf /var/lib/apt/lists/*
COPY deploy/requirements-model-server.lock /tmp/requirements.lock
RUN pip --no-cache-dir install --no-deps -r /tmp/requirements.lock

WORKDIR /opt/kdl
COPY kdl ./kdl
COPY __graft_entry__.py ./
# compile the gfx950 HIP kernels + native executor (kdl/_C) and CPU runtime (kdl/_rt) in-tree
RUN python -m kdl.csrc.build && python -c "import torch, kdl._C, kdl._rt; assert kdl._rt.http2_available()[0]"

# the SavedModel produced by tools/convert.py (or converted by `kdl convert-savedmodel`)
COPY clothing-model /models/clothing-model/1

EXPOSE 8500 8501
# same flags/env contract as tensorflow_model_server's entrypoint
ENTRYPOINT ["python", "-m", "kdl.serving", "--port=8500", "--rest_api_port=8501"]
