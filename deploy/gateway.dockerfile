# Serving gateway image (gateway.dockerfile:1-17). Torch-free: only the HTTP ->
# gRPC bridge, Xception preprocessing and the runtime-built TF-Serving protos.
#   docker build -f deploy/gateway.dockerfile -t model-serving:serving-gateway .
FROM python:3.10.12-slim

ENV PYTHONUNBUFFERED=TRUE

COPY deploy/requirements-gateway.lock /tmp/requirements.lock
RUN pip --no-cache-dir install --no-deps -r /tmp/requirements.lock

WORKDIR /app
COPY kdl/__init__.py kdl/labels.py ./kdl/
COPY kdl/gateway ./kdl/gateway
COPY kdl/serving/__init__.py kdl/serving/protos.py ./kdl/serving/

EXPOSE 9696

# multiple threaded workers (the reference ran gunicorn's single sync worker)
ENTRYPOINT ["gunicorn", "--bind", "0.0.0.0:9696", "--workers", "4", "--threads", "8", "kdl.gateway.wsgi:app"]
