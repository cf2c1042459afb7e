"""Structural checks of the k8s manifests / Dockerfiles (no cluster tooling
offline: kubectl/kind/docker are absent)."""
from pathlib import Path

import yaml

K8S = Path(__file__).resolve().parent.parent / "deploy" / "k8s"
DEPLOY = K8S.parent


def _docs(name):
    return [d for d in yaml.safe_load_all((K8S / name).read_text()) if d]


def test_model_server_deployment():
    docs = _docs("tf-serving-clothing-model-deployment.yaml")
    dep = next(d for d in docs if d["kind"] == "Deployment")
    assert dep["metadata"]["name"] == "tf-serving-clothing-model"
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert {p["containerPort"] for p in c["ports"]} == {8500, 8501}
    assert c["resources"]["limits"]["amd.com/gpu"] == 8
    assert c["readinessProbe"]["httpGet"]["path"] == "/readyz"
    assert c["livenessProbe"]["httpGet"]["path"] == "/healthz"
    env = {e["name"]: e["value"] for e in c["env"]}
    assert env["MODEL_NAME"] == "clothing-model" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    vols = {v["name"]: v for v in dep["spec"]["template"]["spec"]["volumes"]}
    assert vols["dshm"]["emptyDir"]["medium"] == "Memory"
    cm = next(d for d in docs if d["kind"] == "ConfigMap")
    from kdl.serving.config import BatchingParams
    bp = BatchingParams.parse(cm["data"]["batching.config"])
    assert bp.max_batch_size == 32 and bp.allowed_batch_sizes == [1, 2, 4, 8, 16, 32]


def test_services_match_reference_names_and_ports():
    (svc,) = _docs("tf-serving-clothing-model-service.yaml")
    assert svc["metadata"]["name"] == "tf-serving-clothing-model"
    assert svc.get("spec", {}).get("type", "ClusterIP") == "ClusterIP"
    assert {p["port"] for p in svc["spec"]["ports"]} >= {8500}
    assert svc["spec"]["selector"] == {"app": "tf-serving-clothing-model"}
    (gw,) = _docs("serving-gateway-service.yaml")
    assert gw["spec"]["type"] == "LoadBalancer"
    (p,) = gw["spec"]["ports"]
    assert (p["port"], p["targetPort"]) == (80, 9696)


def test_gateway_deployment_points_at_model_service():
    (dep,) = _docs("serving-gateway-deployment.yaml")
    c = dep["spec"]["template"]["spec"]["containers"][0]
    env = {e["name"]: e["value"] for e in c["env"]}
    assert env["TF_SERVING_HOST"] == "tf-serving-clothing-model.default.svc.cluster.local:8500"
    assert c["ports"][0]["containerPort"] == 9696


def test_dockerfiles():
    ms = (DEPLOY / "model-server.dockerfile").read_text()
    assert "MODEL_NAME=clothing-model" in ms and "/models/clothing-model/1" in ms and "kdl.serving" in ms
    gw = (DEPLOY / "gateway.dockerfile").read_text()
    assert "gunicorn" in gw and "9696" in gw and "kdl.gateway.wsgi:app" in gw


def test_images_and_dependencies_are_pinned():
    """Like the reference's Pipfile.lock (Pipfile:8-17): no floating base tags, every pip
    dependency pinned to an exact version, and the lock files cover what the code imports."""
    import re
    for name, lock in (("model-server.dockerfile", "requirements-model-server.lock"),
                       ("gateway.dockerfile", "requirements-gateway.lock")):
        df = (DEPLOY / name).read_text()
        base = re.search(r"^FROM\s+(\S+)", df, re.M).group(1)
        assert ":" in base and not base.endswith(":latest"), base
        assert f"deploy/{lock}" in df and "--no-deps -r" in df
        pins = [ln.strip() for ln in (DEPLOY / lock).read_text().splitlines()
                if ln.strip() and not ln.startswith("#")]
        assert pins and all(re.fullmatch(r"[A-Za-z0-9_.\-]+==[0-9][0-9A-Za-z.+\-]*", p) for p in pins), pins
        names = {p.split("==")[0].lower() for p in pins}
        need = {"grpcio", "protobuf", "numpy", "pillow"} | ({"flask", "gunicorn", "werkzeug"} if "gateway" in name
                                                            else {"safetensors"})
        assert need <= names, need - names
