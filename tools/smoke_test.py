#!/usr/bin/env python
"""Smoke client (reference test.py:1-16): POST {"url": ...} to the gateway and
print the JSON. Also accepts a local file (served on an ephemeral localhost
port, since bit.ly is unreachable offline) or talks gRPC to the model server
directly with --grpc.

  python tools/smoke_test.py --url http://bit.ly/mlbookcamp-pants --gateway http://localhost:9696/predict
  python tools/smoke_test.py --file tests/data/pants.png --gateway http://<elb>/predict
  python tools/smoke_test.py --file tests/data/pants.png --grpc localhost:8500
"""
from __future__ import annotations

import argparse
import http.server
import json
import os
import sys
import threading
import urllib.request

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def serve_file(path: str) -> str:
    d, name = os.path.split(os.path.abspath(path))

    class H(http.server.SimpleHTTPRequestHandler):
        def __init__(self, *a, **k):
            super().__init__(*a, directory=d, **k)

        def log_message(self, *a):
            pass
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return f"http://127.0.0.1:{srv.server_address[1]}/{name}"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", default="http://bit.ly/mlbookcamp-pants")
    ap.add_argument("--file", default=None)
    ap.add_argument("--gateway", default="http://localhost:9696/predict")
    ap.add_argument("--grpc", default=None, help="host:port of the model server (bypass the gateway)")
    a = ap.parse_args(argv)
    if a.grpc:
        import grpc
        from kdl.gateway import preprocess as pp
        from kdl.gateway.client import PredictionStub, make_request, process_response
        from kdl.labels import LABELS
        data = open(a.file, "rb").read() if a.file else pp.fetch(a.url)
        X = pp.image_to_tensor(pp.load_image(data))
        res = PredictionStub(grpc.insecure_channel(a.grpc)).Predict(make_request(X), timeout=20.0)
        print(process_response(res, LABELS))
        return 0
    url = serve_file(a.file) if a.file else a.url
    req = urllib.request.Request(a.gateway, data=json.dumps({"url": url}).encode(),
                                 headers={"Content-Type": "application/json"}, method="POST")
    with urllib.request.urlopen(req, timeout=30) as r:
        print(json.loads(r.read()))
    return 0


if __name__ == "__main__":
    sys.exit(main())
