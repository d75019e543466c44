"""A fake Kubernetes API server (nodes + pods, merge-patch, pod logs) on 127.0.0.1.

Enough of the API for the node agents: GET/PATCH /api/v1/nodes/<n> (JSON merge patch, RFC 7386),
GET/POST/DELETE pods (namespaced and cluster-wide list with spec.nodeName / status.phase field
selectors), GET pod logs, POST pods/<n>/eviction (429 for pods in ``pdb_blocked``).  ``on_pod_created`` lets a test play kubelet (e.g. mark the validator's
plugin-test pod Succeeded with a log).
"""
from __future__ import annotations

import copy
import json
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable, Dict, Optional


def merge_patch(target, patch):
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    out = dict(target) if isinstance(target, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


class FakeKubeAPI:
    def __init__(self):
        self.nodes: Dict[str, dict] = {}
        self.pods: Dict[tuple, dict] = {}
        self.logs: Dict[tuple, str] = {}
        self.requests = []
        self.on_pod_created: Optional[Callable[["FakeKubeAPI", dict], None]] = None
        # (namespace, name) -> message: evictions of these pods are refused (PDB, HTTP 429)
        self.pdb_blocked: Dict[tuple, str] = {}
        self.evictions = []
        self._lock = threading.Lock()
        self._server = None

    def add_node(self, name: str, labels=None) -> None:
        self.nodes[name] = {"metadata": {"name": name, "labels": dict(labels or {}),
                                         "annotations": {}}, "spec": {}, "status": {}}

    def add_pod(self, namespace: str, name: str, node: str, gpus: int = 0, phase="Running") -> None:
        res = {"limits": {"amd.com/gpu": str(gpus)}} if gpus else {}
        self.pods[(namespace, name)] = {
            "metadata": {"name": name, "namespace": namespace},
            "spec": {"nodeName": node, "containers": [{"name": "c", "resources": res}]},
            "status": {"phase": phase}}

    @property
    def url(self) -> str:
        host, port = self._server.server_address
        return f"http://{host}:{port}"

    def start(self) -> "FakeKubeAPI":
        api = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):  # silence
                pass

            def _send(self, code, obj=None, raw=None):
                body = raw.encode() if raw is not None else json.dumps(obj or {}).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def _body(self):
                n = int(self.headers.get("Content-Length") or 0)
                return json.loads(self.rfile.read(n)) if n else None

            def _route(self, method):
                u = urllib.parse.urlparse(self.path)
                q = dict(urllib.parse.parse_qsl(u.query))
                parts = [p for p in u.path.split("/") if p]
                api.requests.append((method, u.path, q))
                with api._lock:
                    return api._handle(method, parts, q, self._body() if method in ("POST", "PATCH") else None)

            def do_GET(self):
                self._reply(self._route("GET"))

            def do_PATCH(self):
                self._reply(self._route("PATCH"))

            def do_POST(self):
                self._reply(self._route("POST"))

            def do_DELETE(self):
                self._reply(self._route("DELETE"))

            def _reply(self, r):
                code, obj, raw = r
                self._send(code, obj, raw)

        self._server = ThreadingHTTPServer(("127.0.0.1", 0), H)
        threading.Thread(target=self._server.serve_forever, daemon=True).start()
        return self

    def stop(self):
        if self._server:
            self._server.shutdown()
            self._server.server_close()

    # ----------------------------------------------------------------- routing
    def _handle(self, method, parts, q, body):
        if parts == ["api", "v1", "nodes"] and method == "GET":
            sel = [c.split("=", 1) for c in q.get("labelSelector", "").split(",") if "=" in c]
            items = [n for n in self.nodes.values()
                     if all(n["metadata"].get("labels", {}).get(k) == v for k, v in sel)]
            return 200, {"items": items}, None
        # /api/v1/nodes/<name>
        if parts[:3] == ["api", "v1", "nodes"] and len(parts) == 4:
            name = parts[3]
            if name not in self.nodes:
                return 404, {"message": "node not found"}, None
            if method == "GET":
                return 200, self.nodes[name], None
            if method == "PATCH":
                self.nodes[name] = merge_patch(self.nodes[name], body)
                return 200, self.nodes[name], None
        if parts[:3] == ["api", "v1", "pods"] and method == "GET":
            return 200, {"items": self._select(None, q)}, None
        if parts[:3] == ["api", "v1", "namespaces"] and len(parts) >= 5 and parts[4] == "pods":
            ns = parts[3]
            if len(parts) == 5:
                if method == "GET":
                    return 200, {"items": self._select(ns, q)}, None
                if method == "POST":
                    pod = copy.deepcopy(body)
                    pod.setdefault("metadata", {})["namespace"] = ns
                    name = pod["metadata"].get("name") or pod["metadata"].get("generateName", "p") + str(len(self.pods))
                    pod["metadata"]["name"] = name
                    pod.setdefault("status", {})["phase"] = "Pending"
                    self.pods[(ns, name)] = pod
                    if self.on_pod_created:
                        self.on_pod_created(self, pod)
                    return 201, pod, None
            name = parts[5]
            key = (ns, name)
            if key not in self.pods:
                return 404, {"message": "pod not found"}, None
            if len(parts) == 7 and parts[6] == "log":
                return 200, None, self.logs.get(key, "")
            if len(parts) == 7 and parts[6] == "eviction" and method == "POST":
                if body.get("kind") != "Eviction" or body.get("metadata", {}).get("name") != name:
                    return 400, {"message": "bad Eviction body"}, None
                if key in self.pdb_blocked:
                    return 429, {"message": self.pdb_blocked[key]}, None
                self.evictions.append(key)
                self.pods.pop(key)
                return 201, {"status": "Success"}, None
            if method == "GET":
                return 200, self.pods[key], None
            if method == "DELETE":
                self.pods.pop(key)
                return 200, {}, None
        return 404, {"message": f"no route {method} {'/'.join(parts)}"}, None

    def _select(self, ns, q):
        out = []
        conds = []
        for c in q.get("fieldSelector", "").split(","):
            if "!=" in c:
                k, v = c.split("!=", 1)
                conds.append((k, v, True))
            elif "=" in c:
                k, v = c.split("=", 1)
                conds.append((k.rstrip("="), v, False))
        get = {"spec.nodeName": lambda p: p["spec"].get("nodeName"),
               "status.phase": lambda p: p["status"].get("phase")}
        for (pns, _), pod in self.pods.items():
            if ns and pns != ns:
                continue
            if all((get[k](pod) != v) if neg else (get[k](pod) == v) for k, v, neg in conds):
                out.append(pod)
        return out
