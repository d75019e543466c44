"""Minimal Kubernetes API client for the operator's node agents (no kubernetes Python package).

Only what the labeller, partition manager and validator need: get/patch a Node, list/create/
delete/watch Pods, read pod logs.  In-cluster credentials come from the mounted ServiceAccount
(``/var/run/secrets/kubernetes.io/serviceaccount``); tests point ``base_url`` at a local fake API
server (tests/fakes/kubeapi.py).  Stdlib ``urllib`` only, so the operator image needs no extra
dependency.
"""
from __future__ import annotations

import json
import os
import ssl
import time
import urllib.error
import urllib.parse
import urllib.request
from typing import Any, Dict, List, Optional

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class KubeError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"HTTP {status}: {message}")
        self.status = status
        self.message = message


class KubeClient:
    def __init__(self, base_url: Optional[str] = None, token: Optional[str] = None,
                 ca_file: Optional[str] = None, timeout: float = 30.0):
        if base_url is None:
            host = os.environ.get("KUBERNETES_SERVICE_HOST")
            port = os.environ.get("KUBERNETES_SERVICE_PORT", "443")
            if not host:
                raise KubeError(0, "not running in a cluster (KUBERNETES_SERVICE_HOST unset) "
                                   "and no base_url given")
            base_url = f"https://{host}:{port}"
            if token is None and os.path.exists(os.path.join(SA_DIR, "token")):
                with open(os.path.join(SA_DIR, "token")) as f:
                    token = f.read().strip()
            if ca_file is None and os.path.exists(os.path.join(SA_DIR, "ca.crt")):
                ca_file = os.path.join(SA_DIR, "ca.crt")
        self.base_url = base_url.rstrip("/")
        self.token = token
        self.timeout = timeout
        self._ctx = None
        if self.base_url.startswith("https"):
            self._ctx = ssl.create_default_context(cafile=ca_file) if ca_file else ssl.create_default_context()

    # ------------------------------------------------------------------ transport
    def request(self, method: str, path: str, body: Any = None,
                content_type: str = "application/json", query: Optional[Dict[str, str]] = None,
                raw: bool = False):
        url = self.base_url + path
        if query:
            url += "?" + urllib.parse.urlencode(query)
        data = None
        headers = {"Accept": "application/json"}
        if body is not None:
            data = json.dumps(body).encode()
            headers["Content-Type"] = content_type
        if self.token:
            headers["Authorization"] = f"Bearer {self.token}"
        req = urllib.request.Request(url, data=data, method=method, headers=headers)
        try:
            with urllib.request.urlopen(req, timeout=self.timeout, context=self._ctx) as resp:
                payload = resp.read()
        except urllib.error.HTTPError as e:
            msg = e.read().decode(errors="replace")
            try:   # a Status object: keep its human-readable message
                msg = json.loads(msg).get("message") or msg
            except (ValueError, AttributeError):
                pass
            raise KubeError(e.code, msg) from None
        except urllib.error.URLError as e:
            raise KubeError(0, str(e.reason)) from None
        if raw:
            return payload.decode(errors="replace")
        return json.loads(payload) if payload else {}

    # ------------------------------------------------------------------ nodes
    def get_node(self, name: str) -> Dict[str, Any]:
        return self.request("GET", f"/api/v1/nodes/{name}")

    def patch_node(self, name: str, patch: Dict[str, Any]) -> Dict[str, Any]:
        return self.request("PATCH", f"/api/v1/nodes/{name}", patch,
                            content_type="application/merge-patch+json")

    def set_node_labels(self, name: str, labels: Dict[str, Optional[str]]) -> Dict[str, Any]:
        """Merge-patch labels; a None value deletes the label."""
        return self.patch_node(name, {"metadata": {"labels": labels}})

    def set_node_annotations(self, name: str, ann: Dict[str, Optional[str]]) -> Dict[str, Any]:
        return self.patch_node(name, {"metadata": {"annotations": ann}})

    def set_taint(self, name: str, key: str, value: str, effect: str = "NoSchedule",
                  present: bool = True) -> Dict[str, Any]:
        node = self.get_node(name)
        taints = [t for t in node.get("spec", {}).get("taints", []) or [] if t.get("key") != key]
        if present:
            taints.append({"key": key, "value": value, "effect": effect})
        # merge-patch replaces the whole list, which is what we want
        return self.patch_node(name, {"spec": {"taints": taints}})

    # ------------------------------------------------------------------ pods
    def list_pods(self, namespace: Optional[str] = None, field_selector: Optional[str] = None,
                  label_selector: Optional[str] = None) -> List[Dict[str, Any]]:
        path = f"/api/v1/namespaces/{namespace}/pods" if namespace else "/api/v1/pods"
        q = {}
        if field_selector:
            q["fieldSelector"] = field_selector
        if label_selector:
            q["labelSelector"] = label_selector
        return self.request("GET", path, query=q or None).get("items", [])

    def get_pod(self, namespace: str, name: str) -> Dict[str, Any]:
        return self.request("GET", f"/api/v1/namespaces/{namespace}/pods/{name}")

    def create_pod(self, namespace: str, pod: Dict[str, Any]) -> Dict[str, Any]:
        return self.request("POST", f"/api/v1/namespaces/{namespace}/pods", pod)

    def delete_pod(self, namespace: str, name: str) -> None:
        try:
            self.request("DELETE", f"/api/v1/namespaces/{namespace}/pods/{name}")
        except KubeError as e:
            if e.status != 404:
                raise

    def evict_pod(self, namespace: str, name: str) -> None:
        """Eviction API (policy/v1): the API server refuses with 429 while the eviction would
        violate a PodDisruptionBudget.  404 (already gone) is success."""
        body = {"apiVersion": "policy/v1", "kind": "Eviction",
                "metadata": {"name": name, "namespace": namespace}}
        try:
            self.request("POST", f"/api/v1/namespaces/{namespace}/pods/{name}/eviction", body)
        except KubeError as e:
            if e.status != 404:
                raise

    def pod_logs(self, namespace: str, name: str, container: Optional[str] = None) -> str:
        q = {"container": container} if container else None
        return self.request("GET", f"/api/v1/namespaces/{namespace}/pods/{name}/log", query=q,
                            raw=True)

    def wait_pod_phase(self, namespace: str, name: str, phases=("Succeeded", "Failed"),
                       timeout: float = 600.0, poll: float = 2.0) -> Dict[str, Any]:
        deadline = time.monotonic() + timeout
        while True:
            pod = self.get_pod(namespace, name)
            if pod.get("status", {}).get("phase") in phases:
                return pod
            if time.monotonic() >= deadline:
                raise TimeoutError(f"pod {namespace}/{name} not in {phases} after {timeout}s "
                                   f"(phase {pod.get('status', {}).get('phase')})")
            time.sleep(poll)


def pod_gpu_request(pod: Dict[str, Any], resource: str = "amd.com/gpu") -> int:
    """Sum of the pod's container limits/requests for ``resource``."""
    total = 0
    for c in pod.get("spec", {}).get("containers", []) or []:
        res = c.get("resources", {}) or {}
        v = (res.get("limits") or {}).get(resource) or (res.get("requests") or {}).get(resource)
        if v:
            total += int(v)
    return total
