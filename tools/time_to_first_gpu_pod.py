#!/usr/bin/env python3
"""Measure time-to-first-GPU-pod (the second half of BASELINE.json's headline metric).

From a start time (``--since`` epoch, e.g. taken just before ``kubectl apply -k
cluster-config/cluster/flux-system/``; default: now) to
  1. the first node labelled ``amd.com/gpu.validated=true`` by the operator's validator, and
  2. the first pod requesting ``amd.com/gpu: 1`` that completes the HIP vectorAdd protocol
     ("Test PASSED" / "Done", reference README.md:292-299) through the device plugin.

Talks to the API through ``kubectl proxy`` (started automatically) or ``--api URL``.  Prints one
JSON line.  The reference has no such measurement; its driver build alone is budgeted 90 minutes
(reference gpu-operator/helmrelease.yaml:7).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from k8s_nvidia_gpus_amd.operator.validator import protocol_passed  # noqa: E402
from k8s_nvidia_gpus_amd.utils.kube import KubeClient  # noqa: E402


def wait_validated_node(kube: KubeClient, timeout: float, poll: float) -> str:
    deadline = time.time() + timeout
    while time.time() < deadline:
        nodes = kube.request("GET", "/api/v1/nodes",
                             query={"labelSelector": "amd.com/gpu.validated=true"}).get("items", [])
        if nodes:
            return nodes[0]["metadata"]["name"]
        time.sleep(poll)
    raise TimeoutError("no node reached amd.com/gpu.validated=true")


def run_gpu_pod(kube: KubeClient, namespace: str, image: str, timeout: float, poll: float) -> dict:
    name = f"ttfgp-{int(time.time())}"
    pod = {"apiVersion": "v1", "kind": "Pod",
           "metadata": {"name": name, "namespace": namespace},
           "spec": {"restartPolicy": "Never", "runtimeClassName": "amd",
                    "containers": [{"name": "vectoradd", "image": image,
                                    "command": ["/opt/amd-gpu-operator/bin/amd-vectoradd"],
                                    "resources": {"limits": {"amd.com/gpu": "1"}}}]}}
    kube.create_pod(namespace, pod)
    try:
        done = kube.wait_pod_phase(namespace, name, timeout=timeout, poll=poll)
        logs = kube.pod_logs(namespace, name)
    finally:
        kube.delete_pod(namespace, name)
    return {"phase": done.get("status", {}).get("phase"), "passed": protocol_passed(logs)}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--since", type=float, default=None, help="start epoch seconds (default: now)")
    ap.add_argument("--api", default=None, help="API base URL (default: start kubectl proxy)")
    ap.add_argument("--namespace", default="gpu-bench")
    ap.add_argument("--image", default="ghcr.io/example-org/amd-gpu-bench:0.1.0")
    ap.add_argument("--timeout", type=float, default=3600)
    ap.add_argument("--poll", type=float, default=2.0)
    args = ap.parse_args(argv)
    t0 = args.since or time.time()
    proxy = None
    api = args.api
    if api is None:
        proxy = subprocess.Popen(["kubectl", "proxy", "--port=8011"], stdout=subprocess.DEVNULL,
                                 stderr=subprocess.DEVNULL)
        api = "http://127.0.0.1:8011"
        time.sleep(1.0)
    try:
        kube = KubeClient(base_url=api)
        node = wait_validated_node(kube, args.timeout, args.poll)
        t_valid = time.time() - t0
        res = run_gpu_pod(kube, args.namespace, args.image, args.timeout, args.poll)
        t_pod = time.time() - t0
    finally:
        if proxy is not None:
            proxy.terminate()
    out = {"metric": "time_to_first_gpu_pod_s", "node": node,
           "time_to_validated_node_s": round(t_valid, 2),
           "time_to_first_gpu_pod_s": round(t_pod, 2), "pod_phase": res["phase"],
           "passed": res["passed"] and res["phase"] == "Succeeded"}
    print(json.dumps(out))
    return 0 if out["passed"] else 1


if __name__ == "__main__":
    sys.exit(main())
