"""Fake kubelet PodResources v1 server on a unix socket (what the validator queries)."""
from __future__ import annotations

import os
from concurrent import futures
from typing import Dict, List, Tuple

import grpc

from k8s_nvidia_gpus_amd.operator import podresources_api as api


class FakePodResources:
    """``pods``: {(namespace, name): [(resource_name, [device ids]), ...]}."""

    def __init__(self, socket_path: str, pods: Dict[Tuple[str, str], List[Tuple[str, List[str]]]]):
        self.socket_path = socket_path
        self.pods = pods
        self.calls = 0
        self.server = None

    def List(self, request, context):  # noqa: N802 - gRPC method name
        self.calls += 1
        resp = api.ListPodResourcesResponse()
        for (ns, name), devs in self.pods.items():
            pr = resp.pod_resources.add(name=name, namespace=ns)
            c = pr.containers.add(name="main")
            for res, ids in devs:
                c.devices.add(resource_name=res, device_ids=list(ids))
        return resp

    def __enter__(self):
        os.makedirs(os.path.dirname(self.socket_path), exist_ok=True)
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
        self.server.add_generic_rpc_handlers((api.generic_handler({"List": self.List}),))
        self.server.add_insecure_port("unix://" + self.socket_path)
        self.server.start()
        return self

    def __exit__(self, *exc):
        self.server.stop(0)
