"""A kubelet stand-in: the Registration service on ``kubelet.sock`` plus a DevicePlugin client.

Used by the CPU tests (tests/fakes/kubelet.py re-exports it) and by the node bring-up rehearsal
(:mod:`.bringup`), which drives the real device plugin on a real GPU node without a cluster.
Mirrors what the real kubelet does with a device plugin: accept ``Register``, dial the plugin's
endpoint in the same directory, consume ``ListAndWatch``, call ``GetPreferredAllocation`` /
``Allocate``.  ``restart()`` reproduces a kubelet restart: every socket in the directory is
removed (kubelet's device-manager wipes the plugin directory) and kubelet.sock comes back as a new
inode, which a correct plugin must notice and re-register against.
"""
from __future__ import annotations

import os
import threading
from concurrent import futures
from typing import List

import grpc

from k8s_nvidia_gpus_amd.operator import deviceplugin_api as api


class KubeletStub:
    def __init__(self, directory: str):
        self.dir = directory
        self.socket = os.path.join(directory, api.KUBELET_SOCKET)
        self.registrations: List[api.RegisterRequest] = []
        self.registered = threading.Event()
        self._server = None

    def _register(self, request, context):
        self.registrations.append(request)
        self.registered.set()
        return api.Empty()

    def start(self) -> "KubeletStub":
        os.makedirs(self.dir, exist_ok=True)
        if os.path.exists(self.socket):
            os.unlink(self.socket)
        s = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
        s.add_generic_rpc_handlers([api.generic_handler("Registration", {"Register": self._register})])
        s.add_insecure_port(api.unix_target(self.socket))
        s.start()
        self._server = s
        return self

    def stop(self) -> None:
        if self._server is not None:
            self._server.stop(grace=0).wait()
            self._server = None

    def restart(self) -> None:
        self.stop()
        for name in os.listdir(self.dir):
            p = os.path.join(self.dir, name)
            if not os.path.isdir(p):
                os.unlink(p)
        self.registered.clear()
        self.start()

    def plugin_channel(self, index: int = -1):
        req = self.registrations[index]
        return grpc.insecure_channel(api.unix_target(os.path.join(self.dir, req.endpoint)))

    def plugin_stub(self, index: int = -1):
        ch = self.plugin_channel(index)
        grpc.channel_ready_future(ch).result(timeout=10)
        return ch, api.Stub(ch, "DevicePlugin")
