"""GPU-client pause protocol around a compute/memory partition switch.

Changing an MI355X's partition mode needs the device quiet: no process may hold ``/dev/kfd`` or a
DRM node of the ASIC, or the sysfs write returns EBUSY.  Besides the drained workload pods, the
operator itself has long-lived GPU clients on every node:

* the metrics exporter (an amd-smi session, ``exporter.py``),
* the driver-readiness loop (``kfd-probe`` opens ``/dev/kfd`` and every render node per probe),
* the device plugin (an amd-smi session for its ECC health criterion),
* the validator (load steps run native tools on the GPUs).

The partition manager writes ``/run/amd/partition-in-progress`` (a JSON ``{"nonce": ...}``; the
device plugin already advertises no devices while it exists).  Each client, on seeing it, drops
its GPU handles and writes ``<ackDir>/<component>`` containing the nonce; the manager applies the
new mode once every expected component has acked (or ``pauseAckSeconds`` passed — the apply then
still retries EBUSY with backoff).  When the marker goes away the clients re-open (re-enumerated)
handles.  A marker from an older manager that holds only a timestamp is treated as its own nonce.
"""
from __future__ import annotations

import json
import logging
import os
import time
from typing import Dict, Iterable, Optional

log = logging.getLogger("amd-gpu-pause")

PAUSE_MARKER = "/run/amd/partition-in-progress"
ACK_DIR = "/run/amd/partition-pause-acks"
COMPONENTS = ("exporter", "driver", "device-plugin")


def read_nonce(marker: str = PAUSE_MARKER) -> Optional[str]:
    """The pause marker's nonce, or None when no pause is in progress."""
    try:
        with open(marker) as f:
            text = f.read().strip()
    except OSError:
        return None
    try:
        doc = json.loads(text)
        if isinstance(doc, dict) and doc.get("nonce"):
            return str(doc["nonce"])
    except ValueError:
        pass
    return text or "paused"


class PauseGuard:
    """One GPU client's side of the protocol: ``paused()`` / ``ack()`` / ``clear()``."""

    def __init__(self, component: str, marker: str = PAUSE_MARKER, ack_dir: str = ACK_DIR):
        self.component = component
        self.marker = marker
        self.ack_dir = ack_dir
        self._acked: Optional[str] = None

    def nonce(self) -> Optional[str]:
        return read_nonce(self.marker)

    def paused(self) -> bool:
        return self.nonce() is not None

    def ack(self) -> None:
        """Call after every GPU handle of this component is closed."""
        n = self.nonce()
        if n is None or n == self._acked:
            return
        try:
            os.makedirs(self.ack_dir, exist_ok=True)
            path = os.path.join(self.ack_dir, self.component)
            with open(path + ".tmp", "w") as f:
                f.write(n + "\n")
            os.replace(path + ".tmp", path)
            self._acked = n
            log.info("%s: GPU handles released for partition change %s", self.component, n)
        except OSError as e:
            log.warning("%s: cannot ack pause: %s", self.component, e)

    def clear(self) -> None:
        self._acked = None


def start_pause(marker: str = PAUSE_MARKER, ack_dir: str = ACK_DIR) -> str:
    """Write the marker with a fresh nonce (stale acks of an older pause no longer match)."""
    nonce = f"{os.getpid()}-{time.time_ns()}"
    os.makedirs(os.path.dirname(marker) or ".", exist_ok=True)
    with open(marker + ".tmp", "w") as f:
        json.dump({"nonce": nonce, "time": time.time()}, f)
    os.replace(marker + ".tmp", marker)
    return nonce


def end_pause(marker: str = PAUSE_MARKER) -> None:
    try:
        os.unlink(marker)
    except FileNotFoundError:
        pass


def acks(nonce: str, ack_dir: str = ACK_DIR, components: Iterable[str] = COMPONENTS) -> Dict[str, bool]:
    out = {}
    for c in components:
        try:
            with open(os.path.join(ack_dir, c)) as f:
                out[c] = f.read().strip() == nonce
        except OSError:
            out[c] = False
    return out
