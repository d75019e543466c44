"""Per-rank GPU telemetry (gfx clock, socket power, hotspot temperature) over a timed window.

A flat or sagging weak-scaling curve on an 8-GPU node has two usual explanations that the timing
alone cannot separate: the chip holding a lower clock under a power cap when all eight boards draw
at once (MI355X_MICROARCH.md "DVFS give-back"), or a slow rank.  ``bench.py`` therefore samples its
own GPU through amd-smi while the timed steps run and reports, per rank, the mean / min gfx clock,
mean power and max hotspot temperature next to that rank's TFLOPS.

The rank's GPU is matched to its amd-smi handle by PCI address (torch's device properties), never by
index: amd-smi and HIP may enumerate in different orders.  Sampling is best-effort — without the
amdsmi module (CPU runs, or an image without it) :class:`Sampler` reports ``None``.
"""
from __future__ import annotations

import statistics
import threading
from typing import Dict, List, Optional


def device_bdf(index: int) -> Optional[str]:
    import torch

    try:
        p = torch.cuda.get_device_properties(index)
        return "%04x:%02x:%02x.0" % (int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id))
    except (AttributeError, RuntimeError, AssertionError):
        return None


def _num(v):
    try:
        f = float(v)
    except (TypeError, ValueError):
        return None
    return None if f in (0xFFFF, 0xFFFFFFFF) or f != f else f


class Sampler:
    """``with Sampler(bdf) as s: ...`` then ``s.summary()``; samples every ``period`` seconds."""

    def __init__(self, bdf: Optional[str], period: float = 0.02, amdsmi_module=None):
        self.bdf = (bdf or "").lower()
        self.period = period
        self.rows: List[Dict[str, Optional[float]]] = []
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.S = None
        self.handle = None
        self.error: Optional[str] = None
        try:
            if amdsmi_module is None:
                import amdsmi as amdsmi_module  # noqa: N813 - optional dependency
            amdsmi_module.amdsmi_init()
            self.S = amdsmi_module
            for h in amdsmi_module.amdsmi_get_processor_handles():
                if str(amdsmi_module.amdsmi_get_gpu_device_bdf(h)).lower() == self.bdf:
                    self.handle = h
                    break
            if self.handle is None:
                self.error = f"no amd-smi handle for {self.bdf or '?'}"
        except Exception as e:  # noqa: BLE001 - telemetry never fails the benchmark
            self.error = f"amdsmi unavailable: {e}"[:200]

    def sample(self) -> None:
        m = self.S.amdsmi_get_gpu_metrics_info(self.handle) or {}
        self.rows.append({
            "gfxclk_mhz": _num(m.get("current_gfxclk")),
            "power_w": _num(m.get("current_socket_power")) or _num(m.get("average_socket_power")),
            "temp_hotspot_c": _num(m.get("temperature_hotspot")),
        })

    def _run(self) -> None:
        while not self._stop.is_set():
            try:
                self.sample()
            except Exception as e:  # noqa: BLE001
                self.error = f"sample failed: {e}"[:200]
                return
            self._stop.wait(self.period)

    def __enter__(self) -> "Sampler":
        if self.handle is not None:
            self._thread = threading.Thread(target=self._run, name="gpu-telemetry", daemon=True)
            self._thread.start()
        return self

    def __exit__(self, *exc) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(2.0)
        try:
            if self.S is not None:
                self.S.amdsmi_shut_down()
        except Exception:  # noqa: BLE001
            pass

    def summary(self) -> Optional[Dict[str, Optional[float]]]:
        if not self.rows:
            return {"error": self.error} if self.error else None

        def col(k):
            return [r[k] for r in self.rows if r.get(k) is not None]

        clk, pw, tmp = col("gfxclk_mhz"), col("power_w"), col("temp_hotspot_c")
        return {
            "bdf": self.bdf, "samples": len(self.rows),
            "gfxclk_mhz_mean": round(statistics.fmean(clk), 1) if clk else None,
            "gfxclk_mhz_min": min(clk) if clk else None,
            "power_w_mean": round(statistics.fmean(pw), 1) if pw else None,
            "power_w_max": max(pw) if pw else None,
            "temp_hotspot_c_max": max(tmp) if tmp else None,
        }


def timed(period: float = 0.02, device_index: Optional[int] = None):
    """A Sampler for this process's GPU (``device_index`` or the current device)."""
    import torch

    if device_index is None:
        device_index = torch.cuda.current_device() if torch.cuda.is_available() else -1
    bdf = device_bdf(device_index) if device_index >= 0 else None
    return Sampler(bdf, period)

