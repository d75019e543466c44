"""GPU metrics exporter (SURVEY.md §2.2 X5 — the dcgm-exporter role) for Prometheus on :9400.

The reference gets GPU metrics only implicitly, from the GPU Operator's default DCGM exporter, and
installs no Prometheus (SURVEY.md §5 "Metrics"); its own observability is Flux's JSON logs and
scrape annotations.  This exporter reads each MI355X through amd-smi (``amdsmi`` Python bindings
over libamd_smi) and falls back to plain DRM sysfs when amd-smi is unavailable.  One
``amdsmi_get_gpu_metrics_info`` call per GPU per scrape returns the firmware metrics table
(temperatures, activity, socket power, clocks, per-link xGMI byte accumulators and link state,
PCIe link speed / width / bandwidth and replay / recovery / NAK accumulators, power-throttle
residency), so a scrape costs 8 ioctls, not 8 × 15.  The validator's measured
results (bf16 GEMM TFLOPS per GPU, RCCL all-reduce bus bandwidth, pass/fail per step) are exported
from /run/amd/validations so they can be graphed and alerted on like any other GPU metric.

Endpoints: ``/metrics`` (Prometheus text), ``/healthz``.
"""
from __future__ import annotations

import glob
import json
import logging
import os
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, Iterable, List, Optional

from ..utils import topology as topo_mod

log = logging.getLogger("amd-gpu-exporter")

NA = "N/A"


def _num(v) -> Optional[float]:
    if v is None or v == NA or isinstance(v, (list, dict)):
        return None
    try:
        return float(v)
    except (TypeError, ValueError):
        return None


class GpuSample(dict):
    """Flat per-GPU sample: identity keys + metric values (None = unsupported)."""


class AmdSmiBackend:
    """Samples every GPU through the amdsmi module (real library, or a fake in tests)."""

    def __init__(self, amdsmi_module=None):
        if amdsmi_module is None:
            import amdsmi as amdsmi_module  # noqa: N813 - optional dependency
        self.S = amdsmi_module
        self.S.amdsmi_init()
        self.active = True
        self._static: Dict[Any, Dict[str, Any]] = {}

    def close(self) -> None:
        try:
            self.S.amdsmi_shut_down()
        except Exception:  # noqa: BLE001
            pass

    def suspend(self) -> None:
        """Release the amd-smi session (partition change in progress, see pause.py)."""
        if self.active:
            self.close()
            self.active = False
            self._static.clear()      # handles / identities change with the re-enumeration

    def resume(self) -> None:
        if not self.active:
            self.S.amdsmi_init()
            self.active = True

    def _call(self, name: str, *args):
        fn = getattr(self.S, name, None)
        if fn is None:
            return None
        try:
            return fn(*args)
        except Exception as e:  # noqa: BLE001 - per-metric failures are expected (N/A features)
            log.debug("%s failed: %s", name, e)
            return None

    def _identity(self, h) -> Dict[str, Any]:
        key = getattr(h, "value", h) or 0  # real handles are ctypes.c_void_p (unhashable)
        if key in self._static:
            return self._static[key]
        asic = self._call("amdsmi_get_gpu_asic_info", h) or {}
        enum = self._call("amdsmi_get_gpu_enumeration_info", h) or {}
        kfd = self._call("amdsmi_get_gpu_kfd_info", h) or {}
        ident = {
            "pci": self._call("amdsmi_get_gpu_device_bdf", h) or "unknown",
            "uuid": self._call("amdsmi_get_gpu_device_uuid", h) or "",
            "product": asic.get("market_name", "unknown"),
            "gfx": asic.get("target_graphics_version", "unknown"),
            "cu": asic.get("num_compute_units"),
            "render_minor": enum.get("drm_render"),
            "kfd_node": kfd.get("node_id"),
            "partition_id": kfd.get("current_partition_id", 0),
        }
        drv = self._call("amdsmi_get_gpu_driver_info", h) or {}
        ident["driver"] = drv.get("driver_version", "unknown")[:48]
        self._static[key] = ident
        return ident

    def samples(self) -> List[GpuSample]:
        if not self.active:
            raise RuntimeError("amd-smi session released (partition change in progress)")
        out = []
        handles = self._call("amdsmi_get_processor_handles") or []
        for idx, h in enumerate(handles):
            s = GpuSample(index=idx, **self._identity(h))
            m = self._call("amdsmi_get_gpu_metrics_info", h) or {}
            s["gfx_activity"] = _num(m.get("average_gfx_activity"))
            s["umc_activity"] = _num(m.get("average_umc_activity"))
            s["power_w"] = _num(m.get("current_socket_power")) or _num(m.get("average_socket_power"))
            s["temp_hotspot"] = _num(m.get("temperature_hotspot"))
            s["temp_mem"] = _num(m.get("temperature_mem"))
            s["temp_vrsoc"] = _num(m.get("temperature_vrsoc"))
            s["gfxclk_mhz"] = _num(m.get("current_gfxclk"))
            s["uclk_mhz"] = _num(m.get("current_uclk"))
            s["energy_acc"] = _num(m.get("energy_accumulator"))
            s["ppt_residency_acc"] = _num(m.get("ppt_residency_acc"))
            s["pcie_bw_acc"] = _num(m.get("pcie_bandwidth_acc"))
            s["pcie_bw_gbps"] = _num(m.get("pcie_bandwidth_inst"))
            s["pcie_replay_acc"] = _num(m.get("pcie_replay_count_acc"))
            s["pcie_recovery_acc"] = _num(m.get("pcie_l0_to_recov_count_acc"))
            s["pcie_nak_sent_acc"] = _num(m.get("pcie_nak_sent_count_acc"))
            s["pcie_nak_rcvd_acc"] = _num(m.get("pcie_nak_rcvd_count_acc"))
            speed = _num(m.get("pcie_link_speed"))  # 0.1 GT/s units (320 = Gen5 x16's 32 GT/s)
            s["pcie_speed_gts"] = speed / 10.0 if speed is not None else None
            s["pcie_width"] = _num(m.get("pcie_link_width"))
            s["xgmi_speed_gbps"] = _num(m.get("xgmi_link_speed"))
            s["xgmi_width"] = _num(m.get("xgmi_link_width"))
            s["xgmi_read_kb"] = [_num(x) for x in (m.get("xgmi_read_data_acc") or [])]
            s["xgmi_write_kb"] = [_num(x) for x in (m.get("xgmi_write_data_acc") or [])]
            s["xgmi_link_status"] = [_num(x) for x in (m.get("xgmi_link_status") or [])]
            pw = self._call("amdsmi_get_power_info", h) or {}
            limit = _num(pw.get("power_limit"))  # µW
            s["power_limit_w"] = limit / 1e6 if limit is not None else None
            vram = self._call("amdsmi_get_gpu_vram_usage", h) or {}
            if _num(vram.get("vram_total")) is not None:
                s["vram_total_bytes"] = _num(vram["vram_total"]) * 1024 * 1024  # MiB → B
                s["vram_used_bytes"] = (_num(vram.get("vram_used")) or 0) * 1024 * 1024
            ecc = self._call("amdsmi_get_gpu_total_ecc_count", h) or {}
            s["ecc_correctable"] = _num(ecc.get("correctable_count"))
            s["ecc_uncorrectable"] = _num(ecc.get("uncorrectable_count"))
            s["ecc_deferred"] = _num(ecc.get("deferred_count"))
            s["compute_partition"] = self._call("amdsmi_get_gpu_compute_partition", h) or "unknown"
            s["memory_partition"] = self._call("amdsmi_get_gpu_memory_partition", h) or "unknown"
            procs = self._call("amdsmi_get_gpu_process_list", h)
            s["processes"] = float(len(procs)) if isinstance(procs, list) else None
            out.append(s)
        return out


class SysfsBackend:
    """amd-smi-free fallback: DRM sysfs attributes of each GPU's PCI device."""

    def __init__(self, root: str = "/", min_gfx: int = topo_mod.GFX950):
        self.root = root
        self.min_gfx = min_gfx

    def _attr(self, dev: topo_mod.GpuDevice, name: str) -> Optional[str]:
        return topo_mod._drm_attr(self.root, dev.card_minor, dev.render_minor, name)

    def _hwmon(self, dev: topo_mod.GpuDevice, name: str) -> Optional[float]:
        pat = os.path.join(self.root, topo_mod.DRM_CLASS, f"card{dev.card_minor}", "device",
                           "hwmon", "hwmon*", name)
        for p in glob.glob(pat):
            try:
                with open(p) as f:
                    return float(f.read().strip())
            except (OSError, ValueError):
                continue
        return None

    def samples(self) -> List[GpuSample]:
        out = []
        try:
            topo = topo_mod.read_topology(self.root, self.min_gfx)
        except FileNotFoundError:
            return out
        for idx, d in enumerate(g for g in topo.gpus if g.partition_index == 0):
            s = GpuSample(index=idx, pci=d.pci_bdf, uuid=d.uuid, product=d.product, gfx=d.gfx_name,
                          cu=d.cu_count * d.partitions_on_asic, render_minor=d.render_minor,
                          kfd_node=d.node_id, partition_id=0, driver="unknown",
                          compute_partition=d.compute_partition, memory_partition=d.memory_partition)
            s["gfx_activity"] = _num(self._attr(d, "gpu_busy_percent"))
            s["vram_total_bytes"] = _num(self._attr(d, "mem_info_vram_total"))
            s["vram_used_bytes"] = _num(self._attr(d, "mem_info_vram_used"))
            p = self._hwmon(d, "power1_average") or self._hwmon(d, "power1_input")
            s["power_w"] = p / 1e6 if p is not None else None
            t = self._hwmon(d, "temp2_input") or self._hwmon(d, "temp1_input")
            s["temp_hotspot"] = t / 1000.0 if t is not None else None
            out.append(s)
        return out


def read_validations(marker_dir: str) -> Dict[str, Any]:
    out = {}
    for p in sorted(glob.glob(os.path.join(marker_dir, "*.json"))):
        try:
            with open(p) as f:
                out[os.path.basename(p)[:-5]] = json.load(f)
        except (OSError, ValueError):
            continue
    return out


class GpuCollector:
    """prometheus_client collector; ``collect`` samples the backend at scrape time."""

    def __init__(self, backend, node_name: str = "", marker_dir: str = "/run/amd/validations",
                 guard=None):
        self.backend = backend
        self.node = node_name
        self.marker_dir = marker_dir
        self.last_error: Optional[str] = None
        self.scrapes = 0
        self.guard = guard            # pause.PauseGuard("exporter"): partition-change pause
        self.paused = False

    def check_pause(self) -> bool:
        """Release / re-open the backend's GPU session around a partition change; returns paused.
        Called by the exporter's watcher loop (every second) and at every scrape."""
        if self.guard is None:
            return False
        if self.guard.paused():
            if not self.paused:
                getattr(self.backend, "suspend", lambda: None)()
                self.paused = True
            self.guard.ack()
        elif self.paused:
            try:
                getattr(self.backend, "resume", lambda: None)()
                self.paused = False
                self.guard.clear()
            except Exception as e:  # noqa: BLE001 - retried at the next check
                log.warning("cannot re-open the GPU session after the partition change: %s", e)
        return self.paused

    def describe(self):
        return []

    def collect(self) -> Iterable:
        from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily

        self.scrapes += 1
        t0 = time.perf_counter()
        base = ["gpu", "uuid", "pci", "node"]
        paused = self.check_pause()
        if paused:
            # stale on purpose: no GPU handle is open while the partition manager switches modes
            samples, self.last_error = [], "paused: partition change in progress"
        else:
            try:
                samples = self.backend.samples()
                self.last_error = None
            except Exception as e:  # noqa: BLE001 - report through the up metric
                log.warning("sampling failed: %s", e)
                samples, self.last_error = [], str(e)
        up = GaugeMetricFamily("amd_gpu_exporter_up", "1 if the last sample succeeded")
        up.add_metric([], 0.0 if self.last_error else 1.0)
        yield up
        pz = GaugeMetricFamily("amd_gpu_exporter_paused",
                               "1 while GPU sampling is paused for a partition change (metrics stale)")
        pz.add_metric([], 1.0 if paused else 0.0)
        yield pz
        info = GaugeMetricFamily("amd_gpu_info", "static GPU identity (value 1)",
                                 labels=base + ["product", "gfx", "driver", "compute_partition",
                                                "memory_partition", "render_minor"])
        gauges = {
            "gfx_activity": ("amd_gpu_utilization_percent", "GFX engine activity"),
            "umc_activity": ("amd_gpu_memory_activity_percent", "HBM controller activity"),
            "power_w": ("amd_gpu_power_watts", "socket power"),
            "gfxclk_mhz": ("amd_gpu_gfx_clock_mhz", "current GFX clock"),
            "uclk_mhz": ("amd_gpu_memory_clock_mhz", "current memory clock"),
            "vram_total_bytes": ("amd_gpu_vram_total_bytes", "HBM capacity"),
            "vram_used_bytes": ("amd_gpu_vram_used_bytes", "HBM in use"),
            "processes": ("amd_gpu_processes", "processes with the GPU open"),
            "power_limit_w": ("amd_gpu_power_limit_watts", "socket power cap"),
            "pcie_bw_gbps": ("amd_gpu_pcie_bandwidth_gbps", "instantaneous PCIe bandwidth (GB/s)"),
            "pcie_speed_gts": ("amd_gpu_pcie_link_speed_gts", "PCIe link speed (GT/s)"),
            "pcie_width": ("amd_gpu_pcie_link_width", "PCIe link width (lanes)"),
            "xgmi_speed_gbps": ("amd_gpu_xgmi_link_speed_gbps", "xGMI link speed (Gb/s per lane)"),
            "xgmi_width": ("amd_gpu_xgmi_link_width", "xGMI link width (lanes)"),
        }
        fams = {k: GaugeMetricFamily(n, h, labels=base) for k, (n, h) in gauges.items()}
        temp = GaugeMetricFamily("amd_gpu_temperature_celsius", "temperature", labels=base + ["sensor"])
        ecc = CounterMetricFamily("amd_gpu_ecc_errors", "ECC error count", labels=base + ["type"])
        energy = CounterMetricFamily("amd_gpu_energy_accumulator", "firmware energy accumulator (raw)",
                                     labels=base)
        throttle = CounterMetricFamily("amd_gpu_power_throttle_residency", "PPT throttle residency "
                                       "accumulator (raw)", labels=base)
        xgmi = CounterMetricFamily("amd_gpu_xgmi_data_bytes", "xGMI bytes moved per link",
                                   labels=base + ["link", "direction"])
        xlink = GaugeMetricFamily("amd_gpu_xgmi_link_up", "xGMI link status", labels=base + ["link"])
        # PCIe link health (dcgm-exporter's DCGM_FI_DEV_PCIE_REPLAY_COUNTER and friends)
        pcie_ev = CounterMetricFamily("amd_gpu_pcie_events", "PCIe link events (firmware accumulators)",
                                      labels=base + ["event"])
        for s in samples:
            lv = [str(s["index"]), str(s.get("uuid", "")), str(s.get("pci", "")), self.node]
            info.add_metric(lv + [str(s.get("product")), str(s.get("gfx")), str(s.get("driver")),
                                  str(s.get("compute_partition")), str(s.get("memory_partition")),
                                  str(s.get("render_minor"))], 1.0)
            for k, fam in fams.items():
                if s.get(k) is not None:
                    fam.add_metric(lv, float(s[k]))
            for sensor, key in (("hotspot", "temp_hotspot"), ("hbm", "temp_mem"), ("vrsoc", "temp_vrsoc")):
                if s.get(key) is not None:
                    temp.add_metric(lv + [sensor], float(s[key]))
            for typ in ("correctable", "uncorrectable", "deferred"):
                v = s.get(f"ecc_{typ}")
                if v is not None:
                    ecc.add_metric(lv + [typ], float(v))
            if s.get("energy_acc") is not None:
                energy.add_metric(lv, float(s["energy_acc"]))
            if s.get("ppt_residency_acc") is not None:
                throttle.add_metric(lv, float(s["ppt_residency_acc"]))
            for direction, key in (("read", "xgmi_read_kb"), ("write", "xgmi_write_kb")):
                for link, v in enumerate(s.get(key) or []):
                    if v is not None:
                        xgmi.add_metric(lv + [str(link), direction], v * 1024.0)
            for link, v in enumerate(s.get("xgmi_link_status") or []):
                if v is not None:
                    xlink.add_metric(lv + [str(link)], v)
            for event, key in (("replay", "pcie_replay_acc"), ("recovery", "pcie_recovery_acc"),
                               ("nak_sent", "pcie_nak_sent_acc"), ("nak_received", "pcie_nak_rcvd_acc")):
                if s.get(key) is not None:
                    pcie_ev.add_metric(lv + [event], float(s[key]))
        yield info
        yield from fams.values()
        for fam in (temp, ecc, energy, throttle, xgmi, xlink, pcie_ev):
            yield fam
        yield from self._validation_metrics()
        dur = GaugeMetricFamily("amd_gpu_exporter_scrape_seconds", "time to sample all GPUs")
        dur.add_metric([], time.perf_counter() - t0)
        yield dur

    def _validation_metrics(self):
        from prometheus_client.core import GaugeMetricFamily

        vals = read_validations(self.marker_dir)
        passed = GaugeMetricFamily("amd_gpu_validation_passed", "validator step result",
                                   labels=["node", "step"])
        tflops = GaugeMetricFamily("amd_gpu_validator_gemm_tflops",
                                   "bf16 MFMA GEMM TFLOPS measured by the validator", labels=["node", "gpu"])
        tflops8 = GaugeMetricFamily("amd_gpu_validator_gemm_fp8_tflops",
                                    "fp8 (e4m3) MFMA GEMM TFLOPS measured by the validator",
                                    labels=["node", "gpu"])
        busbw = GaugeMetricFamily("amd_gpu_validator_allreduce_busbw_gbps",
                                  "RCCL all-reduce bus bandwidth measured by the validator",
                                  labels=["node", "ngpus"])
        prof = GaugeMetricFamily("amd_gpu_validator_gemm_profile",
                                 "rocprofv3 counters of the validator GEMM (mfma_util_pct, clock_ghz, "
                                 "l2_hit_pct)", labels=["node", "quantity"])
        stress = GaugeMetricFamily("amd_gpu_validator_stress",
                                   "sustained-load stress result per GPU (tflops, tflops_min_window, "
                                   "hotspot_max_c, power_mean_w, gfxclk_mean_mhz)",
                                   labels=["node", "gpu", "quantity"])
        bw = GaugeMetricFamily("amd_gpu_validator_bandwidth_gbps",
                               "HBM / PCIe / xGMI bandwidth measured by the validator (amd-proftester)",
                               labels=["node", "gpu", "test", "peer", "engine"])
        secs = GaugeMetricFamily("amd_gpu_validator_step_seconds",
                                 "wall time of each validator step (report = sum of the required steps)",
                                 labels=["node", "step"])
        for step, v in vals.items():
            if isinstance(v, dict) and "passed" in v:
                passed.add_metric([self.node, step], 1.0 if v["passed"] else 0.0)
            if isinstance(v, dict):
                # an incomplete chain (some required step untimed) is not a time-to-validated
                d = ((v.get("chain_seconds") if v.get("chain_complete", True) else None)
                     if step == "report" else v.get("duration_s"))
                if d is not None:
                    secs.add_metric([self.node, step], float(d))
            if step == "gemm" and isinstance(v, dict):
                for r in v.get("devices", []):
                    if r.get("tflops") is not None:
                        tflops.add_metric([self.node, str(r.get("device"))], float(r["tflops"]))
                for r in (v.get("fp8") or {}).get("devices", []):
                    if r.get("tflops") is not None:
                        tflops8.add_metric([self.node, str(r.get("device"))], float(r["tflops"]))
            if step in ("gemm", "profile") and isinstance(v, dict):
                rc = v.get("rocprof_counters") or {}
                for q in ("mfma_util_pct", "clock_ghz", "l2_hit_pct"):
                    if rc.get(q) is not None:
                        prof.add_metric([self.node, q], float(rc[q]))
            if step == "rccl" and isinstance(v, dict) and v.get("peak_busbw_gbps") is not None:
                busbw.add_metric([self.node, str(v.get("ngpus"))], float(v["peak_busbw_gbps"]))
            if step == "stress" and isinstance(v, dict):
                for gpu, g in (v.get("gpus") or {}).items():
                    for q in ("tflops", "tflops_min_window", "hotspot_max_c", "power_mean_w",
                              "gfxclk_mean_mhz"):
                        if g.get(q) is not None:
                            stress.add_metric([self.node, str(gpu), q], float(g[q]))
            if step == "bandwidth" and isinstance(v, dict):
                for r in v.get("results", []):
                    if r.get("skipped") or r.get("value") is None:
                        continue
                    peer = r.get("peer", -1)
                    bw.add_metric([self.node, str(r.get("device")), str(r.get("test")),
                                   "" if peer is None or peer < 0 else str(peer), str(r.get("engine") or "")],
                                  float(r["value"]))
        yield passed
        yield tflops
        yield tflops8
        yield busbw
        yield prof
        yield stress
        yield bw
        yield secs


def make_registry(collector: GpuCollector):
    from prometheus_client import CollectorRegistry

    reg = CollectorRegistry(auto_describe=False)
    reg.register(collector)
    return reg


class ExporterServer:
    def __init__(self, collector: GpuCollector, port: int = 9400, host: str = "0.0.0.0"):
        from prometheus_client import CONTENT_TYPE_LATEST, generate_latest

        registry = make_registry(collector)
        self.collector = collector
        self.lock = lock = threading.Lock()

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_GET(self):
                if self.path.startswith("/metrics"):
                    with lock:  # amd-smi calls are serialised
                        body = generate_latest(registry)
                    self._ok(body, CONTENT_TYPE_LATEST)
                elif self.path.startswith("/healthz"):
                    self._ok(b"ok\n", "text/plain")
                else:
                    self.send_error(404)

            def _ok(self, body: bytes, ctype: str):
                self.send_response(200)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        self.httpd = ThreadingHTTPServer((host, port), H)

    @property
    def port(self) -> int:
        return self.httpd.server_address[1]

    def serve_background(self) -> threading.Thread:
        t = threading.Thread(target=self.httpd.serve_forever, daemon=True)
        t.start()
        return t

    def shutdown(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()

    def watch_pause(self, interval: float = 1.0, stop_event=None) -> None:
        """Release the GPU session within ``interval`` of a partition pause even without scrapes."""
        stop_event = stop_event or threading.Event()
        while not stop_event.is_set():
            with self.lock:
                self.collector.check_pause()
            stop_event.wait(interval)


def make_backend(root: str = "/"):
    try:
        return AmdSmiBackend()
    except Exception as e:  # noqa: BLE001 - no amd-smi in this image / no device access
        log.warning("amd-smi unavailable (%s); using sysfs fallback", e)
        return SysfsBackend(root)
