#!/usr/bin/env python3
"""Dump what the amdsmi Python API returns on this node (read-only) as one JSON document.

Used once per hardware generation to record the shapes the exporter / labeller / partition
manager consume, so their fakes (tests/fixtures) match real MI355X answers.
"""
import json
import sys


def _try(fn, *a):
    try:
        v = fn(*a)
        json.dumps(v, default=str)
        return v
    except Exception as e:  # noqa: BLE001 - we record every failure mode
        return {"error": f"{type(e).__name__}: {e}"}


def main() -> int:
    import amdsmi as S

    S.amdsmi_init()
    out = {"handles": []}
    try:
        handles = S.amdsmi_get_processor_handles()
        for h in handles:
            d = {}
            for name in [
                "amdsmi_get_gpu_asic_info", "amdsmi_get_gpu_board_info", "amdsmi_get_gpu_bdf_id",
                "amdsmi_get_gpu_device_bdf", "amdsmi_get_gpu_device_uuid", "amdsmi_get_gpu_kfd_info",
                "amdsmi_get_gpu_driver_info", "amdsmi_get_gpu_vram_info", "amdsmi_get_gpu_vram_usage",
                "amdsmi_get_gpu_activity", "amdsmi_get_power_info", "amdsmi_get_clock_info",
                "amdsmi_get_gpu_metrics_info", "amdsmi_get_gpu_compute_partition",
                "amdsmi_get_gpu_memory_partition", "amdsmi_get_gpu_ras_feature_info",
                "amdsmi_get_gpu_total_ecc_count", "amdsmi_get_gpu_process_list",
                "amdsmi_get_gpu_xgmi_info", "amdsmi_get_fw_info", "amdsmi_get_gpu_vbios_info",
                "amdsmi_get_gpu_enumeration_info", "amdsmi_get_gpu_accelerator_partition_profile",
                "amdsmi_get_gpu_memory_partition_config",
            ]:
                fn = getattr(S, name, None)
                if fn is not None:
                    d[name] = _try(fn, h)
            temp = {}
            for label in ("EDGE", "HOTSPOT", "VRAM"):
                try:
                    temp[label] = S.amdsmi_get_temp_metric(
                        h, getattr(S.AmdSmiTemperatureType, label),
                        S.AmdSmiTemperatureMetric.CURRENT)
                except Exception as e:  # noqa: BLE001
                    temp[label] = {"error": str(e)}
            d["temperature"] = temp
            out["handles"].append(d)
            if len(out["handles"]) >= 2:
                break
        out["version"] = _try(S.amdsmi_get_lib_version)
    finally:
        S.amdsmi_shut_down()
    json.dump(out, sys.stdout, indent=1, default=str)
    return 0


if __name__ == "__main__":
    sys.exit(main())
