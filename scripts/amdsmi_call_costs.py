#!/usr/bin/env python3
"""Per-call cost of the amdsmi queries the agent's health poll and full sample make, on the real
MI355X (median of N calls, microseconds), plus libmi355x_dev's health_snapshot / snapshot walls.
Decides which fields the 10 Hz health poll can afford."""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def med_us(fn, n=50):
    xs = []
    for _ in range(n):
        t0 = time.perf_counter()
        try:
            fn()
        except Exception as e:  # report unsupported calls instead of failing the run
            return f"error: {e}"
        xs.append((time.perf_counter() - t0) * 1e6)
    return round(statistics.median(xs), 1)


def main() -> None:
    import amdsmi as a
    a.amdsmi_init(a.AmdSmiInitFlags.INIT_AMD_GPUS)
    h = a.amdsmi_get_processor_handles()[0]
    T = a.AmdSmiTemperatureType
    M = a.AmdSmiTemperatureMetric
    out = {
        "total_ecc_count": med_us(lambda: a.amdsmi_get_gpu_total_ecc_count(h)),
        "xgmi_link_status": med_us(lambda: a.amdsmi_get_gpu_xgmi_link_status(h)),
        "temp_hotspot_current": med_us(lambda: a.amdsmi_get_temp_metric(h, T.HOTSPOT, M.CURRENT)),
        "temp_vram_current": med_us(lambda: a.amdsmi_get_temp_metric(h, T.VRAM, M.CURRENT)),
        "temp_edge_current": med_us(lambda: a.amdsmi_get_temp_metric(h, T.EDGE, M.CURRENT)),
        "gpu_activity": med_us(lambda: a.amdsmi_get_gpu_activity(h)),
        "power_info": med_us(lambda: a.amdsmi_get_power_info(h)),
        "memory_usage_vram": med_us(lambda: a.amdsmi_get_gpu_memory_usage(h, a.AmdSmiMemoryType.VRAM)),
        "bad_page_info": med_us(lambda: a.amdsmi_get_gpu_bad_page_info(h)),
        "compute_partition": med_us(lambda: a.amdsmi_get_gpu_compute_partition(h)),
        "memory_partition": med_us(lambda: a.amdsmi_get_gpu_memory_partition(h)),
        "gpu_metrics_info": med_us(lambda: a.amdsmi_get_gpu_metrics_info(h)),
        "ecc_count_umc": med_us(lambda: a.amdsmi_get_gpu_ecc_count(h, a.AmdSmiGpuBlock.UMC)),
        "ecc_count_gfx": med_us(lambda: a.amdsmi_get_gpu_ecc_count(h, a.AmdSmiGpuBlock.GFX)),
        "ecc_enabled": med_us(lambda: a.amdsmi_get_gpu_ecc_enabled(h)),
    }
    try:
        out["ecc_count_umc_value"] = a.amdsmi_get_gpu_ecc_count(h, a.AmdSmiGpuBlock.UMC)
        out["ecc_enabled_value"] = a.amdsmi_get_gpu_ecc_enabled(h)
    except Exception as e:
        out["ecc_values_error"] = str(e)
    a.amdsmi_shut_down()
    from gpupool.ops import devlib
    d = devlib.DeviceLib("amdsmi", node="t", events=False)
    out["devlib_health_snapshot"] = med_us(d.health_snapshot, 30)
    out["devlib_snapshot"] = med_us(d.snapshot, 30)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
