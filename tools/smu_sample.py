#!/usr/bin/env python3
"""SMU sampler: this job's GPU's power, clocks, energy accumulator and
throttle / violation residency while a command runs.

    python3 tools/smu_sample.py OUT.jsonl [--period-ms 2] -- python bench.py ... --marks M.json

Reads the driver's gpu_metrics table and violation status through the amdsmi
Python bindings (sysfs / ioctl, no root, no HIP in this process).  The
command runs as a child process (never exec'd).  Every sample is one JSON
line; the first line is the device's static record (BDF, power cap).
tools/smu_summary.py turns the samples (and the bench's --marks window) into
J/GiB, mean power, clock and throttle residency.
"""
import json
import os
import subprocess
import sys
import threading
import time

KEYS = ("average_socket_power", "current_socket_power", "energy_accumulator",
        "average_gfxclk_frequency", "current_gfxclk", "current_gfxclks", "current_uclk",
        "throttle_status", "indep_throttle_status", "temperature_hotspot", "temperature_mem",
        "temperature_vrgfx", "temperature_vrsoc", "temperature_vrmem", "average_gfx_activity",
        "average_umc_activity", "accumulation_counter", "prochot_residency_acc",
        "ppt_residency_acc", "socket_thm_residency_acc", "vr_thm_residency_acc",
        "hbm_thm_residency_acc", "firmware_timestamp", "system_clock_counter",
        "voltage_gfx", "voltage_soc", "voltage_mem", "gfxclk_lock_status")
VKEYS = ("acc_counter", "acc_prochot_thrm", "acc_ppt_pwr", "acc_socket_thrm", "acc_vr_thrm",
         "acc_hbm_thrm", "acc_gfx_clk_below_host_limit", "acc_gfx_clk_below_host_limit_pwr",
         "acc_gfx_clk_below_host_limit_thm", "acc_gfx_clk_below_host_limit_total",
         "acc_low_utilization", "per_ppt_pwr", "per_socket_thrm", "per_vr_thrm", "per_hbm_thrm",
         "per_gfx_clk_below_host_limit", "per_gfx_clk_below_host_limit_pwr",
         "per_gfx_clk_below_host_limit_thm", "per_gfx_clk_below_host_limit_total",
         "active_ppt_pwr", "active_socket_thrm", "active_vr_thrm", "active_hbm_thrm",
         "active_gfx_clk_below_host_limit")


def jsonable(v):
    if isinstance(v, (list, tuple)):
        return [jsonable(x) for x in v]
    if isinstance(v, (int, float, str, bool)) or v is None:
        return v
    return str(v)


def my_bdf():
    """PCI bus id of HIP device 0 (tools/gpu_hwmon.py in a child process)."""
    here = os.path.dirname(os.path.abspath(__file__))
    try:
        hw = subprocess.run([sys.executable, os.path.join(here, "gpu_hwmon.py")],
                            capture_output=True, text=True, timeout=120).stdout.strip()
        # /sys/bus/pci/devices/0000:xx:yy.z/hwmon/hwmonN
        return hw.split("/")[5].lower() if hw else None
    except Exception:
        return None


def main():
    argv = sys.argv[1:]
    cut = argv.index("--")
    opts, cmd = argv[:cut], argv[cut + 1:]
    out = opts[0]
    period = float(opts[opts.index("--period-ms") + 1]) / 1e3 if "--period-ms" in opts else 0.002
    static, h = {}, None
    try:
        import amdsmi as A
        A.amdsmi_init(A.AmdSmiInitFlags.INIT_AMD_GPUS)
        bdf = my_bdf()
        handles = A.amdsmi_get_processor_handles()
        for x in handles:
            if bdf and A.amdsmi_get_gpu_device_bdf(x).lower() == bdf:
                h = x
        if h is None:
            h = handles[0]
        static = {"bdf": A.amdsmi_get_gpu_device_bdf(h), "wanted_bdf": bdf,
                  "n_handles": len(handles)}
        for name, fn in (("power_cap", A.amdsmi_get_power_cap_info),
                         ("energy", A.amdsmi_get_energy_count)):
            try:
                static[name] = jsonable(fn(h))
            except Exception as e:  # report, keep sampling what is readable
                static[name] = f"error: {e}"
    except Exception as e:  # no amdsmi access: run the command unsampled
        static = {"error": f"amdsmi: {e!r}"}
    f = open(out, "w")
    f.write(json.dumps({"static": static}) + "\n")
    stop = threading.Event()
    errs = {}

    def sample():
        n = 0
        while not stop.is_set():
            rec = {"t": time.time()}
            try:
                m = A.amdsmi_get_gpu_metrics_info(h)
                rec.update({k: jsonable(m.get(k)) for k in KEYS})
            except Exception as e:
                errs["metrics"] = str(e)
            if n % 10 == 0:  # violation status: slower-moving accumulators
                try:
                    v = A.amdsmi_get_violation_status(h)
                    rec["viol"] = {k: jsonable(v.get(k)) for k in VKEYS}
                except Exception as e:
                    errs["violation"] = str(e)
            rec["t1"] = time.time()
            f.write(json.dumps(rec) + "\n")
            n += 1
            time.sleep(period)

    th = threading.Thread(target=sample, daemon=True)
    if h is not None:
        th.start()
    time.sleep(0.3)  # idle samples before the command
    rc = subprocess.call(cmd)
    time.sleep(0.3)
    stop.set()
    if h is not None:
        th.join()
    f.write(json.dumps({"errors": errs, "rc": rc}) + "\n")
    f.close()
    if h is not None:
        A.amdsmi_shut_down()
    sys.exit(rc)


if __name__ == "__main__":
    main()
