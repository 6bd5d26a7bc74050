#!/usr/bin/env python3
"""Prints the hwmon directory of HIP device 0 (the GPU this job sees) from its
PCI bus id, so power sampling reads this GPU and not another job's on a
shared node.  Uses the HIP runtime through ctypes (no torch)."""
import ctypes
import glob
import sys

hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
buf = ctypes.create_string_buffer(64)
if hip.hipDeviceGetPCIBusId(buf, 64, 0) != 0:
    sys.exit("hipDeviceGetPCIBusId failed")
bus = buf.value.decode().lower()
dirs = glob.glob(f"/sys/bus/pci/devices/{bus}/hwmon/hwmon*")
if not dirs:
    sys.exit(f"no hwmon for {bus}")
print(dirs[0])
