#!/usr/bin/env python3
"""HBM bytes per scan launch from a rocprofv3 --pmc pass over the L2's
memory-side read requests: 32/64/128-B request counts x their sizes (the
gfx950 FETCH_SIZE tally counts 128-B requests at 64 B, MI355X_MICROARCH.md).
usage: traffic_json.py <pmc dir> <bytes per launch> <workload> > profiles/traffic_<workload>.json"""
import csv
import glob
import json
import sys
from collections import defaultdict

root, nbytes, workload = sys.argv[1], int(sys.argv[2]), sys.argv[3]
acc = defaultdict(list)
name = None
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "scan" not in row["Kernel_Name"]:
            continue
        name = row["Kernel_Name"]
        acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
mean = {k: sum(v) / len(v) for k, v in acc.items()}
hbm = (32 * mean.get("TCC_EA0_RDREQ_32B_sum", 0.0) + 64 * mean.get("TCC_EA0_RDREQ_64B_sum", 0.0)
       + 128 * mean.get("TCC_EA0_RDREQ_128B_sum", 0.0))
json.dump({
    "bytes": nbytes,
    "workload": workload,
    "kernel": name,
    "counters_mean_per_launch": mean,
    "hbm_bytes_per_launch": hbm,
    "ratio_to_input": hbm / nbytes,
    "note": "rocprofv3 --pmc TCC_EA0_RDREQ{,_32B,_64B,_128B}_sum, mean per scan launch of "
            "bench.py; bytes = 32*n32 + 64*n64 + 128*n128 (L2 -> fabric read requests)",
}, sys.stdout, indent=1)
print()
