#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc/p*/pmc_counter_collection.csv):
per kernel, average per dispatch of every counter, plus derived HBM bytes
(FETCH_SIZE is in KB and reads 1/2 of wide streaming loads on gfx950 —
MI355X_MICROARCH.md §HBM — so it is doubled; WRITE_SIZE in KB is exact)."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    per_dispatch = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for row in csv.DictReader(open(f)):
        kn = row.get("Kernel_Name") or row.get("Kernel-Name")
        did = row.get("Dispatch_Id") or row.get("Correlation_Id")
        cn = row.get("Counter_Name")
        per_dispatch[did][cn] += float(row.get("Counter_Value", 0))
        names[did] = kn
    for did, cs in per_dispatch.items():
        k = names[did].split("(")[0]
        for cn, v in cs.items():
            acc[k][cn].append(v)
out = {}
for k, cs in acc.items():
    d = {cn: sum(v) / len(v) for cn, v in cs.items()}
    d["dispatches"] = max(len(v) for v in cs.values())
    if "FETCH_SIZE" in d:
        d["hbm_read_bytes_corrected"] = d["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in d:
        d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
    out[k] = d
print(json.dumps(out, indent=1))
