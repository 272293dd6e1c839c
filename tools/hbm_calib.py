#!/usr/bin/env python3
"""Summarise tools/hbm_calib.sh: per access pattern, the counted FETCH_SIZE / WRITE_SIZE bytes
over the bytes the kernel moves by construction (tools/hbm_calib.hip)."""
import csv
import glob
import json
import sys

out = sys.argv[1]
known = {}
for line in open(out + "/bytes.jsonl"):
    r = json.loads(line)
    known[r["kernel"]] = r


def counters(sub, name):
    f = glob.glob(f"{out}/{sub}/**/*counter_collection.csv", recursive=True)[0]
    vals = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if k in known and r["Counter_Name"] == name:
            vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"]) * 1024.0  # KiB -> bytes
    return vals


fetch, write = counters("fetch", "FETCH_SIZE"), counters("write", "WRITE_SIZE")
rows = []
for k, r in known.items():
    row = {"kernel": k, "read_bytes": r["read_bytes"], "write_bytes": r["write_bytes"],
           "fetch_size_bytes": fetch.get(k), "write_size_bytes": write.get(k), "ms": r["ms"]}
    if r["read_bytes"] > 0 and fetch.get(k) is not None:
        row["fetch_over_read"] = round(fetch[k] / r["read_bytes"], 4)
    if r["write_bytes"] > 0 and write.get(k) is not None:
        row["write_over_written"] = round(write[k] / r["write_bytes"], 4)
    rows.append(row)
print(json.dumps(rows, indent=1))
