#!/usr/bin/env python3
"""Mean Msamples/s per (variant, mode) of a tools/ab.sh log.   python tools/ab_summary.py LOG..."""
import collections
import json
import re
import sys

for f in sys.argv[1:]:
    d = collections.defaultdict(list)
    v = None
    for line in open(f):
        m = re.match(r"== (\S+) round", line)
        if m:
            v = m.group(1)
        elif line.startswith("{") and "msamples_s" in line:
            j = json.loads(line)
            vv = v + (f"/s{j['streams']}" if j.get("streams") else "")
            d[(j.get("scene", ""), j["mode"], vv)].append(j["msamples_s"])
    print(f)
    for k in sorted(d, key=lambda k: (k[1], k[2])):
        print(f"  mode {k[1]} {k[2]:10s} {sum(d[k]) / len(d[k]):9.1f}   {[round(x, 1) for x in d[k]]}")
