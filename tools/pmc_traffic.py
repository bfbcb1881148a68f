"""HBM traffic per launch of one kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

usage: python tools/pmc_traffic.py <pmc dir> <kernel substring> <out.json> [note]

Counters as MI355X_MICROARCH.md §HBM prescribes: collected in their own passes
(tools/traffic.sh; never combined with trace domains), reported by rocprofv3 in
KiB; on gfx950 FETCH_SIZE tallies 128-B streaming requests at 64 B, so it is
doubled; WRITE_SIZE is taken as is.  bench.py reads the resulting JSON as the
`traffic` of its roofline object.
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import roof_src_hash  # noqa: E402

d, sub, out = sys.argv[1], sys.argv[2], sys.argv[3]
note = sys.argv[4] if len(sys.argv) > 4 else ""
vals = {"FETCH_SIZE": [], "WRITE_SIZE": []}
name = None
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"] and r["Counter_Name"] in vals:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
if not vals["FETCH_SIZE"] or not vals["WRITE_SIZE"]:
    sys.exit(f"no FETCH_SIZE/WRITE_SIZE rows for kernel matching {sub!r} under {d}")
fetch = 2 * 1024 * sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
write = 1024 * sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
res = {"kernel": name, "match": sub, "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
       "traffic_bytes_per_launch": fetch + write, "launches": len(vals["FETCH_SIZE"]),
       "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count), WRITE_SIZE KiB x1024", "note": note,
       "kernel_src_hash": roof_src_hash()}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
