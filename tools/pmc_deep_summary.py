"""Summarise tools/pmc_deep.sh output: per kernel (last dispatch), counters summed over dimensions."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
per = defaultdict(lambda: defaultdict(float))
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    rows = list(csv.DictReader(open(f)))
    last = {}
    for r in rows:
        last[r["Kernel_Name"]] = max(last.get(r["Kernel_Name"], 0), int(r["Dispatch_Id"]))
    for r in rows:
        if int(r["Dispatch_Id"]) == last[r["Kernel_Name"]]:
            per[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in per.items():
    name = k.split("(")[0][-60:]
    print("==", name)
    W = c.get("SQ_WAVE_CYCLES", 1)
    for n in sorted(c):
        extra = f"  ({c[n] / W * 100:.1f}% of wave-cycles)" if n.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_BUSY")) and n != "SQ_BUSY_CYCLES" else ""
        print(f"   {n:28s} {c[n]:16.0f}{extra}")
