"""Summarise rocprofv3 --pmc CSV passes for one kernel (substring match) -> per-dispatch averages."""
import csv
import glob
import json
import sys
from collections import defaultdict

root, pat = sys.argv[1], sys.argv[2]
vals = defaultdict(list)
for f in glob.glob(f"{root}/p*/run_counter_collection.csv"):
    per = defaultdict(float)
    for row in csv.DictReader(open(f)):
        if pat not in row["Kernel_Name"]:
            continue
        per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (d, c), v in per.items():
        vals[c].append(v)
avg = {c: sum(v) / len(v) for c, v in vals.items()}
dur = []
for row in csv.DictReader(open(glob.glob(f"{root}/trace/**/*kernel_trace.csv", recursive=True)[0])):
    if pat in row["Kernel_Name"]:
        dur.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
avg["duration_ns"] = sum(dur) / len(dur) if dur else None
print(json.dumps(avg, indent=1))
