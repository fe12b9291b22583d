"""Print per-kernel average durations of gpurun_out/pb_<variant> rocprofv3 summaries (dev tool)."""
import csv
import glob
import sys

for v in sys.argv[1:]:
    f = glob.glob(f"gpurun_out/pb_{v}/**/*kernel_stats.csv", recursive=True)
    if not f:
        print(v, "missing")
        continue
    print("==", v)
    for r in csv.DictReader(open(f[0])):
        if "at::" in r["Name"]:
            continue
        print(f"   {r['Name'][:80]:80s} calls {r['Calls']:>4s} avg {float(r['AverageNs']) / 1e3:9.1f} us")
