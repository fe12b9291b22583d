"""Per-shape kernel summary of a rocprofv3 --kernel-trace run (dev tool, tools/profile_round.sh).

    python tools/trace_summary.py <trace dir> <out.csv>

rocprofv3's --stats table averages every dispatch of a kernel name together; the step runs some
kernels at two grids (the chunked record backward: chunk-sized launches; the per-kernel timings of
bench.py: one-pass launches), so that average has no per-launch work figure.  This groups the
dispatches of the *_kernel_trace.csv by (kernel name, workgroups, workgroup size) and adds the
bench.py key of each group (tools/profile_summary.KEYS), so a row's average duration and its
credited work per launch give the roofline fraction directly."""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from profile_summary import key_of, workgroups  # noqa: E402


def main():
    src, dst = sys.argv[1], sys.argv[2]
    groups = defaultdict(list)
    for f in glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            wg = workgroups(row)
            wsz = row.get("Workgroup_Size") or row.get("Workgroup_Size_X")
            lds = row.get("LDS_Block_Size")   # (tells shapes with equal grids apart: per-tile scales)
            dur = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
            groups[(row["Kernel_Name"], wg, wsz, lds)].append(dur)
    rows = []
    for (name, wg, wsz, lds), d in groups.items():
        rows.append({"bench_key": key_of(name, wg) or "", "Kernel_Name": name, "Workgroups": wg,
                     "Workgroup_Size": wsz, "LDS_Block_Size": lds, "Calls": len(d), "TotalDurationNs": sum(d),
                     "AverageNs": round(sum(d) / len(d)), "MedianNs": round(statistics.median(d)),
                     "MinNs": min(d), "MaxNs": max(d)})
    rows.sort(key=lambda r: -r["TotalDurationNs"])
    with open(dst, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]) if rows else ["Kernel_Name"])
        w.writeheader()
        w.writerows(rows)
    for r in rows[:12]:
        print(f"{r['AverageNs'] / 1e3:9.1f} us x{r['Calls']:4d}  wg={r['Workgroups']}  {r['bench_key'] or r['Kernel_Name'][:70]}")


if __name__ == "__main__":
    main()
