"""Turn a tools/profile_round.sh output directory into the committed profile artefacts.

    python tools/profile_summary.py gpurun_out/prof_<tag> <tag> [out dir, default profiles/]

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats of the bench command (verbatim)
  profiles/<tag>_bench.json         the bench JSON line printed under the profiler
  profiles/<tag>_pmc.json           per kernel: FETCH_SIZE (raw and x2-corrected), WRITE_SIZE, MFMA busy,
                                    the effective clock of the profiled dispatch (clock_GHz)
  profiles/traffic_latest.json      bench kernel key -> HBM bytes per launch (FETCH x2 + WRITE), which
                                    bench.py reports as roofline.traffic
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")

# bench.py kernel keys -> (normalised rocprof kernel-name pattern, workgroups per launch or None) of
# the D = 128 instantiations at config 3 (4,32,4096,128).  The record backward runs in chunks of
# CHUNK heads (attention_int8._ws_chunk: 32 at config 3), so its kernels appear with two grids: the
# chunk launch the step runs, and the one-pass launch over all 128 heads.
BH, S = 4 * 32, 4096
CHUNK = 32
KEYS = {
    # the q-fused forward with the inline fixup <D, CAUSAL, SPLIT, QF, FIX, INL> (the drop-ins' kernel)
    "int8_attn_fwd_kernel": (r"int8_attn_fwd_kernel(<128,false,false,true,false,true>|"
                             r"ILi128ELb0ELb0ELb1ELb0ELb1E)", None),
    "int8_attn_fwd_kernel<q_i8 in>": (r"int8_attn_fwd_kernel(<128,false,false,false,false,false>|"
                                      r"ILi128ELb0ELb0ELb0ELb0ELb0E)", None),
    "int8_bwd_dkdv_kernel<dK+dV>": (r"int8_bwd_kernel(<128, ?3, ?false, ?false>|ILi128ELi3ELb0ELb0E)", None),
    "int8_bwd_dq_kernel": (r"int8_bwd_kernel(<128, ?2|ILi128ELi2E)", None),
    "int8_bwd_dkdv_kernel<dK+dV, dS out>": (r"int8_bwd_kernel(<128, ?3, ?false, ?true>|ILi128ELi3ELb0ELb1E)",
                                            CHUNK * S // 256),
    "int8_bwd_dkdv_kernel<dK+dV, dS out, one pass>": (
        r"int8_bwd_kernel(<128, ?3, ?false, ?true>|ILi128ELi3ELb0ELb1E)", BH * S // 256),
    "int8_bwd_dqw_kernel": (r"int8_bwd_dqw_kernel(<128|ILi128E)", CHUNK * S // 256),
    "int8_bwd_dqw_kernel<one pass>": (r"int8_bwd_dqw_kernel(<128|ILi128E)", BH * S // 256),
}
SIMDS_PER_XCD = 32 * 4
# credited MFMA work per launch (bench.py per_call) and the dense peaks (2.4 GHz spec)
CREDIT = {"int8_attn_fwd_kernel": 4.0 * BH * S * S * 128, "int8_attn_fwd_kernel<q_i8 in>": 4.0 * BH * S * S * 128,
          "int8_bwd_dkdv_kernel<dK+dV, dS out>": 8.0 * CHUNK * S * S * 128,
          "int8_bwd_dqw_kernel": 2.0 * CHUNK * S * S * 128}
PEAK_I8, PEAK_BF16 = 256 * 8192 * 2.4e9, 256 * 4096 * 2.4e9
# GRBM_GUI_ACTIVE is summed over the 8 XCDs; SQ_VALU_MFMA_BUSY_CYCLES counts 32 busy SIMD-cycles per
# 32x32 MFMA (i8 32x32x32 and f16/bf16 32x32x16 alike: 65536 / 32768 ops at 2048 / 1024 ops/clk/SIMD)
XCDS = 8


def norm(name):
    return re.sub(r"\s+", "", name)


def workgroups(row):
    """Workgroups of a dispatch from a rocprofv3 CSV row (Grid_Size / Workgroup_Size, in work-items)."""
    try:
        g = int(float(row.get("Grid_Size") or row.get("Grid_Size_X") or 0))
        w = int(float(row.get("Workgroup_Size") or row.get("Workgroup_Size_X") or 0))
        return g // w if w else None
    except ValueError:
        return None


def key_of(name, wgs=None):
    n = norm(name)
    for k, (pat, want) in KEYS.items():
        if re.search(pat, n) and (want is None or wgs is None or want == wgs):
            return k
    return None


def counters(d):
    """{bench key: {counter: mean per dispatch}} from one --pmc pass directory."""
    per = defaultdict(float)
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = key_of(row["Kernel_Name"], workgroups(row))
            if k is None:
                continue
            per[(k, row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
            if row.get("Start_Timestamp") and row.get("End_Timestamp"):
                dur[(k, row["Dispatch_Id"])] = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
    acc = defaultdict(lambda: defaultdict(list))
    for (k, _, c), v in per.items():
        acc[k][c].append(v)
    for (k, _), v in dur.items():   # the profiled dispatch's duration (ns)
        acc[k]["dispatch_ns"].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    out_dir = sys.argv[3] if len(sys.argv) > 3 else PROF
    os.makedirs(out_dir, exist_ok=True)
    fetch = counters(os.path.join(src, "fetch"))
    write = counters(os.path.join(src, "write"))
    mfma = counters(os.path.join(src, "mfma"))
    mops = counters(os.path.join(src, "mops")) if os.path.isdir(os.path.join(src, "mops")) else {}
    valu = counters(os.path.join(src, "valu")) if os.path.isdir(os.path.join(src, "valu")) else {}
    out, traffic = {}, {}
    for k in KEYS:
        e = {}
        if k in fetch:
            e["FETCH_SIZE_raw_bytes"] = fetch[k]["FETCH_SIZE"] * 1024
            e["FETCH_bytes_x2"] = 2 * e["FETCH_SIZE_raw_bytes"]
        if k in write:
            e["WRITE_bytes"] = write[k]["WRITE_SIZE"] * 1024
        if k in mfma and mfma[k].get("GRBM_GUI_ACTIVE"):
            m = mfma[k]
            e.update(m)
            cyc = m["GRBM_GUI_ACTIVE"] / XCDS
            e["mfma_util"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * SIMDS_PER_XCD * XCDS)
            e["gpu_cycles"] = cyc
            if m.get("dispatch_ns"):
                # effective shader clock of the profiled dispatch (MI355X_MICROARCH "DVFS give-back":
                # GRBM_GUI_ACTIVE / 8 / wall time; profiled passes run a few % below un-profiled ones)
                e["clock_GHz"] = cyc / m["dispatch_ns"]
        if k in mops:
            # MFMA work the kernel executed (512 ops per MOPS unit), against what bench credits it
            m = mops[k]
            e.update(m)
            e["mfma_ops_executed"] = 512 * sum(m.get(c, 0.0) for c in (
                "SQ_INSTS_VALU_MFMA_MOPS_I8", "SQ_INSTS_VALU_MFMA_MOPS_F16", "SQ_INSTS_VALU_MFMA_MOPS_BF16"))
            if k in CREDIT and e["mfma_ops_executed"] > 0:
                # the MFMA ceiling of the kernel's own mix: its executed i8 and f16/bf16 work at the
                # dense peaks, against the work it is credited with (bf16 runs at half the i8 rate)
                t_peak = (512 * m.get("SQ_INSTS_VALU_MFMA_MOPS_I8", 0.0) / PEAK_I8 + 512 * (
                    m.get("SQ_INSTS_VALU_MFMA_MOPS_F16", 0.0) + m.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0))
                    / PEAK_BF16)
                e["mfma_ceiling_frac"] = CREDIT[k] / t_peak / PEAK_I8
        if k in valu and valu[k].get("GRBM_GUI_ACTIVE"):
            m = valu[k]
            cyc = m["GRBM_GUI_ACTIVE"] / XCDS
            e["valu_pass"] = {c: v for c, v in m.items()}
            # SQ_ACTIVE_INST_VALU: quad-cycles in which a wave issues VALU work (MFMAs included),
            # summed over waves: per SIMD, the share of cycles its vector issue is taken
            e["valu_busy"] = 4 * m.get("SQ_ACTIVE_INST_VALU", 0.0) / (cyc * SIMDS_PER_XCD * XCDS)
            e["vector_insts_per_mfma"] = (m.get("SQ_INSTS_VALU", 0.0) - m.get("SQ_INSTS_MFMA", 0.0)) / max(
                1.0, m.get("SQ_INSTS_MFMA", 0.0))
        if "FETCH_bytes_x2" in e and "WRITE_bytes" in e:
            traffic[k] = e["FETCH_bytes_x2"] + e["WRITE_bytes"]
            e["hbm_bytes_per_launch"] = traffic[k]
        out[k] = e
    with open(os.path.join(out_dir, f"{tag}_pmc.json"), "w") as f:
        json.dump({"note": "FETCH_SIZE/WRITE_SIZE are KB per dispatch from rocprofv3; FETCH doubled "
                           "per MI355X_MICROARCH.md (gfx950 reports half of wide streaming reads)",
                   "kernels": out}, f, indent=1)
    sys.path.insert(0, ROOT)
    from bench import source_hash
    with open(os.path.join(out_dir, "traffic_latest.json"), "w") as f:
        # bench.py reports these only while the kernel sources hash to source_sha256
        json.dump({"tag": tag, "source_sha256": source_hash(), "shape": [4, 32, 4096, 128],
                   "traffic": traffic,
                   "clock_GHz": {k: e["clock_GHz"] for k, e in out.items() if "clock_GHz" in e},
                   "counters": {k: {f: e[f] for f in ("mfma_util", "valu_busy", "mfma_ceiling_frac",
                                                       "vector_insts_per_mfma", "clock_GHz") if f in e}
                                for k, e in out.items()}},
                  f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
