"""Summarise a rocprofv3 kernel trace (rocpd SQLite .db or kernel_trace.csv) into a per-kernel
stats CSV under profiles/ (calls, total/avg/min/max ns, % of GPU time, VGPR/SGPR/LDS/scratch).

  python scripts/prof_summary.py gpurun_out/prof_r01 profiles/r01_kernel_stats.csv
"""
import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def rows_from_db(path):
    c = sqlite3.connect(path)
    q = ("select name, duration, grid_x, workgroup_x, lds_size, scratch_size, vgpr_count, sgpr_count "
         "from kernels")
    for r in c.execute(q):
        yield {"name": r[0], "ns": int(r[1]), "grid": r[2], "wg": r[3], "lds": r[4], "scratch": r[5],
               "vgpr": r[6], "sgpr": r[7]}


def rows_from_csv(path):
    for r in csv.DictReader(open(path)):
        yield {"name": r["Kernel_Name"], "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
               "grid": r.get("Grid_Size_X") or r.get("Grid_Size"), "wg": r.get("Workgroup_Size_X") or r.get("Workgroup_Size"),
               "lds": r.get("LDS_Block_Size") or r.get("Lds_Size"), "scratch": r.get("Scratch_Size"),
               "vgpr": r.get("VGPR_Count") or r.get("Arch_VGPR_Count"), "sgpr": r.get("SGPR_Count")}


def main(src, dst):
    files = glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
    rows = []
    for f in files:
        rows += list(rows_from_db(f))
    if not rows:
        for f in glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True):
            rows += list(rows_from_csv(f))
    agg = defaultdict(list)
    meta = {}
    for r in rows:
        agg[r["name"]].append(r["ns"])
        meta[r["name"]] = r
    total = sum(sum(v) for v in agg.values()) or 1
    out = []
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        m = meta[name]
        out.append([name, len(v), sum(v), sum(v) / len(v), min(v), max(v), 100.0 * sum(v) / total,
                    m["grid"], m["wg"], m["lds"], m["scratch"], m["vgpr"], m["sgpr"]])
    with open(dst, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage",
                    "GridX", "WorkgroupX", "LDS", "ScratchPerLane", "VGPR", "SGPR"])
        w.writerows(out)
    for r in out[:6]:
        print(f"{r[0][:70]:70s} calls={r[1]:3d} avg={r[3] / 1e6:10.3f} ms  {r[6]:5.1f}%  scratch={r[10]} vgpr={r[11]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
