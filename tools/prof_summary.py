"""Summarise rocprofv3 CSV output into profiles/<tag>_summary.{json,md}.

Usage: python tools/prof_summary.py <tag> <stats_dir> [<pmc_dir> ...]

* kernel stats: <stats_dir>/*_kernel_stats.csv (rocprofv3 --kernel-trace --stats -f csv)
* PMC passes:   <pmc_dir>/*_counter_collection.csv (rocprofv3 --kernel-trace --pmc X -f csv),
  one counter per pass.  gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE is in
  KiB and reads 1/2 of the bytes of a wide coalesced stream -> bytes = 2 * 1024 * FETCH_SIZE;
  WRITE_SIZE is in KiB and exact for 16-B/lane stores -> bytes = 1024 * WRITE_SIZE.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.split("(")[0]
    return n.replace("dsr::", "")


def main():
    tag, stats_dir, pmc_dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    out = {"tag": tag, "kernels": {}}
    for f in glob.glob(os.path.join(stats_dir, "*_kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Name"])
            out["kernels"][k] = {"calls": int(r["Calls"]), "total_ms": float(r["TotalDurationNs"]) / 1e6,
                                 "avg_ms": float(r["AverageNs"]) / 1e6, "pct": float(r["Percentage"])}
    counters = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for d in pmc_dirs:
        for f in glob.glob(os.path.join(d, "*_counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                counters[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    pmc = {}
    for k, cs in counters.items():
        e = {name: sum(v) / len(v) for name, v in cs.items()}
        if "FETCH_SIZE" in e:
            e["fetch_bytes_per_launch_corrected"] = 2 * 1024 * e["FETCH_SIZE"]
        if "WRITE_SIZE" in e:
            e["write_bytes_per_launch"] = 1024 * e["WRITE_SIZE"]
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["hbm_bytes_per_launch"] = e["fetch_bytes_per_launch_corrected"] + e["write_bytes_per_launch"]
        e["launches_profiled"] = max(len(v) for v in cs.values())
        e["avg_ms_under_pmc"] = sum(durs[k]) / len(durs[k])
        pmc[k] = e
    out["pmc"] = pmc
    os.makedirs("profiles", exist_ok=True)
    json.dump(out, open(f"profiles/{tag}_summary.json", "w"), indent=1, sort_keys=True)
    lines = [f"# rocprofv3 summary `{tag}`", "", "| kernel | calls | avg ms | total ms | % |", "|---|---|---|---|---|"]
    for k, v in sorted(out["kernels"].items(), key=lambda x: -x[1]["total_ms"]):
        lines.append(f"| {k} | {v['calls']} | {v['avg_ms']:.3f} | {v['total_ms']:.1f} | {v['pct']:.2f} |")
    if pmc:
        lines += ["", "| kernel | counter | avg / launch |", "|---|---|---|"]
        for k, e in sorted(pmc.items()):
            for name, val in sorted(e.items()):
                lines.append(f"| {k} | {name} | {val:.6g} |")
    open(f"profiles/{tag}_summary.md", "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
