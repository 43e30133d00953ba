"""Per-batch timeline of a rocprofv3 kernel trace -> profiles/<tag>_timeline.{json,md}.

Usage: python tools/timeline_summary.py <tag> <trace_dir> [--seg I]

A batch (one dsr_batch_run) starts with its k_init_state launch; segment I (default: the
second-to-last, i.e. a complete batch after warm-up) is summarised: device span (first
start to last end), busy time (union of kernel intervals over all streams), per-kernel
launches / summed and average duration, and the launch gaps on the busiest stream — what a
small batch spends between kernels rather than in them.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "").replace("dsr::", "")


def main():
    tag, tdir = sys.argv[1], sys.argv[2]
    seg = int(sys.argv[sys.argv.index("--seg") + 1]) if "--seg" in sys.argv else -2
    f = glob.glob(os.path.join(tdir, "*_kernel_trace.csv"))[0]
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Stream_Id"])
                for r in csv.DictReader(open(f)))
    starts = [i for i, e in enumerate(ev) if e[2].startswith("k_init_state")]
    lo = starts[seg]
    hi = starts[seg + 1] if seg + 1 < len(starts) and seg != -1 else len(ev)
    b = ev[lo:hi]
    # trailing copies / fills of the next batch's upload belong to that batch
    t0, t1 = b[0][0], max(e[1] for e in b)
    busy, cs, ce = 0, None, None
    for s, e, _, _ in b:
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    per = defaultdict(lambda: [0, 0])
    streams = defaultdict(list)
    for s, e, n, st in b:
        per[n][0] += 1
        per[n][1] += e - s
        streams[st].append((s, e))
    main_st = max(streams, key=lambda k: len(streams[k]))
    iv = streams[main_st]
    gaps = [max(0, iv[i + 1][0] - iv[i][1]) for i in range(len(iv) - 1)]
    out = {
        "tag": tag, "trace": os.path.basename(f), "segment": seg, "segments": len(starts),
        "span_ms": (t1 - t0) / 1e6, "busy_ms": busy / 1e6, "streams": len(streams),
        "launches": len(b),
        "busiest_stream": {"launches": len(iv), "kernel_ms": sum(e - s for s, e in iv) / 1e6,
                           "gap_ms": sum(gaps) / 1e6,
                           "median_gap_us": sorted(gaps)[len(gaps) // 2] / 1e3 if gaps else 0.0},
        "kernels": {n: {"calls": c, "total_ms": d / 1e6, "avg_us": d / c / 1e3}
                    for n, (c, d) in sorted(per.items(), key=lambda x: -x[1][1])},
    }
    os.makedirs("profiles", exist_ok=True)
    json.dump(out, open(f"profiles/{tag}_timeline.json", "w"), indent=1)
    bs = out["busiest_stream"]
    md = [f"# kernel timeline `{tag}` (one batch: segment {seg} of {len(starts)})", "",
          f"device span {out['span_ms']:.3f} ms, kernels busy (union over {out['streams']} streams) "
          f"{out['busy_ms']:.3f} ms, {out['launches']} launches; busiest stream: {bs['launches']} launches, "
          f"{bs['kernel_ms']:.3f} ms in kernels, {bs['gap_ms']:.3f} ms between them "
          f"(median gap {bs['median_gap_us']:.1f} us)", "",
          "| kernel | launches | total ms | avg us | % of span |", "|---|---|---|---|---|"]
    for n, k in out["kernels"].items():
        md.append(f"| {n} | {k['calls']} | {k['total_ms']:.3f} | {k['avg_us']:.1f} | "
                  f"{100 * k['total_ms'] / out['span_ms']:.1f} |")
    open(f"profiles/{tag}_timeline.md", "w").write("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main()
