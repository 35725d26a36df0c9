#!/usr/bin/env python3
"""Per-dispatch durations of one kernel from a rocprofv3 --kernel-trace CSV
(measurement infrastructure): count, mean, median, min, max in microseconds,
optionally skipping the first K dispatches (a one-batch oracle gate, warmup) and
keeping only dispatches with a given grid size.

    python tools/trace_stats.py run_kernel_trace.csv --match crc32_vring_kernel<3 [--skip K] [--grid G] [--out f.json]
"""
import argparse
import csv
import glob
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace", help="run_kernel_trace.csv or a directory holding one")
    ap.add_argument("--match", required=True)
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--out")
    a = ap.parse_args()
    path = a.trace if a.trace.endswith(".csv") else glob.glob(f"{a.trace}/**/*kernel_trace.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(path)) if a.match in r["Kernel_Name"]
            and (not a.grid or int(r["Grid_Size_X"]) == a.grid)]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    kept = rows[a.skip:]
    us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in kept]
    # overlap: dispatches on several streams run concurrently, so each one's own
    # duration counts the time it shared with its neighbours; the union of the
    # intervals is the time the kernel occupied the GPU at all
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kept)
    union, cur = 0, None
    for s0, e0 in iv:
        if cur is None or s0 > cur[1]:
            if cur is not None:
                union += cur[1] - cur[0]
            cur = [s0, e0]
        else:
            cur[1] = max(cur[1], e0)
    if cur is not None:
        union += cur[1] - cur[0]
    doc = {"trace": path, "match": a.match, "skipped": a.skip, "dispatches": len(us),
           "mean_us": round(statistics.mean(us), 3) if us else None,
           "median_us": round(statistics.median(us), 3) if us else None,
           "min_us": round(min(us), 3) if us else None, "max_us": round(max(us), 3) if us else None,
           "union_us": round(union / 1e3, 3) if iv else None,
           "union_per_dispatch_us": round(union / 1e3 / len(iv), 3) if iv else None,
           "span_us": round((max(e for _, e in iv) - iv[0][0]) / 1e3, 3) if iv else None}
    print(json.dumps(doc))
    if a.out:
        json.dump(doc, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
