#!/usr/bin/env python3
"""Per-wave timeline of the lean kernel (enet_hip_diag_trace): start / table
barrier / end of every wave of one launch, relative to the earliest start, in us
(s_memrealtime ticks at 100 MHz).  Prints percentiles and per-XCC spread.

    python tools/timeline.py [--config cfg2] [--lanes 8] [--path 0] [--reps 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "enet-csharp_amd"))

import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--lanes", type=int, default=8)
    ap.add_argument("--path", type=int, default=0)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--waves", type=int, default=16)
    ap.add_argument("--ablate", type=int, default=0)
    a = ap.parse_args()
    import torch
    batches = bench.make_batches(a.config, 5, 0)
    eng = bench.GpuEngine(0, batches, a.lanes, 0, diag=True)
    eng.ctx.set_kernel_path(a.path)
    eng.ctx.diag_ablation(a.ablate)
    nw = 256 * a.waves
    tr = torch.zeros(nw * 8, dtype=torch.int64, device="cuda")
    eng.ctx.diag_trace(tr)
    res = []
    for i in range(a.reps):
        tr.zero_()
        eng.step(i)
        eng.sync()
        res.append(tr.cpu().numpy().view(np.uint64).reshape(nw, 8).copy())
    eng.ctx.diag_trace(None)
    analyze(res)


def analyze(traces):
    """traces: list of (waves, 4) uint64 arrays [start, barrier, end, HW_ID | XCC << 32]
    or (waves, 8) [start, meta, table, barrier, first stage, end, HW_ID | XCC << 32, groups]."""
    res = []
    for t in traces:
        t = t[t[:, 0] > 0]
        t0 = t[:, 0].min()
        rel = lambda c: (t[:, c].astype(np.int64) - np.int64(t0)).astype(np.float64) / 100.0
        if t.shape[1] == 4:
            d = dict(start=rel(0), bar=rel(1), end=rel(2), xcc=(t[:, 3] >> np.uint64(32)).astype(np.int64))
        else:
            d = dict(start=rel(0), meta=rel(1), table=rel(2), bar=rel(3), first=rel(4), end=rel(5),
                     xcc=(t[:, 6] >> np.uint64(32)).astype(np.int64))
            hw = (t[:, 6] & np.uint64(0xFFFFFFFF)).astype(np.int64)
            # HW_ID: CU_ID [11:8], SH_ID [12], SE_ID [15:13]; SIMD_ID [5:4]
            d["cu"] = d["xcc"] * 4096 + ((hw >> 8) & 0xFF)
            d["simd"] = (hw >> 4) & 3
            d["first"] = np.where(t[:, 4] > 0, d["first"], np.nan)
        res.append(d)
    pct = [0, 10, 50, 90, 100]
    for key in ("start", "meta", "table", "bar", "first", "end"):
        if key not in res[0]:
            continue
        v = np.concatenate([r[key] for r in res[2:]])
        v = v[~np.isnan(v)]
        print(json.dumps({key: {f"p{p}": round(float(np.percentile(v, p)), 2) for p in pct}}))
    dur = np.concatenate([r["end"] - r["bar"] for r in res[2:]])
    print(json.dumps({"end-bar": {f"p{p}": round(float(np.percentile(dur, p)), 2) for p in pct}}))
    for r in res[-2:]:
        per = {}
        for x in sorted(set(r["xcc"].tolist())):
            m = r["xcc"] == x
            per[int(x)] = dict(n=int(m.sum()), start_min=round(float(r["start"][m].min()), 2),
                               start_max=round(float(r["start"][m].max()), 2),
                               bar_p50=round(float(np.median(r["bar"][m])), 2),
                               end_p50=round(float(np.median(r["end"][m])), 2),
                               end_max=round(float(r["end"][m].max()), 2))
        print(json.dumps({"per_xcc": per}))
    print(json.dumps({"kernel_span_us_per_rep": [round(float(x["end"].max()), 2) for x in res]}))
    if "cu" in res[-1]:
        r = res[-1]
        cus = sorted(set(r["cu"].tolist()))
        lo = np.array([r["end"][r["cu"] == c].min() for c in cus])
        hi = np.array([r["end"][r["cu"] == c].max() for c in cus])
        med = np.array([np.median(r["end"][r["cu"] == c]) for c in cus])
        print(json.dumps({"cus": len(cus), "cu_end_min_p50": round(float(np.median(lo)), 2),
                          "cu_end_max_p10_p50_p90_p100": [round(float(np.percentile(hi, q)), 2) for q in (10, 50, 90, 100)],
                          "within_cu_spread_p50": round(float(np.median(hi - lo)), 2),
                          "cu_median_end_p10_p90": [round(float(np.percentile(med, q)), 2) for q in (10, 90)]}))
        # end time by wave slot in the workgroup (row i of the trace is wave i % W)
        nw = len(r["end"])
        W = 16
        slots = np.arange(nw) % W
        print(json.dumps({"end_p50_by_wave_slot": [round(float(np.median(r["end"][slots == w])), 2) for w in range(W)]}))
        print(json.dumps({"first_p50_by_wave_slot": [round(float(np.nanmedian(r["first"][slots == w])), 2) for w in range(W)]}))
        st = r["end"] - r["bar"]
        for sm in range(4):
            m = r["simd"] == sm
            print(json.dumps({"simd": sm, "n": int(m.sum()), "stream_p50": round(float(np.median(st[m])), 2)}))

if __name__ == "__main__":
    main()
