#!/usr/bin/env python3
"""Measurement only: per-wave end times of one vring batch-list launch (the trace
instance, enet_hip_diag_trace): how long the waves that finish first wait for the
last, i.e. what a static deal of groups over waves costs a single launch.
    python tools/list_timeline.py [list=20] [wgs=2] [lanes=4]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "enet-csharp_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import enethip  # noqa: E402

BATCH = 65536 * 1200


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    wgs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    lanes = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    big = torch.randint(0, 255, (L * BATCH + 4096,), dtype=torch.uint8, device="cuda")
    off = torch.arange(65536, dtype=torch.int64, device="cuda") * 1200
    lens = torch.full((65536,), 1200, dtype=torch.int32, device="cuda")
    outs = [torch.zeros(65536, dtype=torch.int32, device="cuda") for _ in range(L)]
    descs = [(big[j * BATCH:], off, lens, 65536, outs[j]) for j in range(L)]
    ctx = enethip.Context(0, lanes, wgs, diag=True)
    nw = 256 * wgs * 16
    tr = torch.zeros(nw * 8, dtype=torch.int64, device="cuda")
    ctx.diag_trace(tr)
    for rep in range(3):
        tr.zero_()
        ctx.crc32_batch_list_device(descs, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        t = tr.cpu().numpy().view(np.uint64).reshape(nw, 8)
        if os.environ.get("TIMELINE_DUMP"):                  # raw records for offline analysis
            np.save(f"{os.environ['TIMELINE_DUMP']}_l{L}_w{wgs}_p{lanes}_r{rep}.npy", t)
        t = t[t[:, 0] > 0]
        t0 = t[:, 0].min()
        rel = lambda c: (t[:, c].astype(np.int64) - np.int64(t0)) / 100.0
        start, first, end = rel(0), rel(4), rel(5)
        groups = t[:, 7].astype(np.int64)
        hw = (t[:, 6] & np.uint64(0xFFFFFFFF)).astype(np.int64)
        simd = (hw >> 4) & 3
        cu = ((hw >> 8) & 15) + 16 * ((hw >> 13) & 1) + 32 * ((hw >> 16) & 7)   # HW_ID: CU, SH, SE
        xcc = (t[:, 6] >> np.uint64(32)).astype(np.int64)
        span = end.max()
        # per CU: how long its first-finishing wave idles until its last one ends
        key = xcc * 4096 + cu
        idle = []
        for k in np.unique(key):
            e = end[key == k]
            idle.append(float((e.max() - e).mean()))
        busy = float(((end - first) * 1.0).sum() / (len(end) * span))
        # per XCD (the end of its last wave, the median of its waves' ends) and per
        # workgroup (trace row = 16 x workgroup + wave; its end = its last wave's)
        rows = np.nonzero(tr.cpu().numpy().view(np.uint64).reshape(nw, 8)[:, 0] > 0)[0]
        wg = rows // 16
        wg_end = np.array([end[wg == g].max() for g in np.unique(wg)])
        xcd_end = {int(x): [round(float(np.median(end[xcc == x])), 1), round(float(end[xcc == x].max()), 1)]
                   for x in np.unique(xcc)}
        print(json.dumps({"list": L, "wgs": wgs, "lanes": lanes, "waves": int(len(end)), "span_us": round(float(span), 2),
                          "start_p50_us": round(float(np.median(start)), 2), "first_stage_p50_us": round(float(np.median(first)), 2),
                          "end_min_us": round(float(end.min()), 2), "end_p10_us": round(float(np.percentile(end, 10)), 2),
                          "end_p50_us": round(float(np.median(end)), 2), "end_p90_us": round(float(np.percentile(end, 90)), 2),
                          "end_max_us": round(float(end.max()), 2),
                          "mean_idle_after_own_end_in_cu_us": round(float(np.mean(idle)), 2),
                          "wave_busy_fraction": round(busy, 3),
                          "groups_min_max": [int(groups.min()), int(groups.max())],
                          "wg_end_p10_p50_max_us": [round(float(np.percentile(wg_end, 10)), 1),
                                                    round(float(np.median(wg_end)), 1), round(float(wg_end.max()), 1)],
                          "xcd_end_p50_max_us": xcd_end}), flush=True)
    ctx.diag_trace(None)


if __name__ == "__main__":
    main()
