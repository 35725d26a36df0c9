#!/usr/bin/env python3
"""Measurement only: the vring kernel's end records (trace instance TR = 2, the
product's code path) for the dynamic rounds and the static deal on one cfg2 batch
list -- groups per wave and their sum (every group exactly once: the sum equals the
launch's groups), slots taken, per-wave end times -- and the two deals' CRCs compared.
    python tools/dyn_probe.py [list=5] [wgs=2] [lanes=8]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "enet-csharp_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import enethip  # noqa: E402

BATCH = 65536 * 1200
END_RECORDS = 128 << 11          # enet_hip_diag_ablation: the end-record trace instance
DYNAMIC = 524288                 # ... the dynamic rounds


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    wgs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    lanes = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    big = torch.randint(0, 255, (L * BATCH + 4096,), dtype=torch.uint8, device="cuda")
    off = torch.arange(65536, dtype=torch.int64, device="cuda") * 1200
    lens = torch.full((65536,), 1200, dtype=torch.int32, device="cuda")
    ctx = enethip.Context(0, lanes, wgs, diag=True)
    nw = 256 * wgs * 16
    tr = torch.zeros(nw * 8, dtype=torch.int64, device="cuda")
    groups_total = L * 65536 // (64 // lanes)
    res = {}
    for name, mode in (("dynamic", END_RECORDS | DYNAMIC), ("static", END_RECORDS)):
        ctx.diag_ablation(mode)
        ctx.diag_trace(tr)
        outs = [torch.zeros(65536, dtype=torch.int32, device="cuda") for _ in range(L)]
        descs = [(big[j * BATCH:], off, lens, 65536, outs[j]) for j in range(L)]
        for rep in range(3):
            tr.zero_()
            for o in outs:
                o.fill_(-1)
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            ctx.crc32_batch_list_device(descs, torch.cuda.current_stream().cuda_stream)
            ev1.record()
            torch.cuda.synchronize()
            t = tr.cpu().numpy().view(np.uint64).reshape(nw, 8)
            t = t[t[:, 5] > 0]
            end = (t[:, 5].astype(np.int64) - np.int64(t[:, 5].min())) / 100.0
            groups = t[:, 7].astype(np.int64)
            taken = t[:, 0].astype(np.int64)
            print(json.dumps({"deal": name, "rep": rep, "launch_us": round(ev0.elapsed_time(ev1) * 1000, 2),
                              "waves": int(len(t)), "groups_sum": int(groups.sum()), "groups_total": groups_total,
                              "groups_min_max": [int(groups.min()), int(groups.max())],
                              "taken_min_max": [int(taken.min()), int(taken.max())],
                              "last_slot_max": int(t[:, 1].max()),
                              "end_spread_us_p10_p50_max": [round(float(np.percentile(end, 10)), 2),
                                                            round(float(np.median(end)), 2), round(float(end.max()), 2)]}),
                  flush=True)
        res[name] = torch.stack(outs).cpu().numpy()
    print(json.dumps({"crcs_equal": bool((res["dynamic"] == res["static"]).all()),
                      "unwritten_dynamic": int((res["dynamic"] == -1).sum())}))
    ctx.diag_trace(None)
    ctx.diag_ablation(0)


if __name__ == "__main__":
    main()
