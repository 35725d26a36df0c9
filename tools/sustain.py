#!/usr/bin/env python3
"""Measurement only: per-launch duration of back-to-back batch-list launches over a
long serial run (HIP events between launches), to see whether the rate drops once
the chip has streamed for a while (power / clock management).
    python tools/sustain.py [launches=400] [list=5] [path=0]"""
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
    launches = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    path = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    nb = 10
    big = torch.randint(0, 255, (nb * BATCH + 4096,), dtype=torch.uint8, device="cuda")
    off = torch.arange(65536, dtype=torch.int64, device="cuda") * 1200
    lens = torch.full((65536,), 1200, dtype=torch.int32, device="cuda")
    outs = [torch.zeros(65536, dtype=torch.int32, device="cuda") for _ in range(nb)]
    descs = [(big[j * BATCH:], off, lens, 65536, outs[j]) for j in range(nb)]
    ctx = enethip.Context(0, 0, 2)
    ctx.set_kernel_path(path)
    st = torch.cuda.Stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(launches + 1)]
    for i in range(5):
        ctx.crc32_batch_list_device([descs[(i * L + t) % nb] for t in range(L)], st.cuda_stream)
    torch.cuda.synchronize()
    with torch.cuda.stream(st):
        torch.cuda._sleep(int(4e8))
        ev[0].record(st)
        for i in range(launches):
            ctx.crc32_batch_list_device([descs[(i * L + t) % nb] for t in range(L)], st.cuda_stream)
            ev[i + 1].record(st)
    torch.cuda.synchronize()
    us = np.array([ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(launches)])
    t = np.cumsum(us)
    for k in range(0, launches, max(1, launches // 20)):
        sl = us[k:k + max(1, launches // 20)]
        print(json.dumps({"from_us": round(float(t[k] - us[k]), 1), "launches": len(sl),
                          "us_per_launch": round(float(sl.mean()), 2),
                          "TBps": round(L * BATCH / float(sl.mean()) / 1e6, 3)}), flush=True)
    print(json.dumps({"total_us": round(float(t[-1]), 1), "mean_TBps": round(L * BATCH * launches / float(t[-1]) / 1e6, 3)}))


if __name__ == "__main__":
    main()
