#!/usr/bin/env python3
"""Length-binned checksum entry (enet_hip_crc32_batch_device_binned, packet.cs:142-160 per
DGRAM) in the serial form, on cfg3-shaped batches of several sizes: does the records
kernel's shortfall against its load shape scale with the launch (a fixed ramp / drain)
or with the bytes?  Each size is a packed U[64, 1400] B batch (workloads.mixed); its
copies rotate so at least 768 MB is cycled (> the 256 MB MALL).  Timing: HIP events on
one stream around back-to-back calls (bin kernel + records kernel each), a spin kernel
ahead.  Checked bit-exact against the plain checksum entry on copy 0.

    python tools/binned_bench.py [--sizes 262144,524288,1048576] [--reps 30] [--ablate 38912]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "enet-csharp_amd"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="262144,524288,1048576")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--min-bytes", type=float, default=768e6)
    ap.add_argument("--ablate", type=int, default=0, help="diagnostics ablation (38912: the records skeleton)")
    a = ap.parse_args()
    import torch
    import enethip
    from enethip import workloads
    ctx = enethip.Context(0, diag=bool(a.ablate))
    st = torch.cuda.Stream()
    h = st.cuda_stream
    for n in (int(s) for s in a.sizes.split(",")):
        b = workloads.mixed(n)
        nbytes = b.payload_bytes
        copies = max(1, int(np.ceil(a.min_bytes / nbytes)))
        with torch.cuda.stream(st):
            pay = [torch.from_numpy(b.payload).cuda() for _ in range(copies)]
            d_off = torch.from_numpy(b.off.view(np.int64)).cuda()
            d_len = torch.from_numpy(b.lens.view(np.int32)).cuda()
            outs = [torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(copies)]
            wsb = ctx.binned_workspace_size(n)
            ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
            ref = torch.zeros(n, dtype=torch.int32, device="cuda")
        st.synchronize()
        ctx.crc32_batch_device(pay[0], d_off, d_len, n, ref, h)
        ctx.crc32_batch_device_binned(pay[0], d_off, d_len, n, outs[0], ws, wsb, h)
        st.synchronize()
        ok = bool(torch.equal(ref, outs[0]))
        if a.ablate:
            ctx.diag_ablation(a.ablate)               # (from here on the CRCs are wrong by design)
        for r in range(3):
            ctx.crc32_batch_device_binned(pay[r % copies], d_off, d_len, n, outs[r % copies], ws, wsb, h)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(st):
            torch.cuda._sleep(2_000_000)
            e0.record(st)
            for r in range(a.reps):
                ctx.crc32_batch_device_binned(pay[r % copies], d_off, d_len, n, outs[r % copies], ws, wsb, h)
            e1.record(st)
        st.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        print(json.dumps({"n": n, "payload_mb": round(nbytes / 1e6, 1), "copies": copies, "us_per_call": round(us, 2),
                          "tb_s": round(nbytes / (us * 1e-6) / 1e12, 3), "frac": round(nbytes / (us * 1e-6) / 8e12, 4),
                          "bit_exact": ok, "ablate": a.ablate}), flush=True)
        if a.ablate:
            ctx.diag_ablation(0)
        del pay, outs, ws, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
