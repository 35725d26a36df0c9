#!/usr/bin/env python3
"""Diagnostics: where the vring kernel's own ceiling lies, apart from HBM.

Times serial 5-batch list launches (HIP events around R back-to-back launches, a spin
kernel ahead so host launch cost cannot idle the GPU) of the product kernel, 8 lanes,
on the same packet shape (65 536 x 1200 B per batch) served from three levels:

  hbm  -- five distinct resident batches (375 MiB, past the 256 MiB Infinity Cache):
          the bench's workload;
  mall -- one 78.6 MB batch listed five times (Infinity-Cache resident after the
          first pass);
  l2   -- 65 536 packets whose offsets cycle over 64 packets' bytes (76.8 KB):
          every stage load hits L2, so the kernel's instruction stream alone sets
          the time (the fold, waits, windows, group switches).

With --path 17 / 18 (diagnostics library) the vring with default / nontemporal stage
loads; with --ablation M (diagnostics library) the same on an ablated instance (38912 = the
8-lane skeleton: no lookups, masks or end corrections; WRONG CRCs by design, so the
check is skipped).  Rates are payload bytes / kernel time (TB/s) and fraction of 8 TB/s.
    python tools/ceiling.py [--ablation M] [--wgs W] [--reps R]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "enet-csharp_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import enethip  # noqa: E402
from enethip import workloads  # noqa: E402

N, L = 65_536, 1200


def dev(a):
    a = np.ascontiguousarray(a)
    view = {np.dtype(np.uint64): np.int64, np.dtype(np.uint32): np.int32, np.dtype(np.uint8): np.uint8}[a.dtype]
    return torch.from_numpy(a.view(view)).cuda()


def region_us(ctx, descs, reps, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        torch.cuda._sleep(int(2e8))
        e0.record(stream)
        for _ in range(reps):
            ctx.crc32_batch_list_device(descs, stream=stream.cuda_stream)
        e1.record(stream)
    torch.cuda.synchronize()
    return 1e3 * e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ablation", type=int, default=0)
    ap.add_argument("--wgs", type=int, default=0)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--levels", default="hbm,mall,l2")
    ap.add_argument("--path", type=int, default=0, help="kernel path (diagnostics: 17 = vring, 18 = vring nt)")
    args = ap.parse_args()
    torch.cuda.init()
    ctx = enethip.Context(0, 8, args.wgs, diag=args.ablation != 0 or args.path != 0)
    if args.path:
        ctx.set_kernel_path(args.path)
    if args.ablation:
        ctx.diag_ablation(args.ablation)
    stream = torch.cuda.Stream()
    check = args.ablation == 0
    cb = workloads.cfg2()
    oracle = None
    if check:
        import oracle as orc
        oracle = orc.OracleLib()
    res = {"ablation": args.ablation, "path": args.path, "wgs": args.wgs or "default", "reps": args.reps}
    for level in args.levels.split(","):
        keep, descs, expect = [], [], []
        if level == "hbm":
            for k in range(5):
                b = cb if k == 0 else workloads.fixed(N, L, seed=1000 + k)
                d = (dev(b.payload), dev(b.off), dev(b.lens))
                keep.append(d)
                expect.append(oracle.batch(b.payload, b.off, b.lens, threads=8) if check else None)
                descs.append([d[0], d[1], d[2], N, None])
        elif level == "mall":
            d = (dev(cb.payload), dev(cb.off), dev(cb.lens))
            keep.append(d)
            e = oracle.batch(cb.payload, cb.off, cb.lens, threads=8) if check else None
            for k in range(5):
                expect.append(e)
                descs.append([d[0], d[1], d[2], N, None])
        else:
            small = cb.payload[:64 * L].copy()
            off = (np.arange(N, dtype=np.uint64) % 64) * L
            lens = np.full(N, L, np.uint32)
            d = (dev(small), dev(off), dev(lens))
            keep.append(d)
            e = oracle.batch(small, off, lens, threads=8) if check else None
            for k in range(5):
                expect.append(e)
                descs.append([d[0], d[1], d[2], N, None])
        outs = [torch.full((N,), -1, dtype=torch.int32, device="cuda") for _ in descs]
        for dd, o in zip(descs, outs):
            dd[4] = o
        descs = [tuple(x) for x in descs]
        region_us(ctx, descs, 3, stream)                      # warm
        ok = None
        if check:
            ok = all((o.cpu().numpy().view(np.uint32) == e).all() for o, e in zip(outs, expect))
            if not ok:
                raise SystemExit(f"ceiling.py: {level} CRCs differ from the oracle")
        us = [region_us(ctx, descs, args.reps, stream) for _ in range(3)]
        us_med = float(np.median(us))
        tbs = 5 * N * L / (us_med * 1e-6) / 1e12
        res[level] = {"us_per_launch": round(us_med, 2), "us_all": [round(x, 2) for x in us], "TBps": round(tbs, 3),
                      "frac_of_8TBps": round(tbs / 8.0, 4), "checked": ok}
        print(level, res[level], flush=True)
        del keep, descs, outs
        torch.cuda.synchronize()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
