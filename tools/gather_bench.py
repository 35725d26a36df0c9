#!/usr/bin/env python3
"""Send-side gather-list CRC throughput (c/protocol.cs:1690-1698, SURVEY §8a a5 and
§8f row 2) on cfg5: 4096 x 64 KiB messages -> 200 704 DGRAMs, each a 3-buffer gather
list [8 B header+slot][24 B SendFragment][1360 or 256 B chunk], device-resident.
Algorithmic bytes per call = the DGRAM bytes (274.9 MB).  Times
enet_hip_crc32_gather_device (one lane per DGRAM) against
enet_hip_crc32_gather_binned_device (a length-binned checksum pass over the 602 112
segments, then a join per DGRAM), serial region as bench.py's roofline: HIP events on
the launch stream around back-to-back calls, a spin kernel ahead.  Both outputs are
checked against the oracle first.

    python tools/gather_bench.py [--messages 4096] [--reps 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "enet-csharp_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402


def cpu_gather(lib, g, budget_s: float, runs: int = 5) -> dict:
    """The oracle's gather (kind "port") on contiguous DGRAM ranges, one Python thread
    per range (the ctypes call releases the GIL): 1 thread, then bench.py's thread
    count; GiB/s of DGRAM bytes, the median of `runs` runs over a sample sized to the
    budget."""
    import threading
    import time
    sys.path.insert(0, ROOT)
    import bench
    threads, info = bench.baseline_threads(0)
    sf = g.seg_first.astype(np.uint64)
    lens = g.seg_len.astype(np.uint64)
    csum = np.concatenate([[0], np.cumsum(lens)])
    dbytes = csum[sf[1:]] - csum[sf[:-1]]                   # bytes per DGRAM

    def run(n_dg: int, th: int) -> float:
        cuts = np.linspace(0, n_dg, th + 1).astype(np.int64)
        ts = [threading.Thread(target=lib.gather, args=(g.payload, g.seg_off, g.seg_len,
                                                         g.seg_first[cuts[i]:cuts[i + 1] + 1]))
              for i in range(th)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        return time.perf_counter() - t0

    res = {"kind": "port", "host": info, "unit": "GiB/s of DGRAM bytes"}
    for label, th in (("1thread", 1), ("all", threads)):
        k = min(g.n, 2000 * th)
        dt = max(run(k, th), 1e-6)
        rate = float(dbytes[:k].sum()) / dt
        n_dg = int(min(g.n, max(k, k * (budget_s / 2 / runs) * rate / max(1.0, float(dbytes[:k].sum())))))
        nb = float(dbytes[:n_dg].sum())
        rates = [nb / run(n_dg, th) / 2 ** 30 for _ in range(runs)]
        res[label] = dict(gibps=round(float(np.median(rates)), 3), threads=th, dgrams=n_dg, runs=runs,
                          spread=[round(min(rates), 3), round(max(rates), 3)])
    res["speedup"] = round(res["all"]["gibps"] / max(res["1thread"]["gibps"], 1e-9), 2)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--messages", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--wgs", type=int, default=0, help="workgroups per CU (enet_hip_set_tuning; 0 = default)")
    ap.add_argument("--path", type=int, default=0, help="kernel path (enet_hip_set_kernel_path; 17 = vring records)")
    ap.add_argument("--only", choices=["gather", "gather_binned"], help="time one entry only")
    ap.add_argument("--ablate", type=int, default=0, help="diagnostics: enet_hip_diag_ablation after the oracle "
                                                               "check (wrong CRCs by design)")
    ap.add_argument("--cpu-seconds", type=float, default=0.0,
                    help="also time the oracle's gather (the 3-buffer lists, packet.cs:142-160 over "
                         "protocol.cs:1690-1698's buffers) on this host: 1 thread and the cores the process may "
                         "use (quota-capped, bench.py's rule), median of 5 runs, this many seconds in all")
    ap.add_argument("--probe", type=int, default=0, help="then run the read probe N times over the arena "
                                                              "(FETCH_SIZE calibration)")
    a = ap.parse_args()
    import torch
    import enethip
    from enethip import workloads
    import oracle as orc
    g = workloads.cfg5(a.messages)
    ctx = enethip.Context(0, a.lanes, a.wgs, diag=a.path not in (0, 13, 17) or a.lanes not in (0, 4, 8) or a.ablate != 0)
    if a.path:
        ctx.set_kernel_path(a.path)
    st = torch.cuda.Stream()
    t = lambda x, dt: torch.from_numpy(np.ascontiguousarray(x).view(dt)).cuda()  # noqa: E731
    d_p, d_so, d_sl, d_sf = t(g.payload, np.uint8), t(g.seg_off, np.int64), t(g.seg_len, np.int32), t(g.seg_first, np.int32)
    ns = int(g.seg_first[-1])
    out = torch.zeros(g.n, dtype=torch.int32, device="cuda")
    wsb = ctx.gather_binned_workspace_size(ns)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")

    def plain(_i):
        ctx.gather_device(d_p, d_so, d_sl, d_sf, g.n, out, st.cuda_stream)

    def binned(_i):
        ctx.gather_binned_device(d_p, d_so, d_sl, ns, d_sf, g.n, out, ws, wsb, st.cuda_stream)

    exp = orc.OracleLib().gather(g.payload, g.seg_off, g.seg_len, g.seg_first)
    res = {"kind": "gather-bench", "dgrams": g.n, "segments": ns, "bytes": g.dgram_bytes,
           "lanes": a.lanes or "default"}
    for name, fn in (("gather", plain), ("gather_binned", binned)):
        if a.only and name != a.only:
            continue
        out.zero_()
        fn(0)
        torch.cuda.synchronize()
        ok = bool((out.cpu().numpy().view(np.uint32) == exp).all())
        assert ok, name + " differs from the oracle"
        if a.ablate:
            ctx.diag_ablation(a.ablate)
            res["ablation"] = a.ablate
        for i in range(3):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(st):
            torch.cuda._sleep(int(2e8))
            e0.record(st)
            for i in range(a.reps):
                fn(i)
            e1.record(st)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.reps * 1e3
        res[name + "_us"] = round(us, 2)
        res[name + "_GBps"] = round(g.dgram_bytes / us / 1e3, 1)
        res[name + "_GiBps"] = round(g.dgram_bytes / us * 1e6 / 2 ** 30, 1)
        res[name + "_bit_exact"] = ok
        if a.ablate:
            ctx.diag_ablation(0)
    if a.cpu_seconds > 0:
        res["cpu_baseline"] = cpu_gather(orc.OracleLib(), g, a.cpu_seconds)
    if a.probe:
        sink = torch.zeros(4, dtype=torch.int32, device="cuda")
        for _ in range(a.probe):
            ctx.read_probe_device(d_p, (d_p.numel() // 16) * 16, sink, st.cuda_stream)
        torch.cuda.synchronize()
        res["probe_bytes"] = (d_p.numel() // 16) * 16
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
