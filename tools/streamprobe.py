#!/usr/bin/env python3
"""Measurement only: the chip's long-stream read rate per access shape
(tools/streamprobe.hip) and the vring kernel's rate against batch-list length.

    python tools/streamprobe.py [probe|list|all]

Serial-region timing as bench.py: HIP events around back-to-back launches on one
stream, a spin kernel ahead.  Buffers rotate so no launch re-reads bytes the
Infinity Cache (256 MiB) could still hold."""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SO = os.path.join(HERE, "libstreamprobe.so")
SRC = os.path.join(HERE, "streamprobe.hip")
sys.path.insert(0, os.path.join(ROOT, "enet-csharp_amd"))

BATCH = 65536 * 1200


def build():
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(SRC):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17",
                        SRC, "-o", SO], check=True)


def region_us(torch, st, fn, reps):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        torch.cuda._sleep(int(2e8))
        e0.record(st)
        for i in range(reps):
            fn(i)
        e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    build()
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what == "build":
        return
    import torch
    st = torch.cuda.Stream()
    nb = 40
    big = torch.empty(nb * BATCH + 8192, dtype=torch.uint8, device="cuda")
    # fill with something non-constant, chunk by chunk (int64 view)
    v = big[: (big.numel() // 8) * 8].view(torch.int64)
    for c in range(0, v.numel(), 1 << 26):
        w = v[c:c + (1 << 26)]
        w.copy_(torch.arange(c, c + w.numel(), dtype=torch.int64, device="cuda") * 0x9E3779B97F4A7C15)
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    zero = torch.zeros(256, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    h = ctypes.c_void_p(st.cuda_stream)
    if what in ("probe", "all"):
        lib = ctypes.CDLL(SO)
        lib.sp_name.restype = ctypes.c_char_p
        sizes = ((1, 100), (5, 24), (20, 8), (40, 4)) if what == "all" else ((1, 100), (20, 8))
        cfgs = [int(c) for c in os.environ["SP_CFGS"].split(",")] if os.environ.get("SP_CFGS") else None
        for size_batches, reps in sizes:
            size = size_batches * BATCH
            slots = max(1, nb // size_batches)
            for cfg in cfgs or range(lib.sp_ncfg()):
                def fn(i, cfg=cfg, size=size):
                    base = big.data_ptr() + (i % slots) * size
                    rc = lib.sp_run(cfg, ctypes.c_void_p(base), ctypes.c_uint64(size), ctypes.c_uint32(1200),
                                    ctypes.c_void_p(zero.data_ptr()), ctypes.c_void_p(sink.data_ptr()), h)
                    assert rc == 0, rc
                us = region_us(torch, st, fn, reps)
                print(json.dumps({"kind": "probe", "name": lib.sp_name(cfg).decode(), "MB": size / 1e6,
                                  "us": round(us, 2), "GBps": round(size / us / 1e3, 1)}), flush=True)
    if what in ("list", "all", "abl", "abl8", "pol", "ls"):
        import enethip
        lanes = int(os.environ.get("SP_LANES", "4"))
        combos = [(w, p, 0) for w in (2, 1) for p in (17, 18)]
        if what == "list":
            combos = [(0, 13, 0), (2, 17, 0)]
        if what == "abl8":
            combos = [(w, p, a) for w in (2, 1) for p in (17, 18) for a in (2048 + 4096 + 16384 + 32768,)]
            combos += [(w, 17, 2048 + 4096 + 32768) for w in (2, 1)]
            lanes = 8
        if what == "ls":
            # line-shaped stage loads + 128-B windows (ABL 8, wrong CRCs by design) with the
            # full fold, and its skeleton (ABL 27), plain (17) and nt (18), against the product
            combos = [(w, p, a) for w in (2, 1) for p in (17, 18) for a in (0, 16384, 2048 + 4096 + 16384 + 32768)]
            lanes = 8
        if what == "pol":
            combos = [(w, p, a) for w in (2, 1) for p in (17, 18) for a in (0, 65536)]
        if what == "abl":
            combos = [(w, 17, a) for w in (2, 1) for a in (0, 4096, 2048 + 4096 + 32768)]
        for wgs, path, abl in combos:
            ctx = enethip.Context(0, (8 if lanes == 4 else lanes) if (path == 13 and what == "list") else lanes, wgs,
                                  diag=True)
            ctx.set_kernel_path(path)
            ctx.diag_ablation(abl)
            off = torch.arange(65536, dtype=torch.int64, device="cuda") * 1200
            lens = torch.full((65536,), 1200, dtype=torch.int32, device="cuda")
            outs = [torch.zeros(65536, dtype=torch.int32, device="cuda") for _ in range(nb)]
            descs = [(big[j * BATCH:(j + 1) * BATCH + 4096], off, lens, 65536, outs[j]) for j in range(nb)]
            for L in ((5, 20) if what.startswith("abl") or what in ("pol", "ls") else (1, 2, 5, 10, 20, 40)):
                launches = max(4, 80 // L)

                def fn(i, L=L):
                    first = (i * L) % nb
                    ctx.crc32_batch_list_device([descs[(first + t) % nb] for t in range(L)], st.cuda_stream)
                us = region_us(torch, st, fn, launches)
                print(json.dumps({"kind": "vring-list", "abl": abl, "path": path, "lanes": lanes, "wgs": wgs, "list": L, "us_per_launch": round(us, 2),
                                  "us_per_batch": round(us / L, 3), "GBps": round(L * BATCH / us / 1e3, 1)}), flush=True)
            ctx.close()
    if what == "big":
        # one batch of 20 cfg2 batches' packets (1.57 GB): per-launch start and drain amortised
        import enethip
        n = 20 * 65536
        off = torch.arange(n, dtype=torch.int64, device="cuda") * 1200
        lens = torch.full((n,), 1200, dtype=torch.int32, device="cuda")
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        for path, lanes, wgs in ((17, 4, 2), (17, 4, 1), (17, 8, 2), (13, 8, 0), (13, 4, 0), (14, 8, 0), (14, 4, 0)):
            ctx = enethip.Context(0, lanes, wgs, diag=True)
            ctx.set_kernel_path(path)

            def fn(i, ctx=ctx):
                base = big[(i % 2) * 20 * BATCH:]
                ctx.crc32_batch_device(base, off, lens, n, out, st.cuda_stream)
            us = region_us(torch, st, fn, 8)
            print(json.dumps({"kind": "one-big-batch", "path": path, "lanes": lanes, "wgs": wgs, "MB": n * 1200 / 1e6,
                              "us": round(us, 2), "GBps": round(n * 1200 / us / 1e3, 1)}), flush=True)
            ctx.close()
    print("done", flush=True)


if __name__ == "__main__":
    main()
