#!/usr/bin/env python3
"""Host-memory (PCIe-inclusive) rates of the checksum path, for DESIGN.md.

  * pcie: the raw H2D rate of the same bytes from pinned memory (enet_hip_memcpy_h2d,
    one synchronous copy) -- the bound every host-memory case below is held against;
  * cfg2 through enet_hip_crc32_batch_host (pipelined: 16-MiB chunks on two streams,
    H2D + kernel + D2H), pinned host buffers;
  * cfg5 (4096 x 64 KiB fragmented sends = 200 704 three-buffer DGRAMs) through
    enet_hip_crc32_gather_binned_host (arena H2D in two halves on two streams, the
    binned gather, D2H), pinned host buffers; and the old one-lane-per-DGRAM gather
    kernel behind synchronous copies, for comparison;
  * cfg2 over 2 contexts of the same device (enet_hip_crc32_batch_multi), the
    multi-GPU entry's host path.
Every result is checked against the oracle.  Prints one JSON line per case.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "enet-csharp_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import enethip  # noqa: E402
from enethip import workloads  # noqa: E402
import oracle  # noqa: E402

GIB = float(1 << 30)


class Pinned:
    def __init__(self, lib, src: np.ndarray):
        self.lib = lib
        self.nbytes = max(16, src.nbytes)
        p = ctypes.c_void_p()
        rc = lib.enet_hip_host_alloc(self.nbytes, ctypes.byref(p))
        if rc:
            raise RuntimeError(f"host_alloc {rc}")
        self.ptr = p.value
        buf = (ctypes.c_uint8 * self.nbytes).from_address(self.ptr)
        self.arr = np.frombuffer(buf, dtype=src.dtype, count=src.size)
        self.arr[:] = src

    def free(self):
        self.lib.enet_hip_host_free(self.ptr)


def timed(fn, reps):
    for _ in range(2):
        fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


def case_pcie(ctx, reps):
    lib = ctx.lib
    n = 78_643_200
    h = Pinned(lib, np.zeros(n, np.uint8))
    p = ctypes.c_void_p()
    assert lib.enet_hip_device_alloc(ctx.handle, n, ctypes.byref(p)) == 0
    dt = timed(lambda: lib.enet_hip_memcpy_h2d(ctx.handle, p.value, h.ptr, n), reps)
    lib.enet_hip_device_free(ctx.handle, p.value)
    h.free()
    return {"case": "raw pinned H2D of 75 MiB (one synchronous hipMemcpy)", "GBps": round(n / dt / 1e9, 2),
            "GiBps": round(n / dt / GIB, 2)}


def case_cfg2(ctx, reps):
    lib = ctx.lib
    b = workloads.cfg2()
    hp, ho, hl = Pinned(lib, b.payload), Pinned(lib, b.off), Pinned(lib, b.lens)
    out = Pinned(lib, np.zeros(b.n, np.uint32))
    call = lambda: lib.enet_hip_crc32_batch_host(ctx.handle, hp.ptr, b.payload.nbytes, ho.ptr, hl.ptr,  # noqa: E731
                                                 b.n, out.ptr)
    assert call() == 0
    exp = oracle.OracleLib().batch(b.payload, b.off, b.lens, threads=8)
    assert (out.arr == exp).all(), "cfg2 host path differs from the oracle"
    dt = timed(call, reps)
    for x in (hp, ho, hl, out):
        x.free()
    return {"case": "cfg2 enet_hip_crc32_batch_host (pipelined: 16-MiB chunks, 2 streams), pinned",
            "payload_bytes": b.payload_bytes, "ms_per_batch": round(dt * 1e3, 4),
            "GiBps": round(b.payload_bytes / dt / GIB, 2), "GBps": round(b.payload_bytes / dt / 1e9, 2)}


def case_cfg2_multi(reps):
    b = workloads.cfg2()
    ctxs = [enethip.Context(0), enethip.Context(0)]
    lib = ctxs[0].lib
    hp = Pinned(lib, b.payload)
    exp = oracle.OracleLib().batch(b.payload, b.off, b.lens, threads=8)
    got = enethip.crc32_batch_multi(ctxs, hp.arr, b.off, b.lens)
    assert (got == exp).all()
    dt = timed(lambda: enethip.crc32_batch_multi(ctxs, hp.arr, b.off, b.lens), reps)
    hp.free()
    for c in ctxs:
        c.close()
    return {"case": "cfg2 enet_hip_crc32_batch_multi, 2 contexts on one device (the multi-GPU host path)",
            "ms_per_batch": round(dt * 1e3, 4), "GiBps": round(b.payload_bytes / dt / GIB, 2),
            "GBps": round(b.payload_bytes / dt / 1e9, 2)}


def case_cfg5(ctx, reps):
    lib = ctx.lib
    g = workloads.cfg5()
    hp = Pinned(lib, g.payload)
    ho, hl, hf = Pinned(lib, g.seg_off), Pinned(lib, g.seg_len), Pinned(lib, g.seg_first)
    out = Pinned(lib, np.zeros(g.n, np.uint32))
    call = lambda: lib.enet_hip_crc32_gather_binned_host(  # noqa: E731
        ctx.handle, hp.ptr, g.payload.nbytes, ho.ptr, hl.ptr, len(g.seg_off), hf.ptr, g.n, out.ptr)
    assert call() == 0
    exp = oracle.OracleLib().gather(g.payload, g.seg_off, g.seg_len, g.seg_first)
    assert (out.arr == exp).all(), "cfg5 host gather differs from the oracle"
    dt = timed(call, reps)
    for x in (hp, ho, hl, hf, out):
        x.free()
    return {"case": "cfg5 enet_hip_crc32_gather_binned_host (arena H2D on 2 streams, binned gather, D2H), pinned",
            "dgram_bytes": g.dgram_bytes, "arena_bytes": int(g.payload.nbytes), "dgrams": g.n,
            "ms_per_batch": round(dt * 1e3, 4), "GiBps": round(g.dgram_bytes / dt / GIB, 2),
            "GBps": round(g.dgram_bytes / dt / 1e9, 2),
            "arena_GBps": round(g.payload.nbytes / dt / 1e9, 2)}


def case_cfg5_slices(ctx, reps):
    """The first k DGRAMs of cfg5 (used arena span about 1.4 KB per DGRAM), pinned: the
    span sizes around the in-place threshold of the gather host entry."""
    lib = ctx.lib
    g = workloads.cfg5()
    hp = Pinned(lib, g.payload)
    ho, hl, hf = Pinned(lib, g.seg_off), Pinned(lib, g.seg_len), Pinned(lib, g.seg_first)
    out = Pinned(lib, np.zeros(g.n, np.uint32))
    exp = oracle.OracleLib().gather(g.payload, g.seg_off, g.seg_len, g.seg_first)
    rows = []
    for k in (64, 768, 3072, 12288, 49152, g.n):
        call = lambda: lib.enet_hip_crc32_gather_binned_host(  # noqa: E731
            ctx.handle, hp.ptr, g.payload.nbytes, ho.ptr, hl.ptr, len(g.seg_off), hf.ptr, k, out.ptr)
        assert call() == 0
        assert (out.arr[:k] == exp[:k]).all(), f"cfg5 slice {k} differs from the oracle"
        s0, s1 = int(g.seg_first[0]), int(g.seg_first[k])
        used = g.seg_len[s0:s1] > 0
        span = int((g.seg_off[s0:s1][used] + g.seg_len[s0:s1][used]).max() - g.seg_off[s0:s1][used].min())
        dt = timed(call, reps if k < g.n else max(3, reps // 4))
        rows.append({"case": "cfg5 slice, enet_hip_crc32_gather_binned_host, pinned", "dgrams": k,
                     "span_bytes": span, "us_per_call": round(dt * 1e6, 1),
                     "span_GBps": round(span / dt / 1e9, 2)})
    for x in (hp, ho, hl, hf, out):
        x.free()
    return rows


def case_cfg2_slices(ctx, reps):
    """The first k packets of cfg2 (1200 B each, contiguous), pinned, through
    enet_hip_crc32_batch_host: in place up to a 4-MiB span, copied beyond."""
    lib = ctx.lib
    b = workloads.cfg2()
    hp, ho, hl = Pinned(lib, b.payload), Pinned(lib, b.off), Pinned(lib, b.lens)
    out = Pinned(lib, np.zeros(b.n, np.uint32))
    exp = oracle.OracleLib().batch(b.payload, b.off, b.lens, threads=8)
    rows = []
    for k in (8, 64, 512, 3495, 3496, 16384, b.n):
        call = lambda: lib.enet_hip_crc32_batch_host(ctx.handle, hp.ptr, b.payload.nbytes, ho.ptr, hl.ptr,  # noqa: E731
                                                     k, out.ptr)
        assert call() == 0
        assert (out.arr[:k] == exp[:k]).all(), f"cfg2 slice {k} differs from the oracle"
        dt = timed(call, reps if k < 16384 else max(3, reps // 4))
        rows.append({"case": "cfg2 slice, enet_hip_crc32_batch_host, pinned", "packets": k, "span_bytes": 1200 * k,
                     "us_per_call": round(dt * 1e6, 1), "GBps": round(1200 * k / dt / 1e9, 2)})
    for x in (hp, ho, hl, out):
        x.free()
    return rows


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    ctx = enethip.Context(0)
    if os.environ.get("PCIE_BENCH_SLICES"):
        for r in case_cfg2_slices(ctx, reps) + case_cfg5_slices(ctx, reps):
            print(json.dumps(r), flush=True)
        ctx.close()
        return
    for case in (case_pcie, case_cfg2, case_cfg5):
        print(json.dumps(case(ctx, reps)), flush=True)
    ctx.close()
    print(json.dumps(case_cfg2_multi(reps)), flush=True)


if __name__ == "__main__":
    main()
