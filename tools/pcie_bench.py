#!/usr/bin/env python3
"""Host-memory (PCIe-inclusive) rates of the checksum path, for DESIGN.md.

  * cfg2 through enet_hip_crc32_batch_host with PINNED host buffers
    (enet_hip_host_alloc): H2D of the packet bytes + offsets + lengths, the
    stream kernel, D2H of the CRCs; synchronous per batch.
  * cfg5 (fragmented sends, 3-buffer gather lists): pinned arenas, H2D of the
    segment bytes and tables, crc32_gather_device, D2H of the CRCs.
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


class Device:
    def __init__(self, ctx, nbytes: int):
        self.ctx = ctx
        p = ctypes.c_void_p()
        rc = ctx.lib.enet_hip_device_alloc(ctx.handle, max(16, nbytes), ctypes.byref(p))
        if rc:
            raise RuntimeError(f"device_alloc {rc}")
        self.ptr = p.value

    def free(self):
        self.ctx.lib.enet_hip_device_free(self.ctx.handle, self.ptr)


def case_cfg2(ctx, reps: int):
    lib = ctx.lib
    b = workloads.cfg2()
    hp, ho, hl = Pinned(lib, b.payload), Pinned(lib, b.off), Pinned(lib, b.lens)
    out = Pinned(lib, np.zeros(b.n, np.uint32))
    call = lambda: lib.enet_hip_crc32_batch_host(ctx.handle, hp.ptr, b.payload.nbytes, ho.ptr, hl.ptr,  # noqa: E731
                                                 b.n, out.ptr)
    for _ in range(3):
        assert call() == 0
    exp = oracle.OracleLib().batch(b.payload, b.off, b.lens, threads=8)
    assert (out.arr == exp).all(), "cfg2 host path differs from the oracle"
    t0 = time.perf_counter()
    for _ in range(reps):
        call()
    dt = (time.perf_counter() - t0) / reps
    for x in (hp, ho, hl, out):
        x.free()
    return {"case": "cfg2 host path (pinned H2D + kernel + D2H, synchronous)", "payload_bytes": b.payload_bytes,
            "ms_per_batch": round(dt * 1e3, 4), "GiBps": round(b.payload_bytes / dt / GIB, 2),
            "GBps": round(b.payload_bytes / dt / 1e9, 2)}


def case_cfg5(ctx, reps: int):
    lib = ctx.lib
    g = workloads.cfg5()
    hp = Pinned(lib, g.payload)
    ho, hl, hf = Pinned(lib, g.seg_off), Pinned(lib, g.seg_len), Pinned(lib, g.seg_first)
    out = Pinned(lib, np.zeros(g.n, np.uint32))
    dp, do_, dl, df, dout = (Device(ctx, x.nbytes) for x in (hp, ho, hl, hf, out))

    def h2d(d, h):
        assert lib.enet_hip_memcpy_h2d(ctx.handle, d.ptr, h.ptr, h.nbytes) == 0

    def once(copy_in=True):
        if copy_in:
            for d, h in ((dp, hp), (do_, ho), (dl, hl), (df, hf)):
                h2d(d, h)
        assert lib.enet_hip_crc32_gather_device(ctx.handle, dp.ptr, do_.ptr, dl.ptr, df.ptr, g.n, dout.ptr,
                                                None) == 0
        assert lib.enet_hip_memcpy_d2h(ctx.handle, out.ptr, dout.ptr, out.nbytes) == 0

    for _ in range(2):
        once()
    exp = oracle.OracleLib().gather(g.payload, g.seg_off, g.seg_len, g.seg_first)
    assert (out.arr == exp).all(), "cfg5 gather differs from the oracle"
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    dt = (time.perf_counter() - t0) / reps
    # kernel-only (tables and bytes resident), for comparison
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        assert lib.enet_hip_crc32_gather_device(ctx.handle, dp.ptr, do_.ptr, dl.ptr, df.ptr, g.n, dout.ptr,
                                                None) == 0
    ctx.synchronize()
    dk = (time.perf_counter() - t0) / reps
    for x in (hp, ho, hl, hf, out, dp, do_, dl, df, dout):
        x.free()
    return {"case": "cfg5 gather (pinned H2D of segment arena + tables, gather kernel, D2H)",
            "dgram_bytes": g.dgram_bytes, "arena_bytes": int(g.payload.nbytes), "dgrams": g.n,
            "ms_per_batch": round(dt * 1e3, 4), "GiBps": round(g.dgram_bytes / dt / GIB, 2),
            "GBps": round(g.dgram_bytes / dt / 1e9, 2),
            "kernel_only_ms": round(dk * 1e3, 4), "kernel_only_GiBps": round(g.dgram_bytes / dk / GIB, 2)}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    ctx = enethip.Context(0)
    for case in (case_cfg2, case_cfg5):
        print(json.dumps(case(ctx, reps)), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
