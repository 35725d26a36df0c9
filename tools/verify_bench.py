#!/usr/bin/env python3
"""Receive-verify throughput (enet_hip_verify_batch_device, c/protocol.cs:1012-1014,
1052-1068) on cfg2-shaped DGRAMs: 65 536 x 1200 B packed, the
4-byte checksum slot at offset 4 stamped with the true CRC (computed with the slot
= connectID 0x1234ABCD, as the sender's protocol.cs:1690-1698 does), every 64th
DGRAM corrupted.  5 rotating resident batches (> the 256 MiB Infinity Cache).
Algorithmic bytes per batch = the DGRAM bytes (1 byte read per byte; ok[] and
computed[] writes are 5 B per DGRAM, not counted).  Timing as bench.py's roofline
region: HIP events on the launch stream around back-to-back calls, a spin kernel
ahead.  The checksum entry (enet_hip_crc32_batch_device) on the same batches is
timed beside it.  ok[] and computed[] are checked against the oracle on batch 0.

    python tools/verify_bench.py [--reps 100] [--lanes 0] [--list 5]

verify_noslot times the same call with every slot offset past its DGRAM (no slot work).
--list L also times enet_hip_verify_batch_list_device over L consecutive rotating
batches per call (per-batch time = call time / L), each batch's ok[] / computed[]
in its own slice, checked against batch 0's single call.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "enet-csharp_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

N, L, SLOT, CONNECT = 65536, 1200, 4, 0x1234ABCD


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--rotate", type=int, default=5)
    ap.add_argument("--list", type=int, default=5)
    ap.add_argument("--wgs", type=int, default=0, help="workgroups per CU (enet_hip_set_tuning; 0 = default)")
    ap.add_argument("--path", type=int, default=0, help="kernel path (13 = the lean kernel; 0 = vring at 8 lanes)")
    a = ap.parse_args()
    import torch
    import enethip
    from enethip import workloads
    import oracle as orc
    ctx = enethip.Context(0, a.lanes, a.wgs, diag=a.lanes not in (0, 4, 8) or a.path not in (0, 13, 17))
    ctx.set_kernel_path(a.path)
    st = torch.cuda.Stream()
    off = np.arange(N, dtype=np.uint64) * L
    lens = np.full(N, L, np.uint32)
    slot = np.full(N, SLOT, np.uint32)
    conn = np.full(N, CONNECT, np.uint32)
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    d_len = torch.from_numpy(lens.view(np.int32)).cuda()
    d_slot = torch.from_numpy(slot.view(np.int32)).cuda()
    d_conn = torch.from_numpy(conn.view(np.int32)).cuda()
    batches = []
    for r in range(a.rotate):
        p = workloads.payload_bytes(N * L, seed=0x56455249 + r).reshape(N, L).copy()
        p[:, SLOT:SLOT + 4] = np.frombuffer(np.uint32(CONNECT).tobytes(), np.uint8)
        d = torch.from_numpy(p.reshape(-1)).cuda()
        crc = torch.zeros(N, dtype=torch.int32, device="cuda")
        ctx.crc32_batch_device(d, d_off, d_len, N, crc, st.cuda_stream)
        torch.cuda.synchronize()
        dv = d.view(N, L)
        dv[:, SLOT:SLOT + 4] = crc.view(torch.uint8).view(N, 4)       # the stamp, in wire order
        dv[::64, 100] ^= 1                                            # corrupt every 64th DGRAM
        batches.append(d)
    ok = torch.zeros(N, dtype=torch.uint8, device="cuda")
    comp = torch.zeros(N, dtype=torch.int32, device="cuda")
    crc = torch.zeros(N, dtype=torch.int32, device="cuda")

    def verify(i):
        ctx.verify_batch_device(batches[i % a.rotate], d_off, d_len, d_slot, d_conn, N, ok, comp, st.cuda_stream)

    lok = torch.zeros(max(1, a.list) * N, dtype=torch.uint8, device="cuda")
    lcomp = torch.zeros(max(1, a.list) * N, dtype=torch.int32, device="cuda")

    def vlist(i):
        ctx.verify_batch_list_device([(batches[(i * a.list + t) % a.rotate], d_off, d_len, d_slot, d_conn, N,
                                       lok[t * N:(t + 1) * N], lcomp[t * N:(t + 1) * N]) for t in range(a.list)],
                                     st.cuda_stream)

    # the same call with every slot offset past its DGRAM: no slot to substitute or collect
    # (ok = 0 everywhere) -- what the slot handling costs
    d_noslot = torch.full((N,), 0x7FFFFF00, dtype=torch.int32, device="cuda")

    def verify_noslot(i):
        ctx.verify_batch_device(batches[i % a.rotate], d_off, d_len, d_noslot, d_conn, N, ok, comp, st.cuda_stream)

    def checksum(i):
        ctx.crc32_batch_device(batches[i % a.rotate], d_off, d_len, N, crc, st.cuda_stream)

    # correctness on batch 0 against the oracle
    verify(0)
    torch.cuda.synchronize()
    lib = orc.OracleLib()
    exp_ok, exp_comp = lib.verify(batches[0].cpu().numpy(), off, lens, slot, conn)
    got_ok, got_comp = ok.cpu().numpy(), comp.cpu().numpy().view(np.uint32)
    exact = bool((got_ok == exp_ok).all() and (got_comp == exp_comp).all())
    assert exact, "verify differs from the oracle"
    assert int(exp_ok.sum()) == N - N // 64
    if a.list:
        vlist(0)
        torch.cuda.synchronize()
        for t in range(a.list):
            if (t % a.rotate) == 0:
                assert (lok[t * N:(t + 1) * N] == ok).all() and (lcomp[t * N:(t + 1) * N] == comp).all(), t

    def region_us(fn):
        for i in range(5):
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
        return e0.elapsed_time(e1) / a.reps * 1e3

    res = {"kind": "verify-bench", "path": a.path, "list": a.list, "dgrams": N, "bytes_per_batch": N * L, "lanes": a.lanes or "default",
           "bit_exact_vs_oracle": exact, "ok_count": int(exp_ok.sum())}
    fns = [("verify", verify, 1), ("verify_noslot", verify_noslot, 1), ("checksum", checksum, 1)] + \
        ([("verify_list", vlist, a.list)] if a.list else [])
    for name, fn, per in fns:
        us = region_us(fn) / per
        res[name + "_us"] = round(us, 2)
        res[name + "_GBps"] = round(N * L / us / 1e3, 1)
        res[name + "_GiBps"] = round(N * L / us * 1e6 / 2 ** 30, 1)
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
