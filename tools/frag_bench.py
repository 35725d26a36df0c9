#!/usr/bin/env python3
"""Fragment reassembly throughput (enet_hip_fragment_reassemble_device,
c/protocol.cs:529-637) on cfg5's receive side: 4096 x 64 KiB messages = 200 704
SEND_FRAGMENT DGRAMs in shuffled order, device-resident.  Algorithmic bytes per
call = 2 x fragment data (read from the DGRAM arena, written to the messages).
The bitmaps / remaining counters are reset between calls (untimed); HIP events
bracket each call on its stream.  Result checked against the original messages.

    python tools/frag_bench.py [--messages 4096] [--reps 20]
    python tools/frag_bench.py --messages 1024 --words 2 --first 1   (one fragment
        against a 65 536-word claim space -- the slots path; --messages 1025: the atomic path)
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
    ap.add_argument("--messages", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--in-order", action="store_true",
                    help="fragments in send order instead of shuffled (prices the scattered descriptor stores)")
    ap.add_argument("--words", type=int, default=2, help="bitmap words per message slot")
    ap.add_argument("--copy-ref", action="store_true",
                    help="also time a plain device-to-device copy of the same data bytes (torch copy_)")
    ap.add_argument("--first", type=int, default=0,
                    help="pass only the first N fragments (tiny batch against the whole slot table)")
    a = ap.parse_args()
    import torch
    import enethip
    from enethip import workloads
    fb = (workloads.fragments([65536] * a.messages, shuffle=False, name=f"cfg5 receive, in order: {a.messages} x 65536 B")
          if a.in_order else workloads.cfg5_fragments(a.messages))
    words = a.words
    nf = a.first if a.first else fb.n
    ctx = enethip.Context(0)
    t = lambda x, dt: torch.from_numpy(np.ascontiguousarray(x).view(dt)).cuda()  # noqa: E731
    d_payload = t(fb.payload, np.uint8)
    d_off, d_avail, d_slots = t(fb.cmd_off, np.int64), t(fb.cmd_avail, np.int32), t(fb.slots, np.int32)
    msg_off = np.concatenate([[0], np.cumsum(fb.msg_len.astype(np.uint64))[:-1]]).astype(np.uint64)
    d_msg = torch.zeros(int(fb.msg_len.astype(np.uint64).sum()), dtype=torch.uint8, device="cuda")
    d_moff, d_mlen, d_mcnt = t(msg_off, np.int64), t(fb.msg_len, np.int32), t(fb.msg_count, np.int32)
    d_frag = torch.zeros(len(fb.msg_len) * words, dtype=torch.int32, device="cuda")
    d_rem0 = t(fb.msg_count, np.int32)
    d_rem = d_rem0.clone()
    d_status = torch.zeros(fb.n, dtype=torch.int8, device="cuda")
    s = torch.cuda.Stream()
    times = []
    for r in range(a.reps + 2):
        d_frag.zero_()
        d_rem.copy_(d_rem0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            e0.record(s)
            ctx.fragment_reassemble_device(d_payload, d_off, d_avail, d_slots, nf, 32 << 20, d_msg, d_moff, d_mlen,
                                           d_mcnt, d_frag, words, d_rem, len(fb.msg_len), d_status,
                                           stream=s.cuda_stream)
            e1.record(s)
        torch.cuda.synchronize()
        if r >= 2:
            times.append(e0.elapsed_time(e1) * 1e-3)
    if a.first:                                   # a partial batch: every fragment new, nothing else
        ok = bool((d_status.cpu().numpy()[:nf] == 1).all())
    else:
        ok = bool((d_status.cpu().numpy() == 1).all() and (d_rem.cpu().numpy() == 0).all() and
                  (d_msg.cpu().numpy() == np.concatenate(fb.messages)).all())
    dt = float(np.median(times))
    moved = 2.0 * (float(fb.cmd_avail[:nf].astype(np.uint64).sum()) if a.first else fb.data_bytes)
    claims = len(fb.msg_len) * words * 32
    print(json.dumps({"workload": fb.name, "fragments": nf, "claim_space": claims,
                      "slots_path": claims <= 8 * nf + 65536, "data_bytes": fb.data_bytes,
                      "us_per_call": round(dt * 1e6, 2), "GBps_moved": round(moved / dt / 1e9, 1),
                      "hbm_frac": round(moved / dt / 8e12, 4), "ok": ok}), flush=True)
    if a.copy_ref:                                # the chip's rate for a plain copy of the same bytes
        src = torch.empty_like(d_msg).random_(0, 255)
        rt = []
        for r in range(a.reps + 2):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                e0.record(s)
                d_msg.copy_(src)
                e1.record(s)
            torch.cuda.synchronize()
            if r >= 2:
                rt.append(e0.elapsed_time(e1) * 1e-3)
        rd = float(np.median(rt))
        print(json.dumps({"plain_copy_bytes": int(d_msg.numel()), "us": round(rd * 1e6, 2),
                          "GBps_moved": round(2.0 * d_msg.numel() / rd / 1e9, 1)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
