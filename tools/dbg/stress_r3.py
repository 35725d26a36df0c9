"""Debug: repeat the round-3 kernel paths and count wrong results (intermittent-race hunt):
the records instance (LDS index stash, end-aligned windows, small tz tables) through the
binned checksum entry and the binned gather, and receive verify lists (VF, in-place edge
mask), each output buffer pre-filled with a never-written sentinel.
usage: stress_r3.py REPS"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "enet-csharp_amd"), os.path.join(ROOT, "oracle")]
import enethip  # noqa: E402
import oracle  # noqa: E402
from enethip import workloads  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ol = oracle.OracleLib()
ctx = enethip.Context(0)
st = torch.cuda.current_stream().cuda_stream
SENT = 0x5A5A5A5A


def dev(a, dt):
    return torch.from_numpy(np.ascontiguousarray(a).view(dt)).cuda()


fails = 0
t0 = time.time()

# binned checksum batches: cfg3 lengths, and 16-byte-aligned ends (every window end-aligned)
b3 = workloads.cfg3()
rng = np.random.default_rng(5)
n16 = 200_000
len16 = (rng.integers(1, 90, size=n16) * 16).astype(np.uint32)
off16 = np.zeros(n16, np.uint64)
off16[1:] = np.cumsum(len16[:-1].astype(np.uint64))
pay16 = rng.integers(0, 256, size=int(len16.sum()) + 64, dtype=np.uint8)
for name, (p, o, ln) in (("cfg3", (b3.payload, b3.off, b3.lens)), ("ends16", (pay16, off16, len16))):
    exp = ol.batch(p, o, ln, threads=16)
    n = len(o)
    d_p, d_o, d_l = dev(p, np.uint8), dev(o, np.int64), dev(ln, np.int32)
    wsb = ctx.binned_workspace_size(n)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    for lanes in (4, 8):
        ctx.set_tuning(lanes, 0)
        bad_runs = 0
        for r in range(reps):
            out = torch.full((n,), SENT, dtype=torch.int32, device="cuda")
            ctx.crc32_batch_device_binned(d_p, d_o, d_l, n, out, ws, wsb, stream=st)
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            bad = np.nonzero(got != exp)[0]
            if len(bad):
                bad_runs += 1
                print(f"  BAD binned {name} lanes {lanes} rep {r}: {len(bad)} packets, unwritten "
                      f"{int((got[bad] == SENT).sum())}", flush=True)
        fails += bad_runs
        print(f"binned {name} lanes {lanes}: {reps - bad_runs}/{reps} runs exact", flush=True)
ctx.set_tuning(0, 0)

# binned gather, cfg5 (1024 messages)
g = workloads.cfg5(1024)
expg = ol.gather(g.payload, g.seg_off, g.seg_len, g.seg_first)
ns = int(g.seg_first[-1])
wsb = ctx.gather_binned_workspace_size(ns)
ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
d_p, d_so, d_sl, d_sf = dev(g.payload, np.uint8), dev(g.seg_off, np.int64), dev(g.seg_len, np.int32), \
    dev(g.seg_first, np.int32)
bad_runs = 0
for r in range(reps):
    out = torch.full((g.n,), SENT, dtype=torch.int32, device="cuda")
    ctx.gather_binned_device(d_p, d_so, d_sl, ns, d_sf, g.n, out, ws, wsb, stream=st)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != expg)[0]
    if len(bad):
        bad_runs += 1
        print(f"  BAD gather rep {r}: {len(bad)} DGRAMs", flush=True)
fails += bad_runs
print(f"gather cfg5/1024: {reps - bad_runs}/{reps} runs exact", flush=True)

# receive verify: one batch of MTU-shaped DGRAMs, stamped, some corrupted
n = 65536
lens = np.full(n, 1200, np.uint32)
off = (np.arange(n, dtype=np.uint64) * np.uint64(1200))
slot = np.full(n, 4, np.uint32)
conn = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
pay = rng.integers(0, 256, size=n * 1200, dtype=np.uint8)
for i in range(0, n, 1):
    pay[1200 * i + 4:1200 * i + 8] = np.frombuffer(np.uint32(conn[i]).tobytes(), np.uint8)
stamped = ol.batch(pay, off, lens, threads=16)
v = pay.reshape(n, 1200)
v[:, 4:8] = stamped.view(np.uint8).reshape(n, 4)
v[::97, 600] ^= 1                                        # corrupt some DGRAMs
exp_ok, exp_comp = ol.verify(pay, off, lens, slot, conn)
d = [dev(pay, np.uint8), dev(off, np.int64), dev(lens, np.int32), dev(slot, np.int32), dev(conn, np.int32)]
bad_runs = 0
for r in range(reps):
    ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    comp = torch.full((n,), SENT, dtype=torch.int32, device="cuda")
    ctx.verify_batch_device(*d, n, ok, comp, stream=st)
    torch.cuda.synchronize()
    g_ok, g_comp = ok.cpu().numpy(), comp.cpu().numpy().view(np.uint32)
    if not ((g_ok == exp_ok).all() and (g_comp == exp_comp).all()):
        bad_runs += 1
        print(f"  BAD verify rep {r}: ok {int((g_ok != exp_ok).sum())} computed {int((g_comp != exp_comp).sum())}",
              flush=True)
fails += bad_runs
print(f"verify MTU: {reps - bad_runs}/{reps} runs exact", flush=True)
print(f"stress_r3: {fails} bad runs, {time.time() - t0:.1f} s", flush=True)
ctx.close()
sys.exit(1 if fails else 0)
