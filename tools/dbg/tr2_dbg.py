"""Debug: the product vring code path with end records (TR = 2) at 2 workgroups per
CU on tiny packets; on a bad run, dump the per-wave records of the workgroups
the missing groups belong to."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "enet-csharp_amd"), os.path.join(ROOT, "oracle")]
import enethip, oracle
from enethip import workloads
lanes = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 80
tiny = workloads.mixed(1_200_000, 0, 40, seed=177, len_seed=178)
exp = oracle.OracleLib().batch(tiny.payload, tiny.off, tiny.lens, threads=16)
d_p = torch.from_numpy(tiny.payload).cuda()
d_o = torch.from_numpy(tiny.off.view(np.int64)).cuda()
d_l = torch.from_numpy(tiny.lens.view(np.int32)).cuda()
ctx = enethip.Context(0, diag=True)
ctx.set_tuning(lanes, 2)
ctx.diag_ablation(128 << 11)
cus = torch.cuda.get_device_properties(0).multi_processor_count
tr = torch.zeros(2 * cus * 16 * 8, dtype=torch.int64, device="cuda")
ctx.diag_trace(tr)
kpk = 64 // lanes
groups = (tiny.n + kpk - 1) // kpk
grid = min((groups + 15) // 16, 2 * cus)
wt = grid * 16
print(f"lanes {lanes} groups {groups} grid {grid} cus {cus}", flush=True)
nbad = 0
r = 0
for r in range(reps):
    tr.zero_()
    out = torch.full((tiny.n,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")   # sentinel: never written
    ctx.crc32_batch_device(d_p, d_o, d_l, tiny.n, out, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != exp)[0]
    t = tr.cpu().numpy().view(np.uint64).reshape(-1, 8)[:wt]
    gpw = t[:, 7].astype(np.int64).reshape(grid, 16).sum(1)
    if len(bad) == 0:
        if r == 0:
            print(f"rep {r} ok; groups/WG {gpw.min()}..{gpw.max()} total {gpw.sum()}; taken/wave "
                  f"{t[:, 0].min()}..{t[:, 0].max()}", flush=True)
        continue
    nbad += 1
    bg = np.unique(bad // kpk)
    wg_of = (bg % wt) // 16
    wgs, cnt = np.unique(wg_of, return_counts=True)
    print(f"BAD rep {r}: {len(bad)} packets, {len(bg)} groups, unwritten {(got[bad] == 0x5A5A5A5A).sum()} "
          f"0xFFFFFFFF (reg 0) {(got[bad] == 0xFFFFFFFF).sum()}; "
          f"groups traced {gpw.sum()} of {groups}; {len(wgs)} WGs affected", flush=True)
    print("  WGs (id, missing groups):", list(zip(wgs.tolist()[:24], cnt.tolist()[:24])), flush=True)
    short = np.nonzero(gpw < 280)[0]
    print("  WGs with < 280 groups traced:", [(int(w), int(gpw[w])) for w in short[:24]], flush=True)
    ended = (t[:, 5] > 0).reshape(grid, 16).sum(1)
    print("  WGs with waves that wrote no end record:",
          [(int(w), int(16 - ended[w])) for w in np.nonzero(ended < 16)[0][:24]], flush=True)
    for w in wgs[:4]:
        rec = t[16 * w:16 * w + 16]
        print(f"  WG {w}: taken {rec[:, 0].astype(int).tolist()}", flush=True)
        print(f"         last slot {rec[:, 1].astype(int).tolist()}", flush=True)
        print(f"         groups {rec[:, 7].astype(int).tolist()}  HW_ID {hex(int(rec[0, 6]) & 0xffffffff)} "
              f"XCC {int(rec[0, 6]) >> 32}", flush=True)
    if nbad >= 3:
        break
print(f"{nbad} bad of {r + 1} runs", flush=True)
ctx.diag_trace(None)
ctx.diag_ablation(0)
