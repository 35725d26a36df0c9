"""Debug: catch an intermittent bad run of the vring kernel at 2 workgroups per CU
(tiny packets) with the trace instance on, and dump which workgroups / waves the
missing groups belong to, with their per-wave trace records."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "enet-csharp_amd"), os.path.join(ROOT, "oracle")]
import enethip, oracle
from enethip import workloads
lanes = int(sys.argv[1]) if len(sys.argv) > 1 else 8
path = int(sys.argv[2]) if len(sys.argv) > 2 else 0
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 60
tiny = workloads.mixed(1_200_000, 0, 40, seed=177, len_seed=178)
exp = oracle.OracleLib().batch(tiny.payload, tiny.off, tiny.lens, threads=16)
d_p = torch.from_numpy(tiny.payload).cuda()
d_o = torch.from_numpy(tiny.off.view(np.int64)).cuda()
d_l = torch.from_numpy(tiny.lens.view(np.int32)).cuda()
ctx = enethip.Context(0, diag=True)
ctx.set_kernel_path(path)
ctx.set_tuning(lanes, 2)
cus = torch.cuda.get_device_properties(0).multi_processor_count
tr = torch.zeros(2 * cus * 16 * 8, dtype=torch.int64, device="cuda")
ctx.diag_trace(tr)
kpk = 64 // lanes
groups = (tiny.n + kpk - 1) // kpk
grid = min((groups + 15) // 16, 2 * cus)
wt = grid * 16
print(f"lanes {lanes} path {path} groups {groups} grid {grid} cus {cus}", flush=True)
nbad = 0
for r in range(reps):
    tr.zero_()
    out = torch.full((tiny.n,), -1, dtype=torch.int32, device="cuda")
    ctx.crc32_batch_device(d_p, d_o, d_l, tiny.n, out, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != exp)[0]
    t = tr.cpu().numpy().view(np.uint64).reshape(-1, 8)[:wt]
    gpw = t[:, 7].astype(np.int64).reshape(grid, 16).sum(1)      # groups per workgroup
    if len(bad) == 0:
        if r == 0:
            print(f"rep {r} ok; groups/WG min {gpw.min()} max {gpw.max()} total {gpw.sum()}", flush=True)
        continue
    nbad += 1
    bg = np.unique(bad // kpk)
    wg_of = (bg % wt) // 16 if path != 19 else bg // ((groups + grid - 1) // grid)
    wgs, cnt = np.unique(wg_of, return_counts=True)
    print(f"BAD rep {r}: {len(bad)} packets, {len(bg)} groups, unset {(got[bad] == 0xFFFFFFFF).sum()}; "
          f"total groups traced {gpw.sum()} of {groups}", flush=True)
    print("  workgroups with missing groups:", list(zip(wgs.tolist()[:20], cnt.tolist()[:20])), flush=True)
    lo = np.argsort(gpw)[:12]
    print("  fewest groups per WG:", [(int(w), int(gpw[w])) for w in lo], flush=True)
    for w in wgs[:3]:
        rec = t[16 * w:16 * w + 16]
        hw = rec[:, 6]
        print(f"  WG {w}: groups per wave {rec[:, 7].astype(int).tolist()}", flush=True)
        print(f"    start-min {int(rec[:, 0].min())} end-max {int(rec[:, 5].max())} "
              f"HW_ID {[hex(int(x) & 0xffffffff) for x in hw[:4]]} XCC {sorted(set((hw >> 32).astype(int).tolist()))}",
              flush=True)
        print(f"    t(start,meta,table,B,loop,end) wave0 {[int(x - rec[0, 0]) for x in rec[0, :6]]}", flush=True)
    # co-resident partner: the other WG on the same CU (HW_ID bits: CU_ID [11:8], SH_ID [12], SE_ID [15:13])
    if nbad >= 3:
        break
print(f"{nbad} bad of {r + 1} runs", flush=True)
ctx.diag_trace(None)
