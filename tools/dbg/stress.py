"""Debug: repeat vring launches and count wrong CRCs (intermittent-race hunt).
usage: stress.py REPS"""
import os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "enet-csharp_amd"), os.path.join(ROOT, "oracle")]
import enethip, oracle
from enethip import workloads
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ol = oracle.OracleLib()
sets = {}
for name, b in (("tiny", workloads.mixed(1_200_000, 0, 40, seed=177, len_seed=178)),
                ("mtu", workloads.mixed(100_000, 1200, 1200, seed=181, len_seed=182)),
                ("big", workloads.mixed(40_000, 2000, 9000, seed=179, len_seed=180))):
    sets[name] = (b, ol.batch(b.payload, b.off, b.lens, threads=16),
                  torch.from_numpy(b.payload).cuda(), torch.from_numpy(b.off.view(np.int64)).cuda(),
                  torch.from_numpy(b.lens.view(np.int32)).cuda())
t0 = time.time()
for diag, path in ((False, 0), (True, 19), (True, 21)):
    ctx = enethip.Context(0, diag=diag)
    ctx.set_kernel_path(path)
    for lanes in (4, 8):
        for wgs in (1, 2):
            ctx.set_tuning(lanes, wgs)
            for name, (b, exp, d_p, d_o, d_l) in sets.items():
                nbad, runs_bad = 0, 0
                for r in range(reps):
                    out = torch.full((b.n,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")   # never-written sentinel
                    ctx.crc32_batch_device(d_p, d_o, d_l, b.n, out, torch.cuda.current_stream().cuda_stream)
                    torch.cuda.synchronize()
                    got = out.cpu().numpy().view(np.uint32)
                    bad = np.nonzero(got != exp)[0]
                    if len(bad):
                        runs_bad += 1
                        nbad += len(bad)
                        kpk = 64 // lanes
                        print(f"  BAD path {path} lanes {lanes} wgs {wgs} {name} rep {r}: {len(bad)} packets, "
                              f"idx {bad[:6].tolist()} groups {sorted(set((bad // kpk).tolist()))[:8]} "
                              f"unwritten {(got[bad] == 0x5A5A5A5A).sum()} 0xFFFFFFFF {(got[bad] == 0xFFFFFFFF).sum()}", flush=True)
                print(f"path {path} lanes {lanes} wgs {wgs} {name}: {runs_bad}/{reps} bad runs ({time.time()-t0:.0f}s)",
                      flush=True)
    ctx.close()
