"""Debug: mismatches of the vring walk path at 1 / 2 workgroups per CU (tiny packets)."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "enet-csharp_amd"), os.path.join(ROOT, "oracle")]
import enethip, oracle
from enethip import workloads
tiny = workloads.mixed(1_200_000, 0, 40, seed=177, len_seed=178)
exp = oracle.OracleLib().batch(tiny.payload, tiny.off, tiny.lens, threads=16)
d_p = torch.from_numpy(tiny.payload).cuda()
d_o = torch.from_numpy(tiny.off.view(np.int64)).cuda()
d_l = torch.from_numpy(tiny.lens.view(np.int32)).cuda()
for diag, path in ((False, 0), (True, 19), (True, 20), (True, 21)):
    ctx = enethip.Context(0, diag=diag)
    ctx.set_kernel_path(path)
    for lanes in (4, 8):
        for wgs in (1, 2):
            ctx.set_tuning(lanes, wgs)
            out = torch.full((tiny.n,), -1, dtype=torch.int32, device="cuda")
            ctx.crc32_batch_device(d_p, d_o, d_l, tiny.n, out, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            bad = np.nonzero(got != exp)[0]
            kpk = 64 // lanes
            groups = (tiny.n + kpk - 1) // kpk
            print(f"path {path} lanes {lanes} wgs {wgs}: {len(bad)} bad; first {bad[:8].tolist()} groups "
                  f"{sorted(set((bad // kpk).tolist()))[:12]} of {groups}; unset {(got == 0xFFFFFFFF).sum()}", flush=True)
    ctx.close()
