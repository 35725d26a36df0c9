#!/usr/bin/env python3
"""Batch-pipeline depth experiment: K launches of the cfg batch captured in one
HIP graph, round-robin over D streams (independent batches, so consecutive
launches may overlap: one kernel's prologue runs in CUs the previous kernel's
tail has freed).  Prints ms per step and GiB/s for each D, and checks every
output batch against the oracle afterwards.

    python tools/pipeline.py [--config cfg2] [--lanes 8] [--path 0] [--depths 1,2,3] [--steps 200]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "enet-csharp_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--lanes", type=int, default=8)
    ap.add_argument("--path", type=int, default=0)
    ap.add_argument("--ablate", type=int, default=0)
    ap.add_argument("--depths", default="1,2,3")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rotate", type=int, default=6)
    a = ap.parse_args()
    import torch
    import oracle
    batches = bench.make_batches(a.config, a.rotate, 0)
    eng = bench.GpuEngine(0, batches, a.lanes, 0, diag=True)
    eng.ctx.set_kernel_path(a.path)
    eng.ctx.diag_ablation(a.ablate)
    nbytes = batches[0].payload_bytes
    exp = [oracle.OracleLib().batch(b.payload, b.off, b.lens, threads=16) for b in batches]
    for d in [int(x) for x in a.depths.split(",")]:
        streams = [torch.cuda.Stream() for _ in range(d)]
        main_s = streams[0]
        for b in eng.bufs:
            b["out"].zero_()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=main_s):
            for s in streams[1:]:
                s.wait_stream(main_s)
            for i in range(a.steps):
                b = eng.bufs[i % len(eng.bufs)]
                st = streams[i % d]
                eng.ctx.crc32_batch_device(b["payload"], b["off"], b["lens"], b["n"], b["out"], st.cuda_stream)
            for s in streams[1:]:
                main_s.wait_stream(s)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        ok = all((eng.outputs(j) == exp[j]).all() for j in range(len(batches))) if (a.ablate & 511) in (0, 8, 32, 64, 256) else None
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        dt = float(np.median(ts)) / a.steps
        print(json.dumps({"depth": d, "ms_per_step": round(dt * 1e3, 5), "GiBps": round(nbytes / dt / 2**30, 1),
                          "GBps": round(nbytes / dt / 1e9, 1), "ok": ok}), flush=True)
        del g


if __name__ == "__main__":
    main()
