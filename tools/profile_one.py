#!/usr/bin/env python3
"""Run one checksum configuration N times (for rocprofv3 passes): resident cfg
batches, launches through the C-ABI, nothing else on the GPU.

    rocprofv3 --kernel-trace --stats -d gpurun_out/p -o run -- python3 tools/profile_one.py --lanes 4
    rocprofv3 --pmc FETCH_SIZE -d ... -- python3 tools/profile_one.py --lanes 4
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "enet-csharp_amd"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--path", type=int, default=0)
    ap.add_argument("--ablate", type=int, default=0)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rotate", type=int, default=5)
    ap.add_argument("--probe", action="store_true", help="also run the read probe")
    ap.add_argument("--list", type=int, default=0, help="batches per launch (batch-list entry)")
    ap.add_argument("--wgs", type=int, default=0)
    ap.add_argument("--binned", action="store_true", help="length-binned entry (one batch per launch)")
    a = ap.parse_args()
    batches = bench.make_batches(a.config, a.rotate, 0)
    diag = a.ablate != 0 or a.path not in bench.PRODUCT_PATHS or a.lanes not in bench.PRODUCT_LANES   # sweeps: diag
    eng = bench.GpuEngine(0, batches, a.lanes, a.wgs, diag=diag)
    if a.binned:
        eng.set_binned(True)
    elif a.list:
        eng.set_list(a.list)
    eng.ctx.set_kernel_path(a.path)
    if diag:
        eng.ctx.diag_ablation(a.ablate)
    for first, count in eng.launch_plan(a.reps):          # --reps batches, --list per launch
        eng.launch(first, count)
    if a.probe:
        for i in range(a.reps):
            eng.probe(i)
    eng.sync()
    print("done", a)


if __name__ == "__main__":
    main()
