#!/usr/bin/env python3
"""Tuning sweep on one GPU: per-launch kernel time (HIP events, queued behind a
spin kernel) and graph-replay throughput for each (lanes_per_packet, wgs_per_cu),
plus the read-roofline probe.  Prints one JSON line per point.

    python tools/sweep.py [--config cfg2] [--lanes 1,2,4,8] [--wgs 1,2] [--steps 50]
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
    ap.add_argument("--lanes", default="1,2,4,8")
    ap.add_argument("--wgs", default="1,2")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--rotate", type=int, default=5)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--paths", default="0,1", help="0 = LDS-staged, 1 = direct")
    ap.add_argument("--ablate", default="0", help="staged-kernel ablations to run: 0,1,2")
    a = ap.parse_args()
    batches = bench.make_batches(a.config, a.rotate, 0)
    eng = bench.GpuEngine(0, batches, 0, 0, diag=True)
    nbytes = batches[0].payload_bytes
    exp = None
    if a.check:
        import oracle
        exp = oracle.OracleLib().batch(batches[0].payload, batches[0].off, batches[0].lens, threads=16)
    p_ms, p_span = eng.kernel_ms(eng.probe, a.steps)
    probe_bytes = (batches[0].payload.nbytes // 16) * 16
    print(json.dumps({"probe_ms": p_ms, "probe_GBps": probe_bytes / p_ms / 1e6, "probe_span_ms": p_span}),
          flush=True)
    for path, abl in [(int(x), int(y)) for x in a.paths.split(",") for y in a.ablate.split(",")]:
      if path == 1 and abl != 0:
          continue
      eng.ctx.set_kernel_path(path)
      eng.ctx.diag_ablation(abl)
      for w in ([0] if path == 0 else [int(x) for x in a.wgs.split(",")]):
        for lanes in [int(x) for x in a.lanes.split(",")]:
            eng.ctx.set_tuning(lanes, w)
            ok = None
            if exp is not None:
                eng.step(0)
                eng.sync()
                ok = bool((eng.outputs(0) == exp).all()) if abl == 0 else None
            k_ms, span = eng.kernel_ms(eng.step, a.steps)
            eng.capture(a.steps)
            eng.replay()
            eng.sync()
            t0 = time.perf_counter()
            eng.replay()
            eng.sync()
            dt = (time.perf_counter() - t0) / a.steps
            print(json.dumps({"path": path, "ablate": abl, "lanes": lanes, "wgs": w, "kernel_ms": round(k_ms, 5),
                              "kernel_GBps": round(nbytes / k_ms / 1e6, 1),
                              "event_span_ms": round(span, 5),
                              "graph_ms_per_step": round(dt * 1e3, 5),
                              "graph_GiBps": round(nbytes / dt / 2**30, 1), "ok": ok}), flush=True)


if __name__ == "__main__":
    main()
