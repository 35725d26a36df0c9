#!/usr/bin/env python3
"""Sustained streaming rate of a kernel against time, with the GPU's clocks and
power sampled beside it (VERDICT r2 "settle the sustained-rate gap with evidence").

    python tools/sustain.py --kernel vring|probe [--launches N] [--list L]

vring: N back-to-back enet_hip_crc32_batch_list_device launches of L resident
cfg2-shaped batches (1200-B packets), the bench's default entry; probe: N launches
of the read probe (enet_hip_read_probe_device: 16-B coalesced loads, every byte
once, no compute) over the same L x 75 MiB of bytes.  Every launch is bracketed by
HIP events on one stream (a spin kernel heads the queue, so the host never starves
it).  A thread samples amdsmi's GPU metrics (current gfx / memory clocks, socket
power, PPT and thermal residency counters, throttle status) as fast as the library
answers.  Output: one JSON line per time bucket (1 ms buckets over the first 40 ms,
then 20 ms) with the streaming rate and the metric samples that fall in it, then a
summary line.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "enet-csharp_amd"))
import enethip  # noqa: E402

BATCH = 65536 * 1200


class Sampler(threading.Thread):
    """amdsmi GPU metrics, sampled in a loop; t = perf_counter seconds."""

    FIELDS = ("current_gfxclk", "current_uclk", "current_socket_power", "average_socket_power",
              "ppt_residency_acc", "socket_thm_residency_acc", "hbm_thm_residency_acc", "throttle_status",
              "average_gfx_activity", "average_umc_activity", "firmware_timestamp")

    def __init__(self):
        super().__init__(daemon=True)
        self.samples, self.stop, self.error = [], False, None
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            self.amdsmi = amdsmi
            self.h = amdsmi.amdsmi_get_processor_handles()[0]
        except Exception as e:  # noqa: BLE001 -- report, keep timing
            self.amdsmi, self.error = None, repr(e)

    def run(self):
        if self.amdsmi is None:
            return
        while not self.stop:
            try:
                m = self.amdsmi.amdsmi_get_gpu_metrics_info(self.h)
            except Exception as e:  # noqa: BLE001
                self.error = repr(e)
                return
            self.samples.append((time.perf_counter(), {k: m.get(k) for k in self.FIELDS}))


def refresh_ms(samples, t0, t1):
    """Median host-time gap between samples whose firmware timestamp changed."""
    ts, last = [], object()
    for t, m in samples:
        if t0 <= t <= t1 and m.get("firmware_timestamp") != last:
            ts.append(t)
            last = m.get("firmware_timestamp")
    return round(float(np.median(np.diff(ts)) * 1e3), 3) if len(ts) > 2 else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", choices=["vring", "probe"], default="vring")
    ap.add_argument("--launches", type=int, default=3000)
    ap.add_argument("--list", type=int, default=5)
    ap.add_argument("--ablate", type=int, default=0,
                    help="vring: enet_hip_diag_ablation value (diagnostics library; 4096 = no table lookups, "
                         "2048+4096+32768 = the memory/control skeleton: WRONG CRCs by design)")
    a = ap.parse_args()
    nb = 10
    big = torch.randint(0, 255, (nb * BATCH + 4096,), dtype=torch.uint8, device="cuda")
    off = torch.arange(65536, dtype=torch.int64, device="cuda") * 1200
    lens = torch.full((65536,), 1200, dtype=torch.int32, device="cuda")
    outs = [torch.zeros(65536, dtype=torch.int32, device="cuda") for _ in range(nb)]
    descs = [(big[j * BATCH:], off, lens, 65536, outs[j]) for j in range(nb)]
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    ctx = enethip.Context(0, diag=bool(a.ablate))
    if a.ablate:
        ctx.diag_ablation(a.ablate)
    st = torch.cuda.Stream()
    L = a.list

    def launch(i):
        if a.kernel == "vring":
            ctx.crc32_batch_list_device([descs[(i * L + t) % nb] for t in range(L)], st.cuda_stream)
        else:
            j = (i * L) % (nb - L + 1)
            ctx.read_probe_device(big[j * BATCH:], L * BATCH, sink, st.cuda_stream)

    for i in range(5):
        launch(i)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.launches + 1)]
    smp = Sampler()
    smp.start()
    time.sleep(0.05)
    with torch.cuda.stream(st):
        torch.cuda._sleep(int(2e9))                    # ~1 s of spin: every launch is queued before it ends
        ev[0].record(st)
        for i in range(a.launches):
            launch(i)
            ev[i + 1].record(st)
    ev[0].synchronize()
    t_gpu0 = time.perf_counter()                       # host time the GPU reached ev[0] (+ poll latency)
    torch.cuda.synchronize()
    t_end = time.perf_counter()
    time.sleep(0.05)
    smp.stop = True
    smp.join()
    ends = np.array([ev[0].elapsed_time(ev[i + 1]) for i in range(a.launches)])      # ms since ev[0]
    starts = np.concatenate([[0.0], ends[:-1]])
    nbytes = L * BATCH
    edges = list(np.arange(0, 40, 1.0)) + list(np.arange(40, ends[-1] + 20, 20.0))
    early = []                                          # 1-ms bucket rates over the first 40 ms
    for lo, hi in zip(edges[:-1], edges[1:]):
        sel = (starts >= lo) & (starts < hi)
        if not sel.any():
            continue
        dur = (ends[sel] - starts[sel]).sum()
        ss = [m for t, m in smp.samples if lo <= (t - t_gpu0) * 1e3 < hi]
        row = {"t_ms": [round(lo, 1), round(hi, 1)], "launches": int(sel.sum()),
               "TBps": round(nbytes * int(sel.sum()) / (dur * 1e-3) / 1e12, 3), "smi_samples": len(ss)}
        if hi <= 40:
            early.append(row["TBps"])
        for k in ("current_gfxclk", "current_uclk", "current_socket_power"):
            v = [m[k] for m in ss if isinstance(m.get(k), (int, float))]
            if v:
                row[k] = round(float(np.mean(v)), 1)
        print(json.dumps(row))
    idle = [m for t, m in smp.samples if t < t_gpu0 - 0.9]                 # during the spin / before
    run = [m for t, m in smp.samples if t_gpu0 <= t <= t_end]
    first, last = (run[0], run[-1]) if run else ({}, {})

    def delta(k):
        try:
            return last[k] - first[k]
        except Exception:  # noqa: BLE001
            return None
    print(json.dumps({"summary": a.kernel, "launches": a.launches, "bytes_per_launch": nbytes,
                      "span_ms": round(float(ends[-1]), 2),
                      "TBps_first_2ms": round(nbytes * int((starts < 2).sum()) /
                                              (ends[starts < 2][-1] * 1e-3) / 1e12, 3),
                      "TBps_whole": round(nbytes * a.launches / (ends[-1] * 1e-3) / 1e12, 3),
                      "TBps_1ms_buckets_first_40ms": [min(early, default=None), max(early, default=None)],
                      "smi_samples_run": len(run), "smi_error": smp.error, "ablate": a.ablate,
                      # do the metrics refresh?  distinct firmware timestamps over the run
                      # and the median gap between them (ms of host time)
                      "smi_distinct_fw_timestamps": len({m.get("firmware_timestamp") for m in run}),
                      "smi_refresh_ms_median": refresh_ms(smp.samples, t_gpu0, t_end),
                      "ppt_residency_delta": delta("ppt_residency_acc"),
                      "socket_thm_residency_delta": delta("socket_thm_residency_acc"),
                      "hbm_thm_residency_delta": delta("hbm_thm_residency_acc"),
                      "throttle_status_seen": sorted({str(m.get("throttle_status")) for m in run}),
                      "gfxclk_run": [min((m["current_gfxclk"] for m in run if isinstance(m.get("current_gfxclk"), int)),
                                         default=None),
                                     max((m["current_gfxclk"] for m in run if isinstance(m.get("current_gfxclk"), int)),
                                         default=None)],
                      "uclk_run": [min((m["current_uclk"] for m in run if isinstance(m.get("current_uclk"), int)),
                                       default=None),
                                   max((m["current_uclk"] for m in run if isinstance(m.get("current_uclk"), int)),
                                       default=None)],
                      "power_run_W": [min((m["current_socket_power"] for m in run
                                           if isinstance(m.get("current_socket_power"), int)), default=None),
                                      max((m["current_socket_power"] for m in run
                                           if isinstance(m.get("current_socket_power"), int)), default=None)],
                      "gfxclk_idle": idle[-1].get("current_gfxclk") if idle else None,
                      "power_idle_W": idle[-1].get("current_socket_power") if idle else None}))
    ctx.close()


if __name__ == "__main__":
    main()
