#!/usr/bin/env python3
"""Batched range coder throughput (c/compress.cs:69-943) on the GPU, one DGRAM per
lane: N packets of about 1200 bytes of mixed compressibility (tests/test_range_coder
corpus), compress then decompress, HIP events around each call, results checked
against the input.  The oracle (1 host thread) is timed on the same batch.

    python tools/rc_bench.py [--packets 65536]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "enet-csharp_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--sweep", default="", help="diagnostics: LANES:WAVES[:1],... lanes per wave x waves per CU "
                                                  "[x symbol-major models] (ENET_HIP_RC_LANES / _WAVES / "
                                                  "_INTERLEAVE, libenethip_diag.so); each "
                                                  "config's compressed bytes are checked against the first's")
    a = ap.parse_args()
    import torch
    import enethip
    import oracle
    from test_range_coder import corpus, pack
    msgs = corpus(a.packets, seed=31, max_len=2400)
    data, off, lens = pack(msgs)
    limit = lens * 2 + 64
    lo = np.concatenate([[0], np.cumsum(limit.astype(np.uint64))[:-1]]).astype(np.uint64)
    ctx = enethip.Context(0, diag=bool(a.sweep))
    t = lambda x, dt: torch.from_numpy(np.ascontiguousarray(x).view(dt)).cuda()  # noqa: E731
    d_in, d_off, d_len = t(np.concatenate([data, np.zeros(16, np.uint8)]), np.uint8), t(off, np.int64), t(lens, np.int32)
    d_c = torch.zeros(int(limit.astype(np.uint64).sum()) + 16, dtype=torch.uint8, device="cuda")
    d_lo, d_lim, d_clen = t(lo, np.int64), t(limit, np.int32), torch.zeros(len(off), dtype=torch.int32, device="cuda")
    d_d = torch.zeros(int(limit.astype(np.uint64).sum()) + 16, dtype=torch.uint8, device="cuda")
    d_dlen = torch.zeros(len(off), dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()

    def timed(fn):
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                e0.record(s)
                fn()
                e1.record(s)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e-3)
        return float(np.median(ts))

    nbytes = float(lens.astype(np.uint64).sum())

    def run_once():
        tc = timed(lambda: ctx.range_coder_device(False, d_in, d_off, d_len, len(off), d_c, d_lo, d_lim, d_clen,
                                                  stream=s.cuda_stream))
        # decompress the compressed streams in place (each at its own output slot)
        td = timed(lambda: ctx.range_coder_device(True, d_c, d_lo, d_clen, len(off), d_d, d_lo, d_lim, d_dlen,
                                                  stream=s.cuda_stream))
        clen = d_clen.cpu().numpy().view(np.uint32)
        dd = d_d.cpu().numpy()
        dlen = d_dlen.cpu().numpy().view(np.uint32)
        ok = bool((dlen == lens).all() and all((dd[int(lo[i]):int(lo[i]) + len(m)] == m).all() for i, m in enumerate(msgs)))
        return {"tc": tc, "td": td, "clen": clen, "ok": ok}

    if a.sweep:
        first = None
        for cfg in a.sweep.split(","):
            lanes, waves, *il = cfg.split(":")
            os.environ["ENET_HIP_RC_LANES"], os.environ["ENET_HIP_RC_WAVES"] = lanes, waves
            os.environ["ENET_HIP_RC_INTERLEAVE"] = il[0] if il else "0"
            d_c.zero_()
            d_d.zero_()
            r = run_once()
            comp = (d_c.cpu().numpy().tobytes(), r["clen"].tobytes())
            first = first or comp
            print(json.dumps({"lanes_per_wave": int(lanes), "waves_per_cu": int(waves),
                              "symbol_major": os.environ["ENET_HIP_RC_INTERLEAVE"] != "0",
                              "compress_us": round(r["tc"] * 1e6, 1), "decompress_us": round(r["td"] * 1e6, 1),
                              "compress_GBps": round(nbytes / r["tc"] / 1e9, 3),
                              "decompress_GBps": round(nbytes / r["td"] / 1e9, 3),
                              "round_trip_ok": r["ok"], "same_bytes_as_first": comp == first}), flush=True)
        ctx.close()
        return
    r = run_once()
    tc, td, clen, ok = r["tc"], r["td"], r["clen"], r["ok"]
    lib = oracle.OracleLib()
    sub = min(len(off), 4096)
    t0 = time.perf_counter()
    oracle.range_coder_batch(lib, False, data, off[:sub], lens[:sub], limit[:sub])
    cpu = float(lens[:sub].astype(np.uint64).sum()) / (time.perf_counter() - t0)
    print(json.dumps({"packets": len(off), "input_bytes": int(nbytes), "ratio": round(float(clen.sum()) / nbytes, 4),
                      "compress_us": round(tc * 1e6, 1), "compress_GBps": round(nbytes / tc / 1e9, 3),
                      "decompress_us": round(td * 1e6, 1), "decompress_GBps": round(nbytes / td / 1e9, 3),
                      "cpu_oracle_1thread_MBps": round(cpu / 1e6, 1), "ok": ok}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
