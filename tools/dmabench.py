#!/usr/bin/env python3
"""Drive tools/dmabench.hip (measurement only): memory-side ceilings of LDS-DMA
streamed persistent kernels vs plain coalesced probes, 75 MiB per launch, 5
rotating buffers.  One JSON line per configuration (median event time)."""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libdmabench.so")
SRC = os.path.join(HERE, "dmabench.hip")


def build():
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(SRC):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17",
                        SRC, "-o", SO], check=True)


def main():
    build()
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        return
    import torch
    lib = ctypes.CDLL(SO)
    lib.db_name.restype = ctypes.c_char_p
    nbytes = 78643200
    bufs = [torch.randint(0, 255, (nbytes + 4096,), dtype=torch.uint8, device="cuda") for _ in range(5)]  # +4 KiB: window overrun
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    h = ctypes.c_void_p(st.cuda_stream)
    reps = 60

    def timeit(fn):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
        torch.cuda.synchronize()
        torch.cuda._sleep(int(1e8))
        for i in range(reps):
            ev[2 * i].record(st)
            fn(i)
            ev[2 * i + 1].record(st)
        torch.cuda.synchronize()
        t = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(reps))
        return t[len(t) // 2] * 1e3

    if len(sys.argv) > 1 and sys.argv[1] == "timeline":
        sys.path.insert(0, HERE)
        import numpy as np
        from timeline import analyze
        tr = torch.zeros(256 * 16 * 4, dtype=torch.int64, device="cuda")
        lib.db_trace(ctypes.c_void_p(tr.data_ptr()))
        for cfg in (0, 5):
            traces = []
            for i in range(12):
                tr.zero_()
                lib.db_dma(cfg, ctypes.c_void_p(bufs[i % 5].data_ptr()), ctypes.c_uint64(nbytes), 256,
                           ctypes.c_void_p(sink.data_ptr()), h)
                torch.cuda.synchronize()
                traces.append(tr.cpu().numpy().view(np.uint64).reshape(-1, 4).copy())
            print("== dma cfg", cfg, lib.db_name(cfg).decode())
            analyze(traces)
        lib.db_trace(None)
        return
    for cfg, grid, name in [(0, 512, "probe 512t x4 g512"), (1, 256, "probe 1024t x4 g256"),
                            (2, 256, "probe 1024t x8 g256"), (3, 1024, "probe 256t x4 g1024"),
                            (0, 2048, "probe 512t x4 g2048"), (0, 4800, "probe 512t x4 g4800")]:
        us = timeit(lambda i: lib.db_probe(cfg, ctypes.c_void_p(bufs[i % 5].data_ptr()), ctypes.c_uint64(nbytes),
                                           grid, ctypes.c_void_p(sink.data_ptr()), h))
        print(json.dumps({"kind": "probe", "name": name, "us": round(us, 2), "GBps": round(nbytes / us / 1e3, 1)}),
              flush=True)
    for cfg in range(lib.db_ncfg()):
        us = timeit(lambda i: lib.db_dma(cfg, ctypes.c_void_p(bufs[i % 5].data_ptr()), ctypes.c_uint64(nbytes),
                                         256, ctypes.c_void_p(sink.data_ptr()), h))
        print(json.dumps({"kind": "dma", "cfg": cfg, "name": lib.db_name(cfg).decode(), "us": round(us, 2),
                          "GBps": round(nbytes / us / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
