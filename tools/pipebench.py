#!/usr/bin/env python3
"""Drive tools/pipebench.hip (measurement only): the lean kernel's memory
pipeline with a realistic consumer, per ring depth / table layout / window
alignment.  cfg2 geometry (65536 x 1200 B), 5 rotating buffers.  Prints the
serial-region average (events around 100 launches, kernel boundary included)
and the bracketed median per launch."""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libpipebench.so")
SRC = os.path.join(HERE, "pipebench.hip")


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
    lib.pb_name.restype = ctypes.c_char_p
    n, L = 65536, 1200
    nbytes = n * L
    bufs = [torch.randint(0, 255, (nbytes + 4096,), dtype=torch.uint8, device="cuda") for _ in range(5)]
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * L
    zero = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    h = ctypes.c_void_p(st.cuda_stream)
    ngroups = n // 8
    cfgs = [int(c) for c in sys.argv[1].split(",")] if len(sys.argv) > 1 else list(range(lib.pb_ncfg()))

    def run(cfg, i):
        rc = lib.pb_run(cfg, ctypes.c_void_p(bufs[i % 5].data_ptr()), ctypes.c_void_p(offs.data_ptr()),
                        ctypes.c_uint64(ngroups), ctypes.c_void_p(zero.data_ptr()),
                        ctypes.c_void_p(sink.data_ptr()), h)
        assert rc == 0, rc

    reps = 100
    for cfg in cfgs:
        for i in range(10):
            run(cfg, i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(2e8))
        e0.record(st)
        for i in range(reps):
            run(cfg, i)
        e1.record(st)
        torch.cuda.synchronize()
        region = e0.elapsed_time(e1) / reps * 1e3
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
        torch.cuda._sleep(int(2e8))
        for i in range(reps):
            ev[2 * i].record(st)
            run(cfg, i)
            ev[2 * i + 1].record(st)
        torch.cuda.synchronize()
        t = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(reps))
        print(json.dumps({"cfg": cfg, "name": lib.pb_name(cfg).decode(), "region_us": round(region, 2),
                          "bracket_us": round(t[reps // 2] * 1e3, 2),
                          "GBps_region": round(nbytes / region / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
