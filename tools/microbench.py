#!/usr/bin/env python3
"""Drive tools/microbench.hip (measurement only): read patterns and LDS lookup
rates on one MI355X.  Prints one JSON line per measurement."""
import ctypes
import json
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libmicrobench.so")


def build():
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(os.path.join(HERE, "microbench.hip")):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17",
                        "-I" + os.path.join(HERE, "..", "enet-csharp_amd", "csrc"),
                        "-I" + os.path.join(HERE, "..", "include"),
                        os.path.join(HERE, "microbench.hip"), "-o", SO], check=True)


def timeit(fn, reps=30):
    st = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    torch.cuda.synchronize()
    torch.cuda._sleep(int(2e8))
    for i in range(reps):
        ev[2 * i].record(st)
        fn(i)
        ev[2 * i + 1].record(st)
    torch.cuda.synchronize()
    t = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(reps))
    return t[len(t) // 2]


def main():
    build()
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        return
    L = ctypes.CDLL(SO)
    L.mb_read.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int,
                          ctypes.c_void_p, ctypes.c_void_p]
    L.mb_lds.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.mb_setup()
    torch.cuda.init()
    nbytes = 75 * (1 << 20) // 76800 * 76800          # multiple of 64*1200 and of 1 KiB*S
    bufs = [torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda") for _ in range(5)]
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    h = torch.cuda.current_stream().cuda_stream
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    res = []
    for mode, S, grid in [(0, 16, cus * 8), (0, 16, cus * 4), (0, 16, cus * 16),
                          (1, 1200, cus * 2), (1, 600, cus * 2), (1, 192, cus * 4),
                          (2, 1200, cus * 2), (2, 600, cus * 2), (2, 192, cus * 4),
                          (3, 240, cus * 2), (3, 400, cus * 1), (3, 144, cus * 4)]:
        if mode == 3:
            nb = nbytes // (64 * S) * (64 * S)
        else:
            nb = nbytes // S * S
        ms = timeit(lambda i: L.mb_read(mode, bufs[i % 5].data_ptr(), nb, S, grid, sink.data_ptr(), h))
        r = {"test": "read", "mode": mode, "S": S, "grid": grid, "ms": round(ms, 5), "GBps": round(nb / ms / 1e6, 1)}
        print(json.dumps(r), flush=True)
        res.append(r)
    L.mb_crc_compute.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    # same work as cfg2 at 2 lanes/packet: 131072 lanes x 19 blocks (= 75 MiB / 32 B)
    for layout in (0, 1):
        for grid, blocks in ((256, 19), (512, 38 // 2), (256 * 4, 19)):
            lanes = grid * 512
            ms = timeit(lambda i: L.mb_crc_compute(layout, blocks, grid, sink.data_ptr(), h), reps=10)
            nbyte = lanes * blocks * 32
            print(json.dumps({"test": "crc_compute", "layout": layout, "grid": grid, "blocks": blocks,
                              "ms": round(ms, 5), "GBps_equiv": round(nbyte / ms / 1e6, 1)}), flush=True)
    steps = 64
    for mode in (0, 1):
        for grid in (cus * 2, cus * 4):
            ms = timeit(lambda i: L.mb_lds(mode, steps, grid, sink.data_ptr(), h), reps=10)
            lookups = grid * 512 * steps * 32
            waveinstr_per_cu = lookups / 64 / cus
            clk = 2.1e9
            print(json.dumps({"test": "lds", "mode": mode, "grid": grid, "ms": round(ms, 4),
                              "Glookups_s": round(lookups / ms / 1e6, 1),
                              "cycles_per_wave_instr_at_2.1GHz": round(ms * 1e-3 * clk / waveinstr_per_cu, 2)}),
                  flush=True)


if __name__ == "__main__":
    main()
