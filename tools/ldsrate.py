#!/usr/bin/env python3
"""LDS read-rate microbenchmark driver (tools/microbench.hip k_ldsrate)."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch
import microbench as mb

def main():
    mb.build()
    L = ctypes.CDLL(mb.SO)
    L.mb_setup()
    L.mb_ldsrate.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    h = torch.cuda.current_stream().cuda_stream
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    steps = 256
    names = ["b32 consecutive", "b32 crc-layout", "b32 random 1KiB", "b64 consecutive", "b128 consecutive", "b32 own-column random row"]
    for mode in range(6):
        for grid in (cus, cus * 2):
            ms = mb.timeit(lambda i: L.mb_ldsrate(mode, steps, grid, sink.data_ptr(), h), reps=10)
            instr = grid * 8 * steps * 32            # wave-instructions
            per_cu = instr / cus
            # in-kernel clock unknown; report ns per wave-instruction per CU and cycles at 2.1/2.4 GHz
            ns = ms * 1e6 / per_cu
            print(json.dumps({"mode": mode, "name": names[mode], "grid": grid, "waves_per_cu": grid * 8 // cus,
                              "ms": round(ms, 4), "ns_per_waveinstr_per_cu": round(ns, 3),
                              "cyc@2.1": round(ns * 2.1, 2), "cyc@2.4": round(ns * 2.4, 2)}), flush=True)

if __name__ == "__main__":
    main()
