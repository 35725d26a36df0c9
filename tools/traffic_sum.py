#!/usr/bin/env python3
"""HBM bytes per call of a multi-kernel entry point from a rocprofv3 --pmc
FETCH_SIZE pass (measurement infrastructure): the length-binned checksum
(bin_tile_kernel + the checksum kernel) or the binned gather (+ the join).  Every
dispatch whose kernel name matches --kernels is summed and divided by --calls;
FETCH_SIZE is converted as tools/traffic.py does (KiB x 1024 x 2 on gfx950,
MI355X_MICROARCH.md §HBM), the read probe in the same pass calibrating it.

    python tools/traffic_sum.py <pmc dir> --bytes B --calls N --out f.json [--kernels regex] [--probe-bytes P]
"""
import argparse
import csv
import glob
import json
import re
from collections import defaultdict
import os as _os


def product_library_sha256():
    """sha256 of the product library the pass ran (enet-csharp_amd/libenethip.so, or
    ENET_HIP_LIBRARY): bench.py reads this record only with that same build."""
    import sys as _sys
    root = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
    _sys.path.insert(0, _os.path.join(root, "enet-csharp_amd"))
    import enethip
    return enethip.library_sha256()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--bytes", type=float, required=True, help="algorithmic bytes per call")
    ap.add_argument("--calls", type=int, required=True)
    ap.add_argument("--kernels", default="vring_kernel|lean_kernel|bin_tile_kernel|gather_join|gather_small")
    ap.add_argument("--probe-bytes", type=float, default=0.0, help="bytes one read-probe dispatch reads")
    ap.add_argument("--what", default="")
    ap.add_argument("--binned", action="store_true", help="mark the file as the length-binned entry's "
                                                           "(bench.py --binned reads it)")
    ap.add_argument("--out")
    a = ap.parse_args()
    rx = re.compile(a.kernels)
    per_kernel = defaultdict(list)
    probe = []
    for f in glob.glob(f"{a.dir}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != "FETCH_SIZE":
                continue
            name, v = row["Kernel_Name"], float(row["Counter_Value"])
            if "read_probe" in name:
                probe.append(v)
            elif rx.search(name):
                per_kernel[name.split("(")[0][:90]].append(v)
    total_kib = sum(sum(v) for v in per_kernel.values())
    hbm = total_kib * 2048 / a.calls
    doc = {
        "what": a.what,
        "source": "rocprofv3 --pmc FETCH_SIZE (own pass); every dispatch of the entry's kernels summed per call",
        "correction": "bytes = FETCH_SIZE[KiB] * 1024 * 2 (gfx950 streaming-read 1/2 tally)",
        "calls": a.calls,
        "algorithmic_bytes_per_call": a.bytes,
        "per_kernel_mean_bytes": {k: round(sum(v) / len(v) * 2048) for k, v in per_kernel.items()},
        "per_kernel_dispatches": {k: len(v) for k, v in per_kernel.items()},
        "hbm_bytes_per_call": round(hbm),
        "hbm_bytes_per_batch": round(hbm),                 # (one batch per call)
        # the length-binned entries run bin_tile_kernel: tag them whatever the flag said
        # (bench.py --binned reads traffic_<cfg>_binned.json and checks this tag)
        "binned": bool(a.binned or any("bin_tile_kernel" in k for k in per_kernel)),
        "library_sha256": product_library_sha256(),
        "traffic_over_algorithmic": round(hbm / a.bytes, 4),
        "probe_calibration": (round(sum(probe) / len(probe) * 2048 / a.probe_bytes, 4)
                              if probe and a.probe_bytes else None),
    }
    print(json.dumps(doc, indent=1))
    if a.out:
        json.dump(doc, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
