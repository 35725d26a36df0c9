#!/usr/bin/env python3
"""HBM bytes per launch from a rocprofv3 --pmc FETCH_SIZE pass (test/measurement
infrastructure).  Per MI355X_MICROARCH.md §HBM: FETCH_SIZE is in KiB and on
gfx950 reports 1/2 of the bytes of a wide coalesced streaming read, so
bytes = FETCH_SIZE * 1024 * 2; the read-probe kernel (every payload byte read
once, 16 B/lane) in the same pass calibrates the correction for this image.

    python tools/traffic.py <pmc dir> <payload bytes per batch> <batches per launch> [out.json]
"""
import csv
import glob
import json
import sys
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
    d, batch, per = sys.argv[1], float(sys.argv[2]), int(sys.argv[3])
    payload = batch * per
    out = sys.argv[4] if len(sys.argv) > 4 else None
    vals = defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != "FETCH_SIZE":
                continue
            name = row["Kernel_Name"]
            key = "probe" if "read_probe" in name else "stream" if ("stream_kernel" in name or "lean_kernel" in name or "vring_kernel" in name) else name[:60]
            vals[key].append(float(row["Counter_Value"]))
    res = {k: sum(v) / len(v) for k, v in vals.items()}
    stream = res.get("stream")
    probe = res.get("probe")
    probe_bytes = (int(batch) // 16) * 16                 # the probe reads one batch
    doc = {
        "source": "rocprofv3 --pmc FETCH_SIZE (own pass), tools/profile_one.py --probe",
        "correction": "bytes = FETCH_SIZE[KiB] * 1024 * 2 (gfx950 streaming-read 1/2 tally)",
        "fetch_size_kib_stream": stream,
        "fetch_size_kib_probe": probe,
        "payload_bytes_per_launch": payload,
        "batches_per_launch": per,
        "hbm_bytes_per_launch": None if stream is None else round(stream * 2048),
        "hbm_bytes_per_batch": None if stream is None else round(stream * 2048 / per),
        "probe_bytes_per_launch": None if probe is None else round(probe * 2048),
        "probe_calibration": None if probe is None else round(probe * 2048 / probe_bytes, 4),
        "traffic_over_algorithmic": None if stream is None else round(stream * 2048 / payload, 4),
        "dispatches": {k: len(v) for k, v in vals.items()},
        "library_sha256": product_library_sha256(),
    }
    print(json.dumps(doc, indent=1))
    if out:
        json.dump(doc, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
