#!/usr/bin/env python3
"""Compact table of tools/sweep.py JSON lines (stdin)."""
import json
import sys

for line in sys.stdin:
    try:
        d = json.loads(line)
    except ValueError:
        continue
    if "probe_ms" in d:
        print(f"probe {d['probe_ms'] * 1e3:7.2f} us  {d['probe_GBps']:7.0f} GB/s")
        continue
    print(f"path {d['path']} abl {d['ablate']} lanes {d['lanes']:2d} wgs {d['wgs']}  kernel {d['kernel_ms'] * 1e3:7.2f} us "
          f"{d['kernel_GBps']:7.0f} GB/s  graph {d['graph_ms_per_step'] * 1e3:7.2f} us  ok={d['ok']}")
