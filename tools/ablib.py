#!/usr/bin/env python3
"""Run a script with enethip loading another build of the library (A/B builds).
    python tools/ablib.py LIB.so SCRIPT [args...]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "enet-csharp_amd"))
import enethip  # noqa: E402

enethip.LIB_PATH = os.path.abspath(sys.argv[1])
sys.argv = sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
