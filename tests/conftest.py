"""Shared test setup: the gpu marker and import paths.

`-m "not gpu"` tests run on any CPU host; `-m gpu` tests need an MI355X and call
the HIP path through the C-ABI (libenethip.so)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "enet-csharp_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; calls the HIP path via the C-ABI")


@pytest.fixture(scope="session")
def golden():
    import json
    import numpy as np
    gdir = os.path.join(ROOT, "tests", "golden")
    meta = json.load(open(os.path.join(gdir, "vectors.json")))
    blob = np.fromfile(os.path.join(gdir, "vectors.bin"), dtype=np.uint8)
    return meta["vectors"], blob


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    return oracle.OracleLib()
