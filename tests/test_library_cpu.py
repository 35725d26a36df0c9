"""libenethip.so on a CPU host: it loads, exports every symbol include/enet_hip.h
declares, and its callback path (CPU, c/packet.cs:142-160 drop-in) is bit-exact.
No GPU compute is attempted here."""
import ctypes
import os
import re
import zlib

import numpy as np

import enethip
import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    text = open(os.path.join(ROOT, "include", "enet_hip.h")).read()
    return sorted(set(re.findall(r"ENET_HIP_API\s+[\w\s\*]+?\b(enet_hip_\w+)\s*\(", text)))


def test_header_lists_match_binding():
    assert _header_symbols() == sorted(enethip.EXPORTED_SYMBOLS)


def test_library_loads_and_exports_everything():
    lib = enethip.load()
    for name in _header_symbols():
        assert hasattr(lib, name), name
        assert ctypes.cast(getattr(lib, name), ctypes.c_void_p).value


def test_callback_path_golden(golden):
    vecs, blob = golden
    for v in vecs:
        segs = [bytes(blob[o:o + n]) for o, n in v["segments"]]
        assert enethip.enet_crc32(segs) == int(v["crc"], 16), v["kind"]


def test_callback_path_random_buffers():
    rng = np.random.default_rng(11)
    for _ in range(200):
        k = int(rng.integers(1, 8))
        segs = [rng.integers(0, 256, size=int(rng.integers(0, 700)), dtype=np.uint8).tobytes() for _ in range(k)]
        assert enethip.enet_crc32(segs) == oracle.host_to_net_32(zlib.crc32(b"".join(segs)))


def test_update_register_api():
    lib = enethip.load()
    data = b"123456789"
    buf = ctypes.create_string_buffer(data)
    reg = lib.enet_hip_crc32_update(0xFFFFFFFF, ctypes.cast(buf, ctypes.c_void_p), 4)
    reg = lib.enet_hip_crc32_update(reg, ctypes.cast(ctypes.byref(buf, 4), ctypes.c_void_p), 5)
    assert oracle.host_to_net_32(~reg & 0xFFFFFFFF) == 0x2639F4CB


def test_errors_without_device():
    lib = enethip.load()
    # argument errors are reported as -hipErrorInvalidValue before touching a device
    assert lib.enet_hip_crc32_batch_device(None, None, None, None, 1, None, None) == -1
    assert lib.enet_hip_set_tuning(None, 4, 2) == -1
    assert enethip.error_string(0) == "success"
