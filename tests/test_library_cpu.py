"""libenethip.so on a CPU host: it loads, exports every symbol include/enet_hip.h
declares, and its callback path (CPU, c/packet.cs:142-160 drop-in) is bit-exact.
No GPU compute is attempted here."""
import ctypes
import os
import re
import subprocess
import zlib

import numpy as np

import enethip
import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


SYM = r"ENET_HIP_API\s+[\w\s\*]+?\b(enet_hip_\w+)\s*\("


def _header_symbols(diag_section: bool = False):
    """Declarations outside (or, diag_section, inside) the #ifdef ENET_HIP_DIAG block."""
    text = open(os.path.join(ROOT, "include", "enet_hip.h")).read()
    m = re.search(r"#ifdef ENET_HIP_DIAG(.*?)#endif /\* ENET_HIP_DIAG \*/", text, re.S)
    assert m, "the header's diagnostics section"
    part = m.group(1) if diag_section else text[:m.start()] + text[m.end():]
    return sorted(set(re.findall(SYM, part)))


def test_header_lists_match_binding():
    assert _header_symbols() == sorted(enethip.EXPORTED_SYMBOLS)
    assert _header_symbols(True) == sorted(enethip.DIAG_SYMBOLS)


def _exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], check=True, capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.split()[-1].startswith("enet_hip_")}


def test_library_loads_and_exports_everything():
    lib = enethip.load()
    for name in _header_symbols():
        assert hasattr(lib, name), name
        assert ctypes.cast(getattr(lib, name), ctypes.c_void_p).value
    assert lib.enet_hip_is_diagnostics_build() == 0


def test_product_library_has_no_diagnostics():
    """The library a C# host loads cannot emit a wrong CRC: the ablation switch
    (wrong checksums by design) and the trace exist only in libenethip_diag.so,
    and the exports are exactly the header's product section."""
    assert _exported(enethip.LIB_PATH) == set(_header_symbols())
    diag = enethip.load(diag=True)
    assert diag.enet_hip_is_diagnostics_build() == 1
    assert _exported(enethip.DIAG_LIB_PATH) == set(_header_symbols()) | set(_header_symbols(True))


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
    # the round-5 socket pipelines: a null context or a missing output is refused first
    got = ctypes.c_size_t(7)
    assert lib.enet_hip_udp_receive_verify_submit(None, 0, None, 4096, 1, None, 0, 0, None, None,
                                                  ctypes.byref(got), 0) == -1 and got.value == 0
    assert lib.enet_hip_udp_receive_verify_complete(None, 0) == -1
    assert lib.enet_hip_udp_receive_decompress_verify(None, 0, None, 4096, 1, None, 0, 0, None, None,
                                                      ctypes.byref(got)) == -1
    assert lib.enet_hip_udp_compress_stamp_send(None, 0, None, 0, None, None, 0, None, None, 0, 0, 0,
                                                ctypes.byref(got)) == -1
    assert enethip.error_string(0) == "success"


def test_callback_every_length_and_alignment():
    """The callback's carry-less-multiply folding (buffers of 64 bytes or more, when
    the CPU has PCLMULQDQ) and its table tail: every length 0..320 at every 16-byte
    misalignment, long buffers, and registers chained through enet_hip_crc32_update,
    against zlib's CRC-32 (the same polynomial and register, packet.cs:142-160)."""
    lib = enethip.load()
    rng = np.random.default_rng(5)
    blob = rng.integers(0, 256, size=80000, dtype=np.uint8).tobytes()
    buf = ctypes.create_string_buffer(blob)
    base = ctypes.addressof(buf)
    for n in list(range(0, 321)) + [1023, 1024, 1025, 4095, 65536, 70001]:
        for off in (0, 1, 7, 15):
            reg = lib.enet_hip_crc32_update(0xFFFFFFFF, ctypes.c_void_p(base + off), n)
            assert (~reg & 0xFFFFFFFF) == zlib.crc32(blob[off:off + n]), (n, off)
    for cut in (0, 5, 64, 100, 777):                          # two calls chained
        reg = lib.enet_hip_crc32_update(0xFFFFFFFF, ctypes.c_void_p(base + 3), cut)
        reg = lib.enet_hip_crc32_update(reg, ctypes.c_void_p(base + 3 + cut), 5000 - cut)
        assert (~reg & 0xFFFFFFFF) == zlib.crc32(blob[3:5003]), cut
