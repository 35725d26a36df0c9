"""Python host binding of libenethip.so (ctypes over include/enet_hip.h).

This mirrors the reference's checksum surface for Python hosts and the test /
bench harness:

* ``ENetBuffer`` / ``enet_crc32(buffers)`` -- the callback path
  (enet-csharp/ENet/c/packet.cs:142-160, include/win32.cs:25-29), CPU, never fails.
* ``Context`` -- one GPU: batched device-resident checksum, receive verify
  (c/protocol.cs:1052-1068) and gather-list checksum (c/protocol.cs:1690-1698).
* ``crc32_batch_multi`` -- independent shards over several GPUs, no collective.

The GPU path has no fallback: if libenethip.so is missing or the HIP runtime
reports an error, these calls raise ``ENetHipError``.

``load(diag=True)`` / ``Context(..., diag=True)`` bind libenethip_diag.so instead:
the same library built with -DENET_HIP_DIAG, which adds the sweep-only kernel
paths and the diagnostics entry points (``diag_ablation``: WRONG checksums by
design; ``diag_trace``).  Only tools/ and the sweep tests use it.
"""
from __future__ import annotations

import ctypes
import os
from typing import Sequence

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ENET_HIP_LIBRARY: another build of the product library (measurement A/B only)
LIB_PATH = os.environ.get("ENET_HIP_LIBRARY") or os.path.join(PKG_ROOT, "libenethip.so")
DIAG_LIB_PATH = os.path.join(PKG_ROOT, "libenethip_diag.so")

# Every symbol include/enet_hip.h declares (tests check the .so exports them all).
EXPORTED_SYMBOLS = (
    "enet_hip_crc32", "enet_hip_crc32_update", "enet_hip_device_count", "enet_hip_context_create",
    "enet_hip_context_destroy", "enet_hip_error_string", "enet_hip_set_tuning",
    "enet_hip_crc32_batch_device", "enet_hip_crc32_batch_list_device", "enet_hip_binned_workspace_size", "enet_hip_crc32_batch_device_binned",
    "enet_hip_verify_binned_workspace_size", "enet_hip_verify_batch_device_binned",
    "enet_hip_crc32_batch_host", "enet_hip_verify_batch_device", "enet_hip_verify_batch_list_device",
    "enet_hip_crc32_gather_device", "enet_hip_gather_binned_workspace_size", "enet_hip_crc32_gather_binned_device",
    "enet_hip_crc32_batch_multi", "enet_hip_device_alloc",
    "enet_hip_device_free", "enet_hip_host_alloc", "enet_hip_host_free", "enet_hip_memcpy_h2d",
    "enet_hip_memcpy_d2h", "enet_hip_synchronize", "enet_hip_read_probe_device", "enet_hip_set_kernel_path",
    "enet_hip_is_diagnostics_build", "enet_hip_fragment_reassemble_device",
    "enet_hip_range_compress_device", "enet_hip_range_decompress_device",
    "enet_hip_crc32_gather_binned_host", "enet_hip_udp_receive", "enet_hip_parse_headers", "enet_hip_udp_send",
    "enet_hip_stamp_callback", "enet_hip_verify_callback", "enet_hip_udp_receive_verify", "enet_hip_udp_stamp_send",
    "enet_hip_udp_receive_decompress_verify", "enet_hip_udp_compress_stamp_send",
    "enet_hip_udp_receive_verify_submit", "enet_hip_udp_receive_verify_complete",
)

# include/enet_hip.h socket-harness constants
ERRNO_BASE = 100000
DGRAM_TRUNCATED = 0xFFFFFFFF
DGRAM_CHECKSUM, DROP_SHORT, DROP_PEER, DROP_COMPRESSED, DROP_TRUNCATED = 0, 1, 2, 3, 4
# Declared under #ifdef ENET_HIP_DIAG: exported by libenethip_diag.so only.
DIAG_SYMBOLS = ("enet_hip_diag_ablation", "enet_hip_diag_trace")


class ENetHipBatch(ctypes.Structure):
    """include/enet_hip.h ENetHipBatch: one batch of a batch-list call (device pointers)."""
    _fields_ = [("bytes", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("lengths", ctypes.c_void_p),
                ("count", ctypes.c_size_t), ("out", ctypes.c_void_p)]


class ENetHipVerifyBatch(ctypes.Structure):
    """include/enet_hip.h ENetHipVerifyBatch: one batch of a receive-verify list call."""
    _fields_ = [("bytes", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("lengths", ctypes.c_void_p),
                ("slotOffsets", ctypes.c_void_p), ("connectIds", ctypes.c_void_p), ("count", ctypes.c_size_t),
                ("ok", ctypes.c_void_p), ("computed", ctypes.c_void_p)]


class ENetHipError(RuntimeError):
    def __init__(self, what: str, code: int):
        super().__init__(f"{what} failed: {code} ({error_string(code)})")
        self.code = code


class ENetBuffer(ctypes.Structure):
    """include/win32.cs:25-29 -- length first."""
    _fields_ = [("dataLength", ctypes.c_size_t), ("data", ctypes.c_void_p)]


_libs: dict = {}


def library_sha256(diag: bool = False, path: str | None = None) -> str | None:
    """sha256 of the library file load() would open (None if absent).  Measurements
    committed under profiles/ (the traffic passes) record it, and bench.py uses a record
    only with the very build it was taken with."""
    import hashlib
    p = path or (DIAG_LIB_PATH if diag else LIB_PATH)
    try:
        with open(p, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None


def load(path: str | None = None, diag: bool = False) -> ctypes.CDLL:
    """The product library (or, diag=True, the diagnostics build)."""
    key = path or (DIAG_LIB_PATH if diag else LIB_PATH)
    if key in _libs:
        return _libs[key]
    p = key
    if not os.path.exists(p):
        raise ENetHipError(f"load {p} (run __graft_entry__.build())", -1)
    L = ctypes.CDLL(p)
    vp, sz, i32, u32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint32
    L.enet_hip_crc32.restype = u32
    L.enet_hip_crc32.argtypes = [vp, sz]
    L.enet_hip_crc32_update.restype = u32
    L.enet_hip_crc32_update.argtypes = [u32, vp, sz]
    L.enet_hip_device_count.restype = i32
    L.enet_hip_device_count.argtypes = [ctypes.POINTER(i32)]
    L.enet_hip_context_create.restype = i32
    L.enet_hip_context_create.argtypes = [i32, ctypes.POINTER(vp)]
    L.enet_hip_context_destroy.restype = i32
    L.enet_hip_context_destroy.argtypes = [vp]
    L.enet_hip_error_string.restype = ctypes.c_char_p
    L.enet_hip_error_string.argtypes = [i32]
    L.enet_hip_set_tuning.restype = i32
    L.enet_hip_set_tuning.argtypes = [vp, i32, i32]
    if L.enet_hip_is_diagnostics_build():
        L.enet_hip_diag_ablation.restype = i32
        L.enet_hip_diag_ablation.argtypes = [vp, i32]
        L.enet_hip_diag_trace.restype = i32
        L.enet_hip_diag_trace.argtypes = [vp, vp]
    L.enet_hip_set_kernel_path.restype = i32
    L.enet_hip_set_kernel_path.argtypes = [vp, i32]
    L.enet_hip_crc32_batch_device.restype = i32
    L.enet_hip_crc32_batch_device.argtypes = [vp, vp, vp, vp, sz, vp, vp]
    L.enet_hip_crc32_batch_list_device.restype = i32
    L.enet_hip_crc32_batch_list_device.argtypes = [vp, vp, sz, vp]
    L.enet_hip_verify_batch_list_device.restype = i32
    L.enet_hip_verify_batch_list_device.argtypes = [vp, vp, sz, vp]
    L.enet_hip_binned_workspace_size.restype = sz
    L.enet_hip_binned_workspace_size.argtypes = [sz]
    L.enet_hip_crc32_batch_device_binned.restype = i32
    L.enet_hip_crc32_batch_device_binned.argtypes = [vp, vp, vp, vp, sz, vp, vp, sz, vp]
    L.enet_hip_verify_binned_workspace_size.restype = sz
    L.enet_hip_verify_binned_workspace_size.argtypes = [sz]
    L.enet_hip_verify_batch_device_binned.restype = i32
    L.enet_hip_verify_batch_device_binned.argtypes = [vp, vp, vp, vp, vp, vp, sz, vp, vp, vp, sz, vp]
    L.enet_hip_crc32_batch_host.restype = i32
    L.enet_hip_crc32_batch_host.argtypes = [vp, vp, sz, vp, vp, sz, vp]
    L.enet_hip_verify_batch_device.restype = i32
    L.enet_hip_verify_batch_device.argtypes = [vp, vp, vp, vp, vp, vp, sz, vp, vp, vp]
    L.enet_hip_gather_binned_workspace_size.restype = sz
    L.enet_hip_gather_binned_workspace_size.argtypes = [sz]
    L.enet_hip_crc32_gather_binned_device.restype = i32
    L.enet_hip_crc32_gather_binned_device.argtypes = [vp, vp, vp, vp, sz, vp, sz, vp, vp, sz, vp]
    L.enet_hip_crc32_gather_device.restype = i32
    L.enet_hip_crc32_gather_device.argtypes = [vp, vp, vp, vp, vp, sz, vp, vp]
    L.enet_hip_crc32_batch_multi.restype = i32
    L.enet_hip_crc32_batch_multi.argtypes = [vp, i32, vp, sz, vp, vp, sz, vp]
    L.enet_hip_device_alloc.restype = i32
    L.enet_hip_device_alloc.argtypes = [vp, sz, ctypes.POINTER(vp)]
    L.enet_hip_device_free.restype = i32
    L.enet_hip_device_free.argtypes = [vp, vp]
    L.enet_hip_host_alloc.restype = i32
    L.enet_hip_host_alloc.argtypes = [sz, ctypes.POINTER(vp)]
    L.enet_hip_host_free.restype = i32
    L.enet_hip_host_free.argtypes = [vp]
    L.enet_hip_memcpy_h2d.restype = i32
    L.enet_hip_memcpy_h2d.argtypes = [vp, vp, vp, sz]
    L.enet_hip_memcpy_d2h.restype = i32
    L.enet_hip_memcpy_d2h.argtypes = [vp, vp, vp, sz]
    L.enet_hip_read_probe_device.restype = i32
    L.enet_hip_read_probe_device.argtypes = [vp, vp, sz, vp, vp]
    L.enet_hip_synchronize.restype = i32
    L.enet_hip_synchronize.argtypes = [vp]
    for f in ("enet_hip_range_compress_device", "enet_hip_range_decompress_device"):
        getattr(L, f).restype = i32
        getattr(L, f).argtypes = [vp, vp, vp, vp, sz, vp, vp, vp, vp, vp]
    szp = ctypes.POINTER(sz)
    L.enet_hip_crc32_gather_binned_host.restype = i32
    L.enet_hip_crc32_gather_binned_host.argtypes = [vp, vp, sz, vp, vp, sz, vp, sz, vp]
    L.enet_hip_udp_receive.restype = i32
    L.enet_hip_udp_receive.argtypes = [i32, vp, sz, sz, vp, vp, vp, i32, szp]
    L.enet_hip_parse_headers.restype = i32
    L.enet_hip_parse_headers.argtypes = [vp, sz, vp, sz, vp, sz, vp, vp, vp]
    L.enet_hip_udp_send.restype = i32
    L.enet_hip_udp_send.argtypes = [i32, vp, vp, vp, vp, sz, u32, ctypes.c_uint16, szp]
    L.enet_hip_stamp_callback.restype = i32
    L.enet_hip_stamp_callback.argtypes = [vp, vp, vp, vp, vp, sz]
    L.enet_hip_verify_callback.restype = i32
    L.enet_hip_verify_callback.argtypes = [vp, sz, vp, vp, vp, vp, sz, vp]
    L.enet_hip_udp_receive_verify.restype = i32
    L.enet_hip_udp_receive_verify.argtypes = [vp, i32, vp, sz, sz, vp, sz, i32, vp, vp, szp]
    L.enet_hip_udp_stamp_send.restype = i32
    L.enet_hip_udp_stamp_send.argtypes = [vp, i32, vp, sz, vp, vp, sz, vp, vp, sz, u32, ctypes.c_uint16, szp]
    # (an ENET_HIP_LIBRARY build from before round 5 lacks these: measurement A/B only)
    if p in (os.path.join(PKG_ROOT, "libenethip.so"), DIAG_LIB_PATH) or hasattr(L, "enet_hip_udp_receive_verify_submit"):
        L.enet_hip_udp_receive_verify_submit.restype = i32
        L.enet_hip_udp_receive_verify_submit.argtypes = [vp, i32, vp, sz, sz, vp, sz, i32, vp, vp, szp, i32]
        L.enet_hip_udp_receive_verify_complete.restype = i32
        L.enet_hip_udp_receive_verify_complete.argtypes = [vp, i32]
    if p in (os.path.join(PKG_ROOT, "libenethip.so"), DIAG_LIB_PATH) or hasattr(L, "enet_hip_udp_compress_stamp_send"):
        L.enet_hip_udp_receive_decompress_verify.restype = i32
        L.enet_hip_udp_receive_decompress_verify.argtypes = [vp, i32, vp, sz, sz, vp, sz, i32, vp, vp, szp]
        L.enet_hip_udp_compress_stamp_send.restype = i32
        L.enet_hip_udp_compress_stamp_send.argtypes = [vp, i32, vp, sz, vp, vp, sz, vp, vp, sz, u32, ctypes.c_uint16,
                                                       szp]
    L.enet_hip_is_diagnostics_build.restype = i32
    L.enet_hip_is_diagnostics_build.argtypes = []
    L.enet_hip_fragment_reassemble_device.restype = i32
    L.enet_hip_fragment_reassemble_device.argtypes = [vp, vp, vp, vp, vp, sz, u32, vp, vp, vp, vp, vp, u32, vp, sz,
                                                      vp, vp]
    _libs[key] = L
    return L


def error_string(code: int) -> str:
    try:
        s = load().enet_hip_error_string(int(code))
        return s.decode() if s else "?"
    except Exception:  # noqa: BLE001 - only used to format messages
        return "?"


def _check(what: str, rc: int) -> None:
    if rc != 0:
        raise ENetHipError(what, rc)


def _ptr(x) -> int:
    """Raw address of a numpy array, a torch tensor or an int."""
    if x is None:
        return 0
    if isinstance(x, int):
        return x
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    raise TypeError(type(x))


def enet_crc32(buffers: Sequence[bytes]) -> int:
    """CPU callback path: ENet.enet_crc32 over a gather list (packet.cs:142-160)."""
    L = load()
    keep = [np.frombuffer(bytes(b), dtype=np.uint8) for b in buffers]
    arr = (ENetBuffer * max(1, len(keep)))()
    for i, b in enumerate(keep):
        arr[i].dataLength = len(b)
        arr[i].data = b.ctypes.data if len(b) else None
    return int(L.enet_hip_crc32(ctypes.cast(arr, ctypes.c_void_p), len(keep)))


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = load().enet_hip_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


class Context:
    """One GPU.  Device pointers may be passed as torch tensors or ints."""

    def __init__(self, device: int = 0, lanes_per_packet: int = 0, workgroups_per_cu: int = 0, diag: bool = False):
        self.lib = load(diag=diag)
        self.diag = diag
        self._rx = [None, None]                                 # receive slots' ok[] in flight
        h = ctypes.c_void_p()
        _check("enet_hip_context_create", self.lib.enet_hip_context_create(int(device), ctypes.byref(h)))
        self.handle = h
        self.device = device
        if lanes_per_packet or workgroups_per_cu:
            self.set_tuning(lanes_per_packet, workgroups_per_cu)

    def set_tuning(self, lanes_per_packet: int = 0, workgroups_per_cu: int = 0) -> None:
        _check("enet_hip_set_tuning", self.lib.enet_hip_set_tuning(self.handle, lanes_per_packet, workgroups_per_cu))

    def set_kernel_path(self, path: int) -> None:
        """0 = default; 1 = direct loads, 2 = LDS stream kernel, 13 = lean kernel, 17 = vring
        kernel; the other paths (tuning sweeps) exist in the diagnostics library only."""
        _check("enet_hip_set_kernel_path", self.lib.enet_hip_set_kernel_path(self.handle, int(path)))

    def _need_diag(self, what: str) -> None:
        if not self.lib.enet_hip_is_diagnostics_build():
            raise ENetHipError(f"{what}: diagnostics entry point; open the Context with diag=True "
                               "(libenethip_diag.so) -- libenethip.so does not export it")

    def diag_ablation(self, mode: int) -> None:
        """Diagnostics only: 1 = no lookups, 2 = no DMA (wrong CRCs by design)."""
        self._need_diag("enet_hip_diag_ablation")
        _check("enet_hip_diag_ablation", self.lib.enet_hip_diag_ablation(self.handle, int(mode)))

    def diag_trace(self, device_ptr) -> None:
        """Diagnostics only: per-wave timeline buffer (4 x u64 per wave) or None."""
        self._need_diag("enet_hip_diag_trace")
        p = _ptr(device_ptr) if device_ptr is not None else None
        _check("enet_hip_diag_trace", self.lib.enet_hip_diag_trace(self.handle, p))

    def close(self) -> None:
        if getattr(self, "handle", None):
            self.lib.enet_hip_context_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # --- device-resident batch entry points (async on `stream`) ---
    def crc32_batch_device(self, d_bytes, d_off, d_len, n: int, d_out, stream: int = 0) -> None:
        _check("enet_hip_crc32_batch_device", self.lib.enet_hip_crc32_batch_device(
            self.handle, _ptr(d_bytes), _ptr(d_off), _ptr(d_len), int(n), _ptr(d_out), stream or None))

    def crc32_batch_list_device(self, batches, stream: int = 0) -> None:
        """batches: sequence of (d_bytes, d_off, d_len, n, d_out); one launch per 48 batches."""
        arr = (ENetHipBatch * max(1, len(batches)))()
        for i, (b, o, l, n, out) in enumerate(batches):
            arr[i] = ENetHipBatch(_ptr(b) or None, _ptr(o) or None, _ptr(l) or None, int(n), _ptr(out) or None)
        _check("enet_hip_crc32_batch_list_device", self.lib.enet_hip_crc32_batch_list_device(
            self.handle, ctypes.cast(arr, ctypes.c_void_p), len(batches), stream or None))

    def verify_batch_list_device(self, batches, stream: int = 0) -> None:
        """batches: sequence of (d_bytes, d_off, d_len, d_slot, d_connect, n, d_ok, d_computed or None);
        one launch per 32 batches (c/protocol.cs:1052-1068 per DGRAM)."""
        arr = (ENetHipVerifyBatch * max(1, len(batches)))()
        for i, (b, o, l, so, cid, n, ok, comp) in enumerate(batches):
            arr[i] = ENetHipVerifyBatch(_ptr(b) or None, _ptr(o) or None, _ptr(l) or None, _ptr(so) or None,
                                        _ptr(cid) or None, int(n), _ptr(ok) or None, _ptr(comp) or None)
        _check("enet_hip_verify_batch_list_device", self.lib.enet_hip_verify_batch_list_device(
            self.handle, ctypes.cast(arr, ctypes.c_void_p), len(batches), stream or None))

    def binned_workspace_size(self, n: int) -> int:
        return int(self.lib.enet_hip_binned_workspace_size(int(n)))

    def crc32_batch_device_binned(self, d_bytes, d_off, d_len, n: int, d_out, d_workspace, workspace_bytes: int,
                                  stream: int = 0) -> None:
        _check("enet_hip_crc32_batch_device_binned", self.lib.enet_hip_crc32_batch_device_binned(
            self.handle, _ptr(d_bytes), _ptr(d_off), _ptr(d_len), int(n), _ptr(d_out), _ptr(d_workspace),
            int(workspace_bytes), stream or None))

    def verify_binned_workspace_size(self, n: int) -> int:
        return int(self.lib.enet_hip_verify_binned_workspace_size(int(n)))

    def verify_batch_device_binned(self, d_bytes, d_off, d_len, d_slot, d_connect, n: int, d_ok, d_workspace,
                                   workspace_bytes: int, d_computed=None, stream: int = 0) -> None:
        _check("enet_hip_verify_batch_device_binned", self.lib.enet_hip_verify_batch_device_binned(
            self.handle, _ptr(d_bytes), _ptr(d_off), _ptr(d_len), _ptr(d_slot), _ptr(d_connect), int(n),
            _ptr(d_ok), _ptr(d_computed) or None, _ptr(d_workspace), int(workspace_bytes), stream or None))

    def verify_batch_device(self, d_bytes, d_off, d_len, d_slot, d_connect, n: int, d_ok, d_computed=None,
                            stream: int = 0) -> None:
        _check("enet_hip_verify_batch_device", self.lib.enet_hip_verify_batch_device(
            self.handle, _ptr(d_bytes), _ptr(d_off), _ptr(d_len), _ptr(d_slot), _ptr(d_connect), int(n),
            _ptr(d_ok), _ptr(d_computed) or None, stream or None))

    def gather_device(self, d_bytes, d_seg_off, d_seg_len, d_seg_first, n_dgrams: int, d_out,
                      stream: int = 0) -> None:
        _check("enet_hip_crc32_gather_device", self.lib.enet_hip_crc32_gather_device(
            self.handle, _ptr(d_bytes), _ptr(d_seg_off), _ptr(d_seg_len), _ptr(d_seg_first), int(n_dgrams),
            _ptr(d_out), stream or None))

    def gather_binned_workspace_size(self, seg_count: int) -> int:
        return int(self.lib.enet_hip_gather_binned_workspace_size(int(seg_count)))

    def gather_binned_device(self, d_bytes, d_seg_off, d_seg_len, seg_count: int, d_seg_first, n_dgrams: int,
                             d_out, d_workspace, workspace_bytes: int, stream: int = 0) -> None:
        """Gather-list CRCs via a length-binned pass over the segments and a join (enet_hip.h)."""
        _check("enet_hip_crc32_gather_binned_device", self.lib.enet_hip_crc32_gather_binned_device(
            self.handle, _ptr(d_bytes), _ptr(d_seg_off) or None, _ptr(d_seg_len) or None, int(seg_count),
            _ptr(d_seg_first), int(n_dgrams), _ptr(d_out), _ptr(d_workspace) or None, int(workspace_bytes),
            stream or None))

    def fragment_reassemble_device(self, d_bytes, d_cmd_off, d_cmd_avail, d_slots, n: int, max_packet: int,
                                   d_msg_bytes, d_msg_off, d_msg_len, d_msg_count, d_fragments, words: int,
                                   d_remaining, n_slots: int, d_status, stream: int = 0) -> None:
        """Batched fragment reassembly (c/protocol.cs:529-637): see enet_hip.h."""
        _check("enet_hip_fragment_reassemble_device", self.lib.enet_hip_fragment_reassemble_device(
            self.handle, _ptr(d_bytes), _ptr(d_cmd_off), _ptr(d_cmd_avail), _ptr(d_slots), int(n), int(max_packet),
            _ptr(d_msg_bytes), _ptr(d_msg_off), _ptr(d_msg_len), _ptr(d_msg_count), _ptr(d_fragments), int(words),
            _ptr(d_remaining), int(n_slots), _ptr(d_status), stream or None))

    def range_coder_device(self, decompress: bool, d_in, d_in_off, d_in_len, n: int, d_out, d_out_off,
                           d_out_limit, d_out_len, stream: int = 0) -> None:
        """Batched ENet range coder (c/compress.cs:69-943): see enet_hip.h."""
        name = "enet_hip_range_decompress_device" if decompress else "enet_hip_range_compress_device"
        _check(name, getattr(self.lib, name)(
            self.handle, _ptr(d_in), _ptr(d_in_off), _ptr(d_in_len), int(n), _ptr(d_out), _ptr(d_out_off),
            _ptr(d_out_limit), _ptr(d_out_len), stream or None))

    def read_probe_device(self, d_bytes, nbytes: int, d_sink, stream: int = 0) -> None:
        _check("enet_hip_read_probe_device", self.lib.enet_hip_read_probe_device(
            self.handle, _ptr(d_bytes), int(nbytes), _ptr(d_sink), stream or None))

    def synchronize(self) -> None:
        _check("enet_hip_synchronize", self.lib.enet_hip_synchronize(self.handle))

    # --- host-memory entry points and the GPU socket pipelines (synchronous) ---
    def gather_binned_host(self, payload: np.ndarray, seg_off, seg_len, seg_first) -> np.ndarray:
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        seg_off, seg_len, seg_first = _u(seg_off, np.uint64), _u(seg_len, np.uint32), _u(seg_first, np.uint32)
        n = len(seg_first) - 1
        out = np.zeros(max(1, n), dtype=np.uint32)
        _check("enet_hip_crc32_gather_binned_host", self.lib.enet_hip_crc32_gather_binned_host(
            self.handle, _ptr(payload), payload.nbytes, _ptr(seg_off) if len(seg_off) else None,
            _ptr(seg_len) if len(seg_len) else None, len(seg_off), _ptr(seg_first), n, _ptr(out)))
        return out[:n]

    def udp_receive_verify(self, fd: int, arena, stride: int, max_dgrams: int, peer_connect_ids,
                           timeout_ms: int = 0):
        """-> (count, lengths[count], ok[count]): socket -> header stage -> GPU verify -> keep mask."""
        peers = _u(peer_connect_ids, np.uint32)
        lens = np.zeros(max(1, max_dgrams), np.uint32)
        ok = np.zeros(max(1, max_dgrams), np.uint8)
        got = ctypes.c_size_t(0)
        _check("enet_hip_udp_receive_verify", self.lib.enet_hip_udp_receive_verify(
            self.handle, int(fd), _ptr(arena), int(stride), int(max_dgrams), _ptr(peers) if len(peers) else None,
            len(peers), int(timeout_ms), _ptr(lens), _ptr(ok), ctypes.byref(got)))
        n = got.value
        return n, lens[:n], ok[:n]

    def udp_stamp_send(self, fd: int, payload, seg_off, seg_len, seg_first, slot_off, addr: int, port: int) -> int:
        """GPU stamp of the gather-list DGRAMs (payload modified in place), then sendmmsg."""
        seg_off, seg_len, seg_first, slot_off = (_u(seg_off, np.uint64), _u(seg_len, np.uint32),
                                                 _u(seg_first, np.uint32), _u(slot_off, np.uint32))
        sent = ctypes.c_size_t(0)
        _check("enet_hip_udp_stamp_send", self.lib.enet_hip_udp_stamp_send(
            self.handle, int(fd), _ptr(payload), int(payload.nbytes), _ptr(seg_off), _ptr(seg_len), len(seg_off),
            _ptr(seg_first), _ptr(slot_off), len(seg_first) - 1, int(addr), int(port), ctypes.byref(sent)))
        return sent.value

    def udp_receive_verify_submit(self, slot: int, fd: int, arena, stride: int, max_dgrams: int, peer_connect_ids,
                                  timeout_ms: int = 0):
        """-> (count, lengths[count], ok[count]) with ok[] filled only by
        udp_receive_verify_complete(slot): the receive and its queued GPU verify of slot
        0 or 1 (the GPU work overlaps the caller's next receive)."""
        peers = _u(peer_connect_ids, np.uint32)
        lens = np.zeros(max(1, max_dgrams), np.uint32)
        ok = np.zeros(max(1, max_dgrams), np.uint8)
        got = ctypes.c_size_t(0)
        _check("enet_hip_udp_receive_verify_submit", self.lib.enet_hip_udp_receive_verify_submit(
            self.handle, int(fd), _ptr(arena), int(stride), int(max_dgrams), _ptr(peers) if len(peers) else None,
            len(peers), int(timeout_ms), _ptr(lens), _ptr(ok), ctypes.byref(got), int(slot)))
        self._rx[slot] = ok                                     # (held until its complete)
        n = got.value
        return n, lens[:n], ok[:n]

    def udp_receive_verify_complete(self, slot: int) -> None:
        _check("enet_hip_udp_receive_verify_complete", self.lib.enet_hip_udp_receive_verify_complete(self.handle, int(slot)))
        self._rx[slot] = None

    def udp_receive_decompress_verify(self, fd: int, arena, stride: int, max_dgrams: int, peer_connect_ids,
                                      timeout_ms: int = 0):
        """-> (count, lengths[count], ok[count]): as udp_receive_verify, compressed DGRAMs
        decompressed on the GPU first (range coder) and left decompressed in their arena
        slots with their new lengths (c/protocol.cs:1033-1068)."""
        peers = _u(peer_connect_ids, np.uint32)
        lens = np.zeros(max(1, max_dgrams), np.uint32)
        ok = np.zeros(max(1, max_dgrams), np.uint8)
        got = ctypes.c_size_t(0)
        _check("enet_hip_udp_receive_decompress_verify", self.lib.enet_hip_udp_receive_decompress_verify(
            self.handle, int(fd), _ptr(arena), int(stride), int(max_dgrams), _ptr(peers) if len(peers) else None,
            len(peers), int(timeout_ms), _ptr(lens), _ptr(ok), ctypes.byref(got)))
        n = got.value
        return n, lens[:n], ok[:n]

    def udp_compress_stamp_send(self, fd: int, payload, seg_off, seg_len, seg_first, slot_off, addr: int,
                                port: int) -> int:
        """GPU range compress of each DGRAM's commands, header flag where shorter, GPU
        stamp over the uncompressed lists (payload modified in place), then sendmmsg of
        the wire form (c/protocol.cs:1665-1705)."""
        seg_off, seg_len, seg_first, slot_off = (_u(seg_off, np.uint64), _u(seg_len, np.uint32),
                                                 _u(seg_first, np.uint32), _u(slot_off, np.uint32))
        sent = ctypes.c_size_t(0)
        _check("enet_hip_udp_compress_stamp_send", self.lib.enet_hip_udp_compress_stamp_send(
            self.handle, int(fd), _ptr(payload), int(payload.nbytes), _ptr(seg_off), _ptr(seg_len), len(seg_off),
            _ptr(seg_first), _ptr(slot_off), len(seg_first) - 1, int(addr), int(port), ctypes.byref(sent)))
        return sent.value

    # --- host-memory entry point (synchronous) ---
    def crc32_batch_host(self, payload: np.ndarray, off: np.ndarray, lens: np.ndarray) -> np.ndarray:
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        out = np.zeros(len(off), dtype=np.uint32)
        _check("enet_hip_crc32_batch_host", self.lib.enet_hip_crc32_batch_host(
            self.handle, _ptr(payload), payload.nbytes, _ptr(off), _ptr(lens), len(off), _ptr(out)))
        return out


def _u(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


# ------------------------------------------------------------------ socket harness
# (include/enet_hip.h "UDP socket batching harness"; fd = socket.fileno() of a bound
# IPv4 UDP socket, addresses as host-order ints)

def udp_receive(fd: int, arena: np.ndarray, stride: int, max_dgrams: int, timeout_ms: int = 0):
    """-> (count, lengths[count], src_addr[count], src_port[count]); DGRAM i at arena[i*stride:]."""
    L = load()
    lens = np.zeros(max(1, max_dgrams), np.uint32)
    addr = np.zeros(max(1, max_dgrams), np.uint32)
    port = np.zeros(max(1, max_dgrams), np.uint16)
    got = ctypes.c_size_t(0)
    _check("enet_hip_udp_receive", L.enet_hip_udp_receive(int(fd), _ptr(arena), int(stride), int(max_dgrams),
                                                          _ptr(lens), _ptr(addr), _ptr(port), int(timeout_ms),
                                                          ctypes.byref(got)))
    n = got.value
    return n, lens[:n], addr[:n], port[:n]


def parse_headers(arena: np.ndarray, stride: int, lengths: np.ndarray, peer_connect_ids: np.ndarray):
    """ENet's receive header stage (c/protocol.cs:1001-1030) -> (slot_off, connect_id, verdict)."""
    L = load()
    n = len(lengths)
    lengths = _u(lengths, np.uint32)
    peers = _u(peer_connect_ids, np.uint32)
    slot, conn, verdict = np.zeros(max(1, n), np.uint32), np.zeros(max(1, n), np.uint32), np.zeros(max(1, n), np.uint8)
    _check("enet_hip_parse_headers", L.enet_hip_parse_headers(_ptr(arena), int(stride), _ptr(lengths), n,
                                                              _ptr(peers) if len(peers) else None, len(peers),
                                                              _ptr(slot), _ptr(conn), _ptr(verdict)))
    return slot[:n], conn[:n], verdict[:n]


def udp_send(fd: int, payload: np.ndarray, seg_off, seg_len, seg_first, addr: int, port: int) -> int:
    """sendmmsg of the gather-list DGRAMs; returns how many the socket accepted."""
    L = load()
    seg_off, seg_len, seg_first = _u(seg_off, np.uint64), _u(seg_len, np.uint32), _u(seg_first, np.uint32)
    sent = ctypes.c_size_t(0)
    _check("enet_hip_udp_send", L.enet_hip_udp_send(int(fd), _ptr(payload), _ptr(seg_off), _ptr(seg_len),
                                                    _ptr(seg_first), len(seg_first) - 1, int(addr), int(port),
                                                    ctypes.byref(sent)))
    return sent.value


def stamp_callback(payload: np.ndarray, seg_off, seg_len, seg_first, slot_off) -> None:
    """Per-DGRAM callback stamp (protocol.cs:1690-1698), in place, on the CPU."""
    L = load()
    seg_off, seg_len, seg_first, slot_off = (_u(seg_off, np.uint64), _u(seg_len, np.uint32),
                                             _u(seg_first, np.uint32), _u(slot_off, np.uint32))
    _check("enet_hip_stamp_callback", L.enet_hip_stamp_callback(_ptr(payload), _ptr(seg_off), _ptr(seg_len),
                                                                _ptr(seg_first), _ptr(slot_off), len(seg_first) - 1))


def verify_callback(arena: np.ndarray, stride: int, lengths, slot_off, connect_ids, verdict=None) -> np.ndarray:
    """Per-DGRAM callback verify (protocol.cs:1052-1068) on the CPU, slot replaced in place."""
    L = load()
    n = len(lengths)
    lengths, slot_off, connect_ids = _u(lengths, np.uint32), _u(slot_off, np.uint32), _u(connect_ids, np.uint32)
    vd = None if verdict is None else _u(verdict, np.uint8)
    ok = np.zeros(max(1, n), np.uint8)
    _check("enet_hip_verify_callback", L.enet_hip_verify_callback(_ptr(arena), int(stride), _ptr(lengths),
                                                                  _ptr(slot_off), _ptr(connect_ids),
                                                                  _ptr(vd) if vd is not None else None, n, _ptr(ok)))
    return ok[:n]


def crc32_batch_multi(contexts: Sequence[Context], payload: np.ndarray, off: np.ndarray,
                      lens: np.ndarray) -> np.ndarray:
    L = load()
    payload = np.ascontiguousarray(payload, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    out = np.zeros(len(off), dtype=np.uint32)
    handles = (ctypes.c_void_p * len(contexts))(*[c.handle.value for c in contexts])
    _check("enet_hip_crc32_batch_multi", L.enet_hip_crc32_batch_multi(
        ctypes.cast(handles, ctypes.c_void_p), len(contexts), _ptr(payload), payload.nbytes, _ptr(off),
        _ptr(lens), len(off), _ptr(out)))
    return out
