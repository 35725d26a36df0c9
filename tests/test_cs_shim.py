"""The C# P/Invoke shim (enet-csharp_amd/cs/EnetHip.cs) binds every
entry point of the product library's header with the same number of parameters
(CPU only; no .NET toolchain here or on the GPU box to compile it)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    text = open(os.path.join(ROOT, "include", "enet_hip.h")).read()
    text = re.sub(r"#ifdef ENET_HIP_DIAG.*?#endif /\* ENET_HIP_DIAG \*/", "", text, flags=re.S)   # product only
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    out = {}
    for m in re.finditer(r"ENET_HIP_API\s+[^;(]*?\b(enet_hip_\w+)\s*\(([^;]*?)\)\s*;", text, flags=re.S):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def _cs_functions():
    text = open(os.path.join(ROOT, "enet-csharp_amd", "cs", "EnetHip.cs")).read()
    out = {}
    for m in re.finditer(r"static extern\s+[\w*]+\s+(enet_hip_\w+)\s*\(([^;]*?)\)\s*;", text, flags=re.S):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params == "" else params.count(",") + 1
    return out


def test_cs_shim_binds_every_product_entry_point():
    h, cs = _header_functions(), _cs_functions()
    assert len(h) > 40
    missing = sorted(set(h) - set(cs))
    assert not missing, missing
    wrong = {f: (h[f], cs[f]) for f in h if h[f] != cs[f]}
    assert not wrong, wrong
    extra = sorted(set(cs) - set(h))
    assert not extra, extra                                      # no diagnostics entry in the shim
