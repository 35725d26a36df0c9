"""The C-ABI from a plain C host (tests/native/c_host.c): only include/enet_hip.h and
libenethip.so, no HIP headers and no Python in between -- the boundary a native ENet
host or the C# P/Invoke shim binds.  The program checks the CPU
callback (c/packet.cs:142-160), and with a device the batch, batch-list, receive-verify
(c/protocol.cs:1052-1068) and host-memory entries, against a bit-at-a-time CRC-32 it
carries itself.  CPU suite: builds it with gcc -Werror and runs it (no device here: the
callback and the no-device contract); GPU suite: the device half."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "enet-csharp_amd")


def build(tmp_path):
    if not shutil.which("gcc"):
        pytest.skip("gcc not found")
    if not os.path.exists(os.path.join(LIBDIR, "libenethip.so")):
        pytest.fail("libenethip.so not built (python -c 'import __graft_entry__ as g; g.build()')")
    exe = str(tmp_path / "c_host")
    subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "c_host.c"), "-L", LIBDIR, "-lenethip",
                    "-Wl,-rpath," + LIBDIR, "-o", exe], check=True, capture_output=True, text=True)
    return exe


def run(exe):
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_c_host_builds_and_runs(tmp_path):
    out = run(build(tmp_path))
    assert "c_host: ok (" in out


@pytest.mark.gpu
def test_c_host_device_entries(tmp_path):
    out = run(build(tmp_path))
    assert "c_host: ok (device)" in out, out
