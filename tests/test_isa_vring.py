"""Static ISA checks of the VGPR-ring kernel (crc32_vring.hip), CPU only.

The kernel issues its global loads as inline asm and waits for them by hand
(counted vmcnt), so correctness depends on properties of the generated code,
checked here on the gfx950 ISA hipcc emits with the Makefile's flags:
  * no scratch (private) memory in the product instances: scratch ops are VMEM and
    would need vmcnt(0);
  * no instruction reads or overwrites a register while a load into it may be in
    flight, on any path of the control-flow graph (tools/isa_inflight_check.py);
  * no compiler instruction writes a ring register (v48-v63: the allocator limit
    amdgpu_num_vgpr(24) is what keeps it out of them); only inline asm does (the
    stage loads, and the edge path's masking of a landed slot);
  * at most 64 VGPRs: a launch runs one 16-wave workgroup per CU, and the next
    launch's workgroup (another stream) can share the CU as this one drains.
Both builds are checked: the product library and the diagnostics one (-DENET_HIP_DIAG).
"""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "enet-csharp_amd")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module", params=["product", "diag"])
def vring_isa(tmp_path_factory, request):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / f"vring_{request.param}.s"
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-mllvm", "-simplifycfg-sink-common=false",
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "csrc"), "--cuda-device-only", "-S",
           os.path.join(PKG, "csrc", "crc32_vring.hip"), "-o", str(out)]
    if request.param == "diag":
        cmd.insert(1, "-DENET_HIP_DIAG")
    subprocess.run(cmd, check=True, capture_output=True)
    return str(out)


def test_vring_makefile_flags_match():
    mk = open(os.path.join(PKG, "Makefile")).read()
    assert "build/crc32_vring.o:" in mk and "-simplifycfg-sink-common=false" in mk


def test_vring_no_scratch_and_vgpr_budget(vring_isa):
    text = open(vring_isa).read()
    names = [l.split(":", 1)[1].strip() for l in text.splitlines() if l.strip().startswith(".name:")]
    vgprs = [int(l.split(":")[1]) for l in text.splitlines() if l.strip().startswith(".vgpr_count:")]
    sizes = [int(l.split(":")[1]) for l in text.splitlines() if l.strip().startswith(".private_segment_fixed_size:")]
    assert names and len(names) == len(vgprs) == len(sizes)
    for name, v, priv in zip(names, vgprs, sizes):
        assert v <= 64, (name, v)
        # the product instances stream with no scratch; the diagnostics (trace)
        # instance may spill a few dwords (its loads are still checked below)
        trace = re.findall(r"crc32_vring_kernelILi\d+ELi(\d+)E", name) != ["0"]
        assert trace or priv == 0, (name, priv)


def test_vring_loads_not_touched_before_wait(vring_isa):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_inflight_check as chk
    assert chk.main(vring_isa) == 0


def test_ring_write_check_catches_a_compiler_write():
    """The checker flags a compiler instruction that writes a ring register (it
    would corrupt a landed slot before its fold), and passes the asm loads."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_inflight_check as chk
    body = [";;#ASMSTART", "global_load_dwordx4 v[48:51], v[0:1], off", ";;#ASMEND",
            "s_waitcnt vmcnt(0)", "v_xor_b32_e32 v1, v48, v2", "s_endpgm"]
    assert chk.check(body, "k") == []
    bad = body[:-1] + ["v_mov_b32_e32 v52, 0", "s_endpgm"]
    assert any("writes ring" in e for e in chk.check(bad, "k"))


def test_ring_write_check_asm_writes():
    """An inline-asm write to a landed slot (the edge path's in-place masking) passes;
    the same write while the slot's load may still be in flight is flagged."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_inflight_check as chk
    load = [";;#ASMSTART", "global_load_dwordx4 v[48:51], v[0:1], off", ";;#ASMEND"]
    mask = [";;#ASMSTART", "v_and_b32 v48, v48, v2", ";;#ASMEND"]
    assert chk.check(load + ["s_waitcnt vmcnt(0)"] + mask + ["s_endpgm"], "k") == []
    errs = chk.check(load + mask + ["s_waitcnt vmcnt(0)", "s_endpgm"], "k")
    assert any("may be in flight" in e for e in errs)


def test_inflight_check_follows_structurizer_flags():
    """hipcc's structurizer may lay an if / else out as two conditional blocks joined by
    a flag pair.  Both arms issue a stage and wait for the previous one; the checker
    must not report the infeasible path that skips both arms -- but must still report
    a real miss (an arm that forgets its wait, or a flag it cannot know)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_inflight_check as chk

    def kernel(meta_wait="s_waitcnt vmcnt(2)", else_flag="s_mov_b64 s[10:11], -1"):
        return [";;#ASMSTART", "global_load_dwordx4 v[48:51], v[0:1], off", ";;#ASMEND",
                else_flag,
                "s_cbranch_scc1 .LBB0_2",                    # -> the else arm
                "s_mov_b64 s[10:11], 0",                     # the if arm
                ";;#ASMSTART", "global_load_lds_dword v[2:3], off", ";;#ASMEND",
                ";;#ASMSTART", "global_load_dwordx4 v[56:59], v[4:5], off", ";;#ASMEND",
                ";;#ASMSTART", meta_wait, ";;#ASMEND",
                ".LBB0_2:",
                "s_andn2_b64 vcc, exec, s[10:11]",
                "s_cbranch_vccnz .LBB0_3",
                ";;#ASMSTART", "global_load_dwordx4 v[56:59], v[4:5], off", ";;#ASMEND",   # the else arm
                ";;#ASMSTART", "s_waitcnt vmcnt(1)", ";;#ASMEND",
                ".LBB0_3:",
                "v_xor_b32_e32 v1, v48, v2",                 # the fold of the first stage
                "s_waitcnt vmcnt(0)",
                "s_endpgm"]
    assert chk.check(kernel(), "k") == []
    assert any("may be in flight" in e for e in chk.check(kernel(meta_wait="s_waitcnt vmcnt(3)"), "k"))
    assert any("may be in flight" in e for e in chk.check(kernel(else_flag="s_mov_b64 s[12:13], -1"), "k"))
