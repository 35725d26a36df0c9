#!/usr/bin/env python3
"""Static check of crc32_vring.hip's hand-counted loads (test infrastructure).

The vring kernel issues its global loads as inline asm and waits for them with
explicit `s_waitcnt vmcnt(N)`; the compiler sees the loaded registers as ready
at once, so nothing may read or copy them before that wait.  This scans the
kernel's ISA (hipcc -S) in program order: for every asm `global_load*` it
collects the destination VGPRs and fails if any instruction before the next asm
`s_waitcnt vmcnt` reads or overwrites one of them.

    python tools/isa_inflight_check.py path/to/kernel.s
"""
import re
import sys

VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def check(lines, name):
    errors = []
    in_asm = False
    pending = []                          # (line no, dest regs)
    for no, raw in enumerate(lines):
        line = raw.split(";")[0].strip() if not raw.strip().startswith(";;#") else raw.strip()
        if raw.strip() == ";;#ASMSTART":
            in_asm = True
            continue
        if raw.strip() == ";;#ASMEND":
            in_asm = False
            continue
        if not line or line.endswith(":") or line.startswith("."):
            continue
        op = line.split()[0]
        if in_asm and op.startswith("global_load"):
            dst, rest = line[len(op):].split(",", 1)
            busy = regs(dst)
            for pno, preg in pending:     # a load may not reuse a pending destination
                if preg & (regs(rest) | busy):
                    errors.append(f"{name}:{no + 1}: load touches registers of the load at {pno + 1}")
            pending.append((no, busy))
            continue
        if in_asm and op == "s_waitcnt" and "vmcnt" in line:
            pending = []
            continue
        if pending:
            used = regs(line)
            for pno, preg in pending:
                if preg & used:
                    errors.append(f"{name}:{no + 1}: '{line}' touches v{sorted(preg & used)} "
                                  f"loaded at {pno + 1} before its wait")
    return errors


def kernels(text):
    cur, body = None, []
    for raw in text.splitlines():
        m = re.match(r"^(_Z\S*crc32_vring\S*):", raw)
        if m:
            cur, body = m.group(1), []
            continue
        if cur is not None:
            body.append(raw)
            if "s_endpgm" in raw:
                yield cur, body
                cur = None


def main(path):
    errs, n = [], 0
    for name, body in kernels(open(path).read()):
        n += 1
        errs += check(body, name)
    for e in errs[:40]:
        print(e)
    print(f"{n} kernels checked, {len(errs)} violations")
    return 1 if errs or n == 0 else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
