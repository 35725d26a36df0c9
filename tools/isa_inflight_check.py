#!/usr/bin/env python3
"""Static check of crc32_vring.hip's hand-counted loads (test infrastructure).

The vring kernel issues its global loads as inline asm and waits for them with
explicit `s_waitcnt vmcnt(N)`; the compiler sees a loaded register as written at
once, so nothing may read or overwrite it before the wait that retires the load
(a register reused while its load is in flight is clobbered when the load lands).

This is a dataflow analysis over the kernel's control-flow graph (hipcc -S
output): the state at each point is the ordered list of VMEM operations that may
still be in flight (the destination VGPRs of asm loads; other VMEM ops --
compiler loads, LDS-DMA, scratch loads -- count with no tracked registers;
stores are not queued, since they may complete out of order with the loads).
`s_waitcnt vmcnt(N)` keeps only the N youngest; at a join the lists are merged
aligned at their youngest end (element-wise union), which over-approximates what
may be in flight on any path.  Any instruction that names a register of an
in-flight asm load (other than the waits that tie them) is reported.

hipcc's CFG structurizer can turn an if / else into two conditional blocks joined by a
flag (`s_mov_b64 s[a:b], 0 / -1` in the arms, then `s_andn2_b64 vcc, exec, s[a:b]` +
`s_cbranch_vccnz` before the second block).  Path-insensitive, the analysis would also
follow the infeasible path that skips both arms; so it carries the SGPR pairs known to
hold 0 or -1 (and vcc's zero-ness derived from them) along every path into a point,
and follows only the feasible edge of a vcc branch they decide.

    python tools/isa_inflight_check.py path/to/kernel.s
"""
import re
import sys

VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
MAXQ = 64


def regs(text):
    out = set()
    for m in VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return frozenset(out)


RING = frozenset(range(48, 64))


def writes(line, op):
    """VGPRs an instruction writes: the first operand of a VALU op, a load or an LDS
    read / returning atomic (stores, DS writes and scalar ops write no VGPR)."""
    rest = line[len(op):]
    if not rest.strip():
        return frozenset()
    first = rest.split(",", 1)[0]
    if op.startswith("v_") and not op.startswith(("v_cmp_", "v_cmpx_", "v_readlane", "v_readfirstlane")):
        return regs(first)
    if op.startswith(("global_load", "buffer_load", "scratch_load", "flat_load")) and "lds" not in op:
        return regs(first)
    if op.startswith("ds_") and ("read" in op or "_rtn" in op or "bpermute" in op or "permute" in op):
        return regs(first)
    if "atomic" in op and " glc" in line + " ":
        return regs(first)
    return frozenset()


def parse(lines):
    """-> list of instructions (kind, text, regs, target, lineno) and label -> index."""
    insts, labels = [], {}
    in_asm = False
    for no, raw in enumerate(lines):
        st = raw.strip()
        if st == ";;#ASMSTART":
            in_asm = True
            continue
        if st == ";;#ASMEND":
            in_asm = False
            continue
        line = st.split(";")[0].strip()
        if not line:
            continue
        if line.endswith(":"):
            labels[line[:-1]] = len(insts)
            continue
        if line.startswith("."):
            continue
        op = line.split()[0]
        kind = "other"
        if in_asm and op.startswith("global_load") and "lds" not in op:
            kind = "aload"
        elif op.startswith(("global_", "buffer_", "scratch_", "flat_")):
            # a store (or an atomic without return) may complete out of order with
            # the loads, so it is no younger op a wait can count on: not queued
            # (loads return in order, so an in-flight load has every younger load
            # still counted by vmcnt, whatever the stores do)
            ret = "_load" in op or ("atomic" in op and " glc" in line + " ")
            kind = "vmem" if ret else "other"
        elif op == "s_waitcnt" and "vmcnt" in line:
            kind = "wait"
        elif op.startswith("s_cbranch") or op == "s_branch":
            kind = "branch"
        elif op == "s_endpgm":
            kind = "end"
        target = line.split()[1] if kind == "branch" and len(line.split()) > 1 else None
        insts.append((kind, line, op, target, no, in_asm))
    return insts, labels


def merge(a, b):
    if a is None:
        return b
    if b is None:
        return a
    n = max(len(a), len(b))
    pa = [frozenset()] * (n - len(a)) + list(a)
    pb = [frozenset()] * (n - len(b)) + list(b)
    return tuple(x | y for x, y in zip(pa, pb))


def step(state, inst):
    kind, line, op, _, _, _ = inst
    if kind == "aload":
        dst = line[len(op):].split(",", 1)[0]
        return (state + (frozenset((r, inst[4]) for r in regs(dst)),))[-MAXQ:]
    if kind == "vmem":
        return (state + (frozenset(),))[-MAXQ:]
    if kind == "wait":
        n = int(re.search(r"vmcnt\((\d+)\)", line).group(1))
        return state[len(state) - n:] if n < len(state) else state
    return state


SPAIR = re.compile(r"^s\[(\d+):(\d+)\]$")


def consts_step(consts, inst):
    """The known flag constants after an instruction: {'s[a:b]': 0 | -1, 'vcc': 'z' | 'nz'}."""
    kind, line, op, _, _, _ = inst
    ops = [x.strip() for x in line[len(op):].split(",")] if line[len(op):].strip() else []
    dst = ops[0] if ops else ""
    c = dict(consts)
    if op == "s_mov_b64" and SPAIR.match(dst) and len(ops) == 2 and ops[1] in ("0", "-1"):
        c[dst] = int(ops[1])
        return frozenset(c.items())
    if op in ("s_andn2_b64", "s_and_b64") and dst == "vcc" and len(ops) == 3 and ops[1] == "exec" and ops[2] in c \
            and isinstance(c[ops[2]], int):
        v = c[ops[2]]
        # (exec is non-zero wherever this kernel branches on vcc)
        nz = (v == 0) if op == "s_andn2_b64" else (v == -1)
        c["vcc"] = "nz" if nz else "z"
        return frozenset(c.items())
    # anything else that may write a tracked register forgets it
    written = set()
    if dst:
        written.add(dst)
    if op.startswith(("v_cmp", "v_cmpx")) and op.endswith("_e32"):
        written.add("vcc")
    if op.startswith("v_"):
        # a VALU op may also write an SGPR pair or vcc past its first operand (carry-outs
        # of v_add_co / v_sub_co / v_mad_u64, ...): forget every one it names
        for x in ops[1:]:
            if x == "vcc" or SPAIR.match(x) or re.match(r"^s\d+$", x):
                written.add(x)
    if "vcc" in dst:
        written.add("vcc")
    if written:
        def clash(key):
            if key == "vcc":
                return "vcc" in written
            a, b = map(int, SPAIR.match(key).groups())
            for w in written:
                m = SPAIR.match(w)
                lo, hi = (int(m.group(1)), int(m.group(2))) if m else ((int(w[1:]),) * 2 if re.match(r"^s\d+$", w) else (-1, -1))
                if lo <= b and a <= hi:
                    return True
            return False
        c = {k: v for k, v in c.items() if not clash(k)}
    return frozenset(c.items())


def check(lines, name):
    insts, labels = parse(lines)
    n = len(insts)
    succ = []
    for i, (kind, line, op, target, _, _) in enumerate(insts):
        s = []
        if kind == "branch" and target in labels:
            s.append(labels[target])
        # s_cbranch_execnz falls through only with EXEC == 0, which no wave of this
        # kernel reaches outside a divergent region (those are skipped with execz);
        # hipcc emits it as the exit of uniform loops, with implicit-defs on the dead
        # fall-through path
        if kind not in ("end",) and op not in ("s_branch", "s_cbranch_execnz") and i + 1 < n:
            s.append(i + 1)
        succ.append(s)
    # per point: {known flag constants: in-flight list} -- one entry per set of constants
    # (a disjunction over paths, so an if / else's two arms stay apart), collapsed to one
    # entry if more than MAXK sets reach a point
    MAXK = 32
    sets = [None] * n
    sets[0] = {frozenset(): ()}
    work = [0]
    while work:
        i = work.pop()
        kind, line, op, target, _, _ = insts[i]
        adds = {}
        for cin, st in sets[i].items():
            out = step(st, insts[i])
            cout = consts_step(cin, insts[i])
            targets = succ[i]
            known = dict(cin).get("vcc")
            if op in ("s_cbranch_vccnz", "s_cbranch_vccz") and known is not None and target in labels:
                taken = (known == "nz") == (op == "s_cbranch_vccnz")
                targets = [labels[target]] if taken else [j for j in succ[i] if j == i + 1]
            for j in targets:
                adds.setdefault(j, []).append((cout, out))
        for j, items in adds.items():
            cur = dict(sets[j]) if sets[j] is not None else {}
            for cout, out in items:
                cur[cout] = merge(cur.get(cout), out)
            if len(cur) > MAXK:
                meet = frozenset.intersection(*cur.keys())
                acc = None
                for v in cur.values():
                    acc = merge(acc, v)
                cur = {meet: acc}
            if sets[j] is None or cur != sets[j]:
                sets[j] = cur
                work.append(j)
    state_in = []
    for d in sets:
        if d is None:
            state_in.append(None)
            continue
        acc = None
        for v in d.values():
            acc = merge(acc, v)
        state_in.append(acc)
    errors = []
    # the ring registers v48-v63 are written only by inline asm (the stage loads and
    # the edge path's in-place masking of a landed slot): a compiler instruction
    # writing one (a temporary the allocator placed there) would corrupt a slot
    # between its wait and its fold, and the in-flight pass cannot see that.  (The
    # asm writes are still checked below: none may touch a slot in flight.)
    for i, inst in enumerate(insts):
        kind, line, op, _, no, asm = inst
        if kind == "aload" or asm:
            continue
        hit = writes(line, op) & RING
        if hit:
            errors.append(f"{name}:{no + 1}: '{line}' writes ring register(s) v{sorted(hit)}")
    for i, inst in enumerate(insts):
        kind, line, op, _, no, _ = inst
        st = state_in[i]
        if st is None or kind == "wait":
            continue
        busy_pairs = frozenset().union(*st) if st else frozenset()
        busy = frozenset(r for r, _ in busy_pairs)
        if not busy:
            continue
        used = regs(line)
        if kind == "aload":
            dst, rest = line[len(op):].split(",", 1)
            # a load may overwrite its own earlier in-flight destination (same register,
            # loads land in order) but may not read one as its address
            used = regs(rest)
        hit = busy & used
        if hit:
            src = sorted({o + 1 for r, o in busy_pairs if r in hit})
            errors.append(f"{name}:{no + 1}: '{line}' touches v{sorted(hit)} while the load(s) at {src} may be in flight")
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
            if "s_endpgm" in raw and not raw.strip().startswith(";"):
                yield cur, body
                cur = None


def main(path, skip_trace=False):
    errs, n = [], 0
    for name, body in kernels(open(path).read()):
        # crc32_vring_kernel<LG, TR>: skip the diagnostics (TR = 1) instance if asked
        targs = re.findall(r"ILi(\d+)ELi(\d+)E", name)
        if skip_trace and targs and targs[0][1] == "1":
            continue
        n += 1
        errs += check(body, name)
    for e in errs[:40]:
        print(e)
    print(f"{n} kernels checked, {len(errs)} violations")
    return 1 if errs or n == 0 else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
