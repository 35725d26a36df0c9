"""Which VGPRs does the compiler use in a kernel (outside inline-asm blocks)?

usage: python3 tools/isa_regs.py build/crc32_vring.s [substring-of-symbol ...]
Prints, per kernel whose symbol contains every substring: the highest VGPR the
compiler names, the free registers below 48 (the vring kernel's allocator
limit), and the instruction count.
"""
import re
import sys


def kernels(text):
    for m in re.finditer(r"^(_Z\S+):\s*; @", text, re.M):
        name = m.group(1)
        end = text.index(".Lfunc_end", m.end())
        yield name, text[m.end():end]


def compiler_lines(body):
    inasm = False
    for line in body.split("\n"):
        if ";;#ASMSTART" in line:
            inasm = True
        if not inasm:
            yield line.split(";")[0]
        if ";;#ASMEND" in line:
            inasm = False


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    text = open(path).read()
    for name, body in kernels(text):
        if not all(s in name for s in subs):
            continue
        regs, n = set(), 0
        for line in compiler_lines(body):
            if re.match(r"\s+[vsdg]\w+_", line):
                n += 1
            for m in re.finditer(r"\bv\[(\d+):(\d+)\]", line):
                regs.update(range(int(m.group(1)), int(m.group(2)) + 1))
            for m in re.finditer(r"\bv(\d+)\b", line):
                regs.add(int(m.group(1)))
        free = sorted(set(range(48)) - regs)
        print(f"{name}: max v{max(regs) if regs else -1}, free<48 {free}, {n} instructions")


if __name__ == "__main__":
    main()
