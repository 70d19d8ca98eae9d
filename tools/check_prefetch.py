#!/usr/bin/env python3
"""Check the pipelined kernel's asm granule prefetches in compiler assembly output.

g_prefetch64 (pipe_common.h) issues `global_load_dwordx2` from inline asm into a register the
loop carries, and the kernel waits for it with an explicit `s_waitcnt vmcnt` before reading it.
The compiler does not know the load is pending: if it copies the register (an AGPR spill under
register pressure, a move at a merge) or reads it before that wait, the copy holds the value from
before the load, and the late return can overwrite a register the compiler has since re-used.
This script follows each asm prefetch (the `;;#ASMSTART` blocks of `--cuda-device-only -S`
output) along the fall-through path to the first `s_waitcnt` that counts vector memory and
reports any instruction that reads its destination before it.  A branch, a label or the end of
the function ends the walk (the loop back edge carries the register to its wait by design).

    hipcc ... --cuda-device-only -S pipe.hip -o pipe.dev.s; python3 tools/check_prefetch.py pipe.dev.s
"""
from __future__ import annotations

import re
import sys

REG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")


def regs(text: str) -> set[tuple[str, int]]:
    out: set[tuple[str, int]] = set()
    for m in REG.finditer(text):
        if m.group(4) is not None:
            out.add((m.group(4), int(m.group(5))))
        else:
            out.update((m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def sources(ins: str) -> str:
    """The operands an instruction reads (stores, compares and scalar ops: all of them)."""
    op, _, args = ins.partition(" ")
    if op.startswith(("global_store", "buffer_store", "flat_store", "ds_write", "global_atomic", "s_", "v_cmp")):
        return args if not op.startswith("v_cmp") else args.split(",", 1)[-1]
    return args.split(",", 1)[1] if "," in args else ""


def main(paths: list[str]) -> int:
    bad = total = 0
    for path in paths:
        lines = open(path).read().splitlines()
        func = ""
        for i, ln in enumerate(lines):
            if re.match(r"^_Z\S+:", ln):
                func = ln.split(":")[0]
            ins = ln.split(";")[0].strip()
            if not (ins.startswith("global_load_dwordx2") and "off sc1" in ins):
                continue
            if not (i > 0 and "ASMSTART" in lines[i - 1] and i + 1 < len(lines) and "ASMEND" in lines[i + 1]):
                continue  # a compiler load (tracked) or a load that waits for itself
            total += 1
            dst = regs(ins.split(",")[0])
            for j in range(i + 2, len(lines)):
                nxt = lines[j].split(";")[0].strip()
                if not nxt or nxt.startswith("."):
                    continue
                if nxt.endswith(":"):
                    break  # a label: another path joins here
                if nxt.startswith("s_waitcnt") and "vmcnt" in nxt:
                    break
                if nxt.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc")):
                    break
                if dst & regs(sources(nxt)):
                    bad += 1
                    print(f"EARLY READ in {func}: {ins} -> {nxt} (+{j - i} lines)")
                    break
    print(f"asm prefetches checked {total}, read before their wait {bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
