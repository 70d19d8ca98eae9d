#!/usr/bin/env python3
"""Check a disassembled gfx950 code object for the DPP read-after-VALU-write hazard.

gfx9 needs two wait states between a VALU instruction that writes a VGPR and a DPP instruction
that reads it (the DPP source, src0).  Inline asm that carries its own DPP is invisible to the
compiler's hazard recognizer, so a build that drops the asm's own `s_nop` relies on the
surrounding schedule: this script checks every DPP instruction of the named kernels.  A label
inside the window (a possible branch target) is reported as UNKNOWN (checked by hand).

    llvm-objdump -d CODE_OBJECT > k.s; python3 tools/dpp_hazards.py k.s [KERNEL_SUBSTRING]
"""
from __future__ import annotations

import re
import sys

REG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)")


def regs(text: str) -> set[int]:
    out: set[int] = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def main(path: str, kernel: str = "pipe_viterbi_kernel") -> int:
    lines = open(path).read().splitlines()
    inside = False
    window: list[tuple[str, set[int], int]] = []  # (mnemonic, written VGPRs, wait states provided)
    bad = unknown = checked = 0
    for ln in lines:
        if re.match(r"^[0-9a-f]+ <", ln):
            if "<L" in ln:  # a local label: a possible branch target
                window.append(("label", set(), 0))
            else:  # a function symbol
                inside = kernel in ln
                window = []
            continue
        if not inside:
            continue
        ins = ln.strip().split("//")[0].strip()
        if not ins:
            continue
        op = ins.split()[0]
        args = ins[len(op):]
        if "_dpp" in op or " row_" in ins or "wave_shr" in ins or "quad_perm" in ins:
            parts = [a.strip() for a in args.split(",")]
            src0 = regs(parts[1]) if len(parts) > 1 else set()
            states = 0
            for mn, wr, ws in reversed(window):
                if mn == "label":
                    unknown += 1
                    break
                if wr & src0 and states < 2:
                    bad += 1
                    print("HAZARD:", ins, "<- written", 2 - states, "wait state(s) short")
                    break
                states += ws
                if states >= 2:
                    break
            checked += 1
        written: set[int] = set()
        ws = 1
        if op.startswith("s_nop"):
            ws = int(args.strip() or "0", 0) + 1
        elif op.startswith("v_") and not op.startswith("v_readlane") and not op.startswith("v_cmp"):
            first = args.split(",")[0]
            written = regs(first)
        window.append((op, written, ws))
        window = window[-4:]
    print(f"dpp reads checked {checked}, hazards {bad}, after a label (check by hand) {unknown}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:]))
