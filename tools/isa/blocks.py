#!/usr/bin/env python3
"""Instruction mix per basic block of one kernel in a gfx950 .s file (hipcc --cuda-device-only -S).
  blocks.py file.s kernel_symbol [block ...]   -> per-block counts, and the sum over the listed blocks
Classes: VALU (v_*), SALU (s_* but waits/branches/nops), LDS (ds_*), VMEM (global_/buffer_/flat_),
WAIT (s_waitcnt), BR (s_branch / s_cbranch_*)."""
import re
import sys


def blocks(path, sym):
    out, cur, on = {}, None, False
    for line in open(path):
        if line.startswith(sym + ":"):
            on, cur = True, "entry"
            out[cur] = []
            continue
        if not on:
            continue
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):", line)
        if m:
            cur = m.group(1).replace("; %", "")
            out[cur] = []
            continue
        ins = line.strip().split()
        if ins and re.match(r"^[a-z]", ins[0]):
            out[cur].append(ins[0])
            if ins[0] == "s_endpgm":
                break
    return out


def cls(op):
    if op.startswith("v_"):
        return "VALU"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    if op.startswith("s_waitcnt"):
        return "WAIT"
    if op.startswith(("s_branch", "s_cbranch")):
        return "BR"
    if op.startswith("s_nop"):
        return "NOP"
    return "SALU"


def mix(ops):
    c = {}
    for o in ops:
        k = cls(o)
        c[k] = c.get(k, 0) + 1
    return c


if __name__ == "__main__":
    B = blocks(sys.argv[1], sys.argv[2])
    sel = sys.argv[3:] or list(B)
    tot = {}
    for b in sel:
        m = mix(B.get(b, []))
        print("%-10s %4d  %s" % (b, len(B.get(b, [])), " ".join("%s=%d" % kv for kv in sorted(m.items()))))
        for k, v in m.items():
            tot[k] = tot.get(k, 0) + v
    if len(sel) > 1:
        print("sum        %4d  %s" % (sum(tot.values()), " ".join("%s=%d" % kv for kv in sorted(tot.items()))))
