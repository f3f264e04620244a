#!/usr/bin/env python3
"""Scan gfx950 assembly (.s from `hipcc --cuda-device-only -S`, or
llvm-objdump disassembly) for 64-bit VALU shifts whose shift-amount operand
is the last VGPR of an 8-register allocation granule with the next VGPR
outside the kernel's allocation.

LLVM works around exactly this case on gfx90a (GCNHazardRecognizer::
fixShift64HighRegBug: "v_lshlrev_b64 / v_lshrrev_b64 / v_ashrrev_i64 with the
amount in v(8k+7) and v(8k+8) unallocated read a wrong amount") but does not
enable the workaround for gfx940+; this tool checks our own code objects.

usage: shift64_scan.py file.s [...]   (exit 1 when any kernel is affected)
"""
import re
import sys

SHIFT = re.compile(r"^\s*(v_lshlrev_b64|v_lshrrev_b64|v_ashrrev_i64)(?:_e64)?\s+(\S+),\s*v(\d+)\b")
FUNC = re.compile(r"^([A-Za-z_.$][\w.$]*):\s*(;.*)?$")


def scan(path):
    hits = []
    funcs = {}  # name -> (list of (line, amt), total vgprs)
    cur = None
    shifts = []
    with open(path) as f:
        lines = f.readlines()
    for ln, line in enumerate(lines, 1):
        m = FUNC.match(line)
        if m and not m.group(1).startswith(".L") and not m.group(1).startswith("$"):
            cur = m.group(1)
            funcs.setdefault(cur, {"shifts": [], "vgpr": None, "agpr": 0, "total": None})
            continue
        if cur is None:
            continue
        s = SHIFT.match(line)
        if s:
            funcs[cur]["shifts"].append((ln, int(s.group(3)), line.strip()))
            continue
        if line.startswith("\t.set ") or line.startswith(".set "):
            pass
        m2 = re.match(r"^\s*;\s*NumVgprs:\s*(\d+)", line)
        if m2:
            funcs[cur]["vgpr"] = int(m2.group(1))
        m3 = re.match(r"^\s*;\s*NumAgprs:\s*(\d+)", line)
        if m3:
            funcs[cur]["agpr"] = int(m3.group(1))
        m4 = re.match(r"^\s*;\s*TotalNumVgprs:\s*(\d+)", line)
        if m4:
            funcs[cur]["total"] = int(m4.group(1))
    for name, d in funcs.items():
        total = d["total"] if d["total"] is not None else d["vgpr"]
        if total is None:
            continue
        alloc = (total + 7) // 8 * 8
        for ln, amt, text in d["shifts"]:
            if amt % 8 == 7 and amt + 1 >= alloc:
                hits.append((name, ln, amt, total, text))
    return funcs, hits


def main(argv):
    bad = False
    for p in argv[1:]:
        funcs, hits = scan(p)
        nshift = sum(len(d["shifts"]) for d in funcs.values())
        print(f"{p}: {len(funcs)} functions, {nshift} 64-bit shifts, {len(hits)} with the amount in the last allocated VGPR")
        for name, ln, amt, total, text in hits:
            bad = True
            print(f"  {name} (VGPRs {total}) line {ln}: {text}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
