#!/usr/bin/env python3
"""Build check: no kernel of the given device objects may execute a 64-bit
VALU shift (v_lshlrev_b64 / v_lshrrev_b64 / v_ashrrev_i64) whose shift-amount
VGPR is the last of an 8-register allocation granule while the VGPR after it
lies outside the kernel's allocation.

Why: on gfx90a LLVM rewrites exactly that instruction form
(GCNHazardRecognizer::fixShift64HighRegBug) because the hardware then reads a
wrong amount; the workaround is disabled for gfx940+ (gfx950 included), and
every decoder build that decoded wrong letters on MI355X in rounds 1-2 had
that form (v71 of 72, v63 of 64, v79 of 80, v95 of 96 VGPRs) while every clean
build had none ("The 64-bit shift hazard"). So a hit fails the
build instead of shipping silent corruption.

usage: check_shift64.py [--allow REGEX] obj.o [...]
  obj.o: host objects with an embedded .hip_fatbin (hipcc -c output) or
         bare gfx950 code objects. Exit status 1 on any hit.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
SHIFT = re.compile(r"^\s*(v_lshlrev_b64|v_lshrrev_b64|v_ashrrev_i64)(?:_e64)?\s+(\S+),\s*v(\d+)\b")
LABEL = re.compile(r"^[0-9a-f]+ <(.+)>:$")


def run(*cmd):
    return subprocess.run(cmd, check=True, capture_output=True, text=True).stdout


def code_object(obj, tmp):
    """The gfx950 code object of a hipcc -c object (or obj itself)."""
    with open(obj, "rb") as f:
        if f.read(4) != b"\x7fELF":
            raise SystemExit(f"{obj}: not an ELF file")
    secs = run(f"{LLVM}/llvm-objdump", "-h", obj)
    if ".hip_fatbin" not in secs:
        return obj
    base = os.path.join(tmp, os.path.basename(obj))
    run(f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={base}.fatbin", obj, f"{base}.host")
    run(f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={base}.fatbin",
        f"--targets={TARGET}", f"--output={base}.co")
    return base + ".co"


def vgpr_counts(co):
    notes = run(f"{LLVM}/llvm-readelf", "--notes", co)
    counts, cur = {}, {}
    for line in notes.splitlines():
        m = re.match(r"^\s*-?\s*\.(name|vgpr_count|agpr_count|symbol):\s+(\S+)", line)
        if not m:
            continue
        key, val = m.groups()
        if key == "agpr_count" and line.lstrip().startswith("-"):
            cur = {}
        cur[key] = val
        if "name" in cur and "vgpr_count" in cur:
            counts[cur["name"]] = int(cur["vgpr_count"])
    return counts


def scan(co):
    counts = vgpr_counts(co)
    hits, nshift, fn = [], 0, None
    for line in run(f"{LLVM}/llvm-objdump", "-d", co).splitlines():
        m = LABEL.match(line)
        if m:
            fn = m.group(1)
            continue
        s = SHIFT.match(line)
        if not s or fn is None:
            continue
        nshift += 1
        amt = int(s.group(3))
        nv = counts.get(fn)
        if nv is None:  # a non-kernel function: no allocation of its own known
            nv = max(counts.values()) if counts else 0
        if amt % 8 == 7 and amt + 1 >= nv:
            hits.append((fn, nv, line.split("//")[0].strip()))
    return counts, nshift, hits


def main(argv):
    allow = None
    args = argv[1:]
    if args[:1] == ["--allow"]:
        allow = re.compile(args[1])
        args = args[2:]
    bad = 0
    with tempfile.TemporaryDirectory() as tmp:
        for obj in args:
            counts, nshift, hits = scan(code_object(obj, tmp))
            for fn, nv, text in hits:
                if allow and allow.search(fn):
                    print(f"{obj}: allowed (diagnostic) {fn} ({nv} VGPRs): {text}")
                    continue
                bad += 1
                print(f"{obj}: {fn} ({nv} VGPRs): {text}")
    if bad:
        print(f"check-shift64: {bad} 64-bit shift(s) with the amount in the last allocated VGPR (see DESIGN.md §3)")
        return 1
    print("check-shift64: no kernel shifts 64 bits by its last allocated VGPR")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
