#!/usr/bin/env python3
"""Static scan of gfx950 assembly for one pattern: a VALU (or other vector)
instruction overwriting the ADDRESS or DATA VGPR of a DS instruction that may
still be outstanding (issued, not yet covered by an s_waitcnt lgkmcnt).

    python tools/ds_war_scan.py <file.s> <kernel symbol substring> [...]

Outstanding DS ops retire in order: lgkmcnt(N) retires all but the newest N.
Straight-line scan per kernel (branches reset nothing; conservative enough to
rank kernels). Prints each hit with the line number and the pending DS op.
"""
import re
import sys


def vregs(op):
    """VGPR numbers named by one operand (v7, v[4:7])"""
    op = op.strip()
    m = re.match(r"^v\[(\d+):(\d+)\]$", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"^v(\d+)$", op)
    if m:
        return {int(m.group(1))}
    return set()


def scan(lines, name):
    out = []
    pending = []  # (line_no, text, {address/data vgprs})
    for no, raw in lines:
        t = raw.split(";")[0].strip()
        if not t or t.endswith(":") or t.startswith("."):
            continue
        ins = t.split()[0]
        ops = [o.strip() for o in t[len(ins):].split(",")] if len(t) > len(ins) else []
        if ins == "s_waitcnt":
            m = re.search(r"lgkmcnt\((\d+)\)", t)
            if m:
                keep = int(m.group(1))
                pending = pending[len(pending) - keep:] if keep < len(pending) else pending
                if keep == 0:
                    pending = []
            continue
        if ins.startswith("ds_"):
            srcs = set()
            dst = set()
            if ins.startswith("ds_read") or ins.startswith("ds_bpermute") or ins.startswith("ds_permute"):
                dst = vregs(ops[0]) if ops else set()
                for o in ops[1:]:
                    srcs |= vregs(o)
            else:
                for o in ops:
                    srcs |= vregs(o)
            # a write to a pending op's sources by this DS op's destination
            for pno, ptxt, psrc in pending:
                if dst & psrc:
                    out.append((no, t, pno, ptxt))
            pending.append((no, t, srcs))
            continue
        if ins.startswith("v_") and ops:
            written = vregs(ops[0])
            if ins.startswith("v_cmp") or ins.startswith("v_readlane") or ins.startswith("v_readfirstlane"):
                written = set()
            for pno, ptxt, psrc in pending:
                if written & psrc:
                    out.append((no, t, pno, ptxt))
        if (ins.startswith("global_load") or ins.startswith("buffer_load") or ins.startswith("scratch_load")) and ops:
            written = vregs(ops[0]) if "lds" not in t else set()
            for pno, ptxt, psrc in pending:
                if written & psrc:
                    out.append((no, t, pno, ptxt))
    print(f"{name}: {len(out)} overwrite(s) of a pending DS op's VGPRs")
    for no, t, pno, ptxt in out[:int(__import__("os").environ.get("DSWAR_MAX", "40"))]:
        print(f"  line {no}: {t}    <- pending line {pno}: {ptxt}")


def main():
    path = sys.argv[1]
    text = open(path).read().splitlines()
    for want in sys.argv[2:]:
        start = None
        for i, l in enumerate(text):
            if l.startswith(want + ":") and start is None:
                start = i
                break
        if start is None:
            print(f"{want}: not found")
            continue
        body = []
        for i in range(start + 1, len(text)):
            if "s_endpgm" in text[i]:
                break
            body.append((i + 1, text[i]))
        scan(body, want)


if __name__ == "__main__":
    main()
