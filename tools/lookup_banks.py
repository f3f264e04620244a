#!/usr/bin/env python3
"""Bank model of k_decode_fixed's table lookups: the 64
lanes of a wave each decode 64 consecutive codes of a 4,096-symbol task; a
lookup is one LDS read per lane (two 32-lane groups; bank = dword % 32; each
extra distinct dword on a bank costs one LDS cycle, identical dwords
broadcast, MI355X_MICROARCH.md §LDS). Prints LDS cycles per task for

  single : u16 entries, one code per lookup (today's table, K-bit window)
  pair   : u32 entries holding the window's first one or two codes
  triple : u64 entries (ds_read_b64, 64 banks) with up to three codes

on a synthetic Zipf(alpha) / uniform / text-like stream (numpy only; codes
are canonical Huffman codes of the sample's own counts, the same lengths as
the reference tree's).  python tools/lookup_banks.py [--alpha 1.2] [--tasks 64]
"""
import argparse
import heapq

import numpy as np


def code_lengths(counts):
    h = [(int(c), i, None) for i, c in enumerate(counts) if c > 0]
    heapq.heapify(h)
    nxt = len(counts)
    parent = {}
    while len(h) > 1:
        a, b = heapq.heappop(h), heapq.heappop(h)
        parent[a[1]] = nxt
        parent[b[1]] = nxt
        heapq.heappush(h, (a[0] + b[0], nxt, None))
        nxt += 1
    L = np.zeros(len(counts), np.int64)
    for i, c in enumerate(counts):
        if c > 0:
            d, x = 0, i
            while x in parent:
                x = parent[x]
                d += 1
            L[i] = max(d, 1)
    return L


def canonical(L):
    order = sorted((l, s) for s, l in enumerate(L) if l > 0)
    code, prev, C = 0, order[0][0], np.zeros(len(L), np.int64)
    for l, s in order:
        code <<= l - prev
        prev = l
        C[s] = code
        code += 1
    return C


def bits_of(sym, L, C):
    lens = L[sym]
    total = int(lens.sum())
    out = np.zeros(total + 64, np.uint8)
    pos = np.concatenate([[0], np.cumsum(lens)[:-1]])
    maxl = int(L.max())
    for k in range(maxl):  # bit k of each code (MSB first)
        m = lens > k
        out[pos[m] + k] = (C[sym[m]] >> (lens[m] - 1 - k)) & 1
    return out, pos


def windows(bits, K):
    w = np.zeros(len(bits) - K, np.int64)
    for k in range(K):
        w = (w << 1) | bits[k:len(bits) - K + k]
    return w


def group_cycles(addr, active, banks=32):
    """LDS cycles of one wave instruction: per 32-lane group, the most
    distinct dwords on one bank (0 when no lane of the group is active)"""
    cyc = 0
    for g in (slice(0, 32), slice(32, 64)):
        a = addr[g][active[g]]
        if a.size:
            u = np.unique(a)
            cyc += np.bincount(u % banks, minlength=banks).max()
    return cyc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--alpha", type=float, default=1.2)
    ap.add_argument("--dist", default="zipf", choices=["zipf", "uniform", "text"])
    ap.add_argument("--tasks", type=int, default=48)
    ap.add_argument("--K", type=int, default=12)
    ap.add_argument("--levels", type=int, nargs="*", default=[5, 6, 7, 8])
    ap.add_argument("--no-multi", action="store_true", help="skip the pair/triple models (slow)")
    args = ap.parse_args()
    rng = np.random.default_rng(5)
    n = args.tasks * 4096
    if args.dist == "zipf":
        p = np.arange(1, 257, dtype=np.float64) ** -args.alpha
    elif args.dist == "uniform":
        p = np.ones(256)
    else:  # English-like: ~40 frequent letters
        p = np.concatenate([np.arange(1, 41, dtype=np.float64) ** -0.9, np.full(216, 1e-5)])
    p /= p.sum()
    sym = rng.choice(256, n, p=p)
    L = code_lengths(np.bincount(sym, minlength=256))
    C = canonical(L)
    bits, pos = bits_of(sym, L, C)
    K = args.K
    win = windows(bits, 40)  # 40-bit lookahead per position
    maxl = int(L.max())
    print(f"{args.dist} alpha {args.alpha}: mean code {L[sym].mean():.2f} bits, max {maxl}, K {K}")

    def first_codes(w40, kbits, maxn):
        """codes wholly inside the first kbits of each 40-bit window (<= maxn)"""
        out = np.zeros(len(w40), np.int64)
        used = np.zeros(len(w40), np.int64)
        # decode by lengths: canonical code -> symbol via first-code table
        firsts = {}
        order = sorted((l, s) for s, l in enumerate(L) if l > 0)
        code, prev = 0, order[0][0]
        lim = {}
        for l, s in order:
            code <<= l - prev
            prev = l
            lim[l] = code  # last code of length l after loop
            code += 1
        # max code value (exclusive) per length for canonical decode
        ends = {}
        for l in range(1, maxl + 1):
            cs = [C[s] for s in range(256) if L[s] == l]
            if cs:
                ends[l] = max(cs) + 1
        for j in range(maxn):
            rem = kbits - used
            nl = np.zeros(len(w40), np.int64)
            for l in range(1, maxl + 1):
                if l not in ends:
                    continue
                top = (w40 >> (40 - used - l)) & ((1 << l) - 1)
                hit = (nl == 0) & (top < ends[l]) & (top >= (min(C[s] for s in range(256) if L[s] == l)))
                nl[hit] = l
            ok = (nl > 0) & (nl <= rem) & (used + nl <= 40)
            if j == 0:
                ok = nl > 0  # the first code always decodes (slow path beyond K, counted as one lookup)
            out += ok
            used += np.where(ok, nl, 0)
            if not ok.any():
                break
            if j == 0:
                continue
        return out, used

    res = {"single": 0, "pair": 0, "triple": 0}
    lookups = {"single": 0, "pair": 0, "triple": 0}
    for k1 in args.levels:
        res[f"2lvl{k1}"] = 0
        lookups[f"2lvl{k1}"] = 0
    for t in range(args.tasks):
        lane_pos = pos[t * 4096: (t + 1) * 4096: 64]
        # single: 64 lockstep lookups
        cur = lane_pos.copy()
        for j in range(64):
            idx = win[cur] >> (40 - K)
            res["single"] += group_cycles(idx // 2, np.ones(64, bool))
            lookups["single"] += 1
            # two levels: a 2^k1-entry u16 table first (codes <= k1 bits), the
            # K-bit table for the lanes whose code is longer (a masked read)
            clen = L[sym[t * 4096 + np.arange(64) * 64 + j]]
            # one read: lanes whose code is <= k1 bits read a 2^k1-entry region
            # after the table (indexed by the prefix, the predicate from a
            # register mask), the rest the K-bit table itself
            for k1 in args.levels:
                pre = win[cur] >> (40 - k1)
                short = clen <= k1
                dw = np.where(short, (1 << (K - 1)) + pre // 2, idx // 2)
                key = f"l1x{k1}"
                # the same inside the K-bit table: prefix j reads entry
                # (j << (K - k1)) | 2 (j & 31), any entry of its range
                alt = (pre << (K - k1)) | ((2 * pre) & ((1 << (K - k1)) - 1))
                dwi = np.where(short, alt, idx) // 2
                k2 = f"in{k1}"
                res[k2] = res.get(k2, 0) + group_cycles(dwi, np.ones(64, bool))
                lookups[k2] = lookups.get(k2, 0) + 1
                res[key] = res.get(key, 0) + group_cycles(dw, np.ones(64, bool))
                lookups[key] = lookups.get(key, 0) + 1
            for k1 in args.levels:
                i1 = win[cur] >> (40 - k1)
                res[f"2lvl{k1}"] += group_cycles(i1 // 2, np.ones(64, bool))
                longer = clen > k1
                if longer.any():
                    res[f"2lvl{k1}"] += group_cycles(idx // 2, longer)
                lookups[f"2lvl{k1}"] += 1
            cur = pos[t * 4096 + np.arange(64) * 64 + j + 1] if j < 63 else cur
        for mode, maxn, dwords in (() if args.no_multi else (("pair", 2, 1), ("triple", 3, 2))):
            got = np.zeros(64, np.int64)
            cur = lane_pos.copy()
            while (got < 64).any():
                active = got < 64
                w = win[cur]
                idx = w >> (40 - K)
                ncode, nbits = first_codes(w, K, maxn)
                ncode = np.minimum(ncode, 64 - got)
                # recompute bits for a truncated count
                take_bits = np.zeros(64, np.int64)
                for li in range(64):
                    s0 = t * 4096 + li * 64 + got[li]
                    take_bits[li] = sum(int(L[sym[s0 + q]]) for q in range(int(ncode[li])) if s0 + q < n)
                addr = idx * dwords
                if dwords == 2:  # ds_read_b64: bank = dword % 64, a lane takes banks 2i, 2i+1
                    res[mode] += group_cycles(idx, active, banks=32)
                else:
                    res[mode] += group_cycles(addr, active)
                lookups[mode] += 1
                cur = np.where(active, cur + take_bits, cur)
                got = np.where(active, got + ncode, got)
    for m in res:
        print(f"{m:7s} LDS cycles per task {res[m] / args.tasks:7.1f}  wave lookups per task {lookups[m] / args.tasks:6.1f}")


if __name__ == "__main__":
    main()
