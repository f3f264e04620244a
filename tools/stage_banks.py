"""Bank model behind kernels.hpp fixed_decode_pad: the 64 lanes of a
k_decode_fixed wave refill from the LDS stage with ds_read_b32 (two 32-lane
groups, bank = dword % 32; each extra distinct dword on a bank costs one LDS
cycle). Lane l's stream starts ~ s * l dwords into the stage (s = dwords per
64 symbols = 2 * mean code bits), jittered by the local code-length variance
(0.6 dwords per lane segment). Prints the stride bands where the swizzled
stage (dword i at i ^ ((i >> 3) & 28)) costs >= 1 cycle fewer per read than
the plain one.  python tools/stage_banks.py"""
import numpy as np

TRIALS, JITTER = 600, 0.6


def cycles(s, swz, rng):
    off = rng.uniform(0, 32, (TRIALS, 1))
    steps = rng.normal(s, JITTER, (TRIALS, 64))
    pos = np.concatenate([np.zeros((TRIALS, 1)), np.cumsum(steps, 1)[:, :-1]], 1) + off
    a = np.floor(pos).astype(np.int64)
    if swz:
        a = a ^ ((a >> 3) & 28)
    tot = 0.0
    for g in (a[:, :32], a[:, 32:]):
        for row in g:
            tot += np.bincount(np.unique(row) & 31, minlength=32).max()
    return tot / TRIALS


def main():
    rng = np.random.default_rng(7)
    band = []
    for s in np.arange(1.0, 26.01, 0.1):
        p, x = cycles(s, False, rng), cycles(s, True, rng)
        if x + 1.0 < p:
            band.append(round(float(s), 2))
        print(f"{s:5.2f} plain {p:5.2f} swizzled {x:5.2f}")
    print("swizzle wins at", band)


if __name__ == "__main__":
    main()
