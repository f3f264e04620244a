"""Randomised parity: many random trees and lengths through the GPU paths.

Each case draws a letter distribution (geometric, Zipf over a random subset,
a few letters, near-equal weights, Fibonacci-like counts that give deep
codes), a length from 1 byte to 1.5 MB and a seed; the bytes then go
1. through the device job (pass 1, host tree, pass 2, restart-index decode),
   byte-compared with the oracle's stream and the input, and
2. as the oracle's bare stream (what the reference writes: no restart index)
   through huff_dev_decompress.
The oracle (oracle/huff_oracle.c, the C restatement of the reference) is the
checker only. Seeds are fixed, so a failure names a reproducible case.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = 160


def _draw(rng):
    kind = rng.integers(0, 6)
    n = int(rng.choice([1, 2, 7, 63, 64, 65, 4095, 4097, 65535, 65537, 300_001, 1_500_000]))
    if kind == 0:  # geometric bytes: codes from 1 bit to > 20
        data = np.minimum(rng.geometric(rng.uniform(0.05, 0.6), n) - 1, 255)
    elif kind == 1:  # Zipf over a random subset of letters
        k = int(rng.integers(2, 257))
        letters = rng.permutation(256)[:k]
        p = 1.0 / np.arange(1, k + 1) ** rng.uniform(0.6, 1.6)
        data = letters[rng.choice(k, n, p=p / p.sum())]
    elif kind == 2:  # a few letters
        k = int(rng.integers(1, 5))
        data = rng.permutation(256)[:k][rng.integers(0, k, n)]
    elif kind == 3:  # near-equal weights (ties decide the tree shape)
        k = int(rng.integers(2, 257))
        data = rng.integers(0, k, n)
    elif kind == 4:  # Fibonacci-like counts: deep codes (<= 32 bits here)
        k = int(rng.integers(3, 30))
        f = [1, 1]
        while len(f) < k:
            f.append(f[-1] + f[-2])
        w = np.array(f, dtype=np.float64)
        data = rng.permutation(256)[:k][rng.choice(k, n, p=w / w.sum())]
    else:  # uniform bytes with one letter dominating
        data = rng.integers(0, 256, n)
        data[rng.random(n) < rng.uniform(0.5, 0.99)] = int(rng.integers(0, 256))
    return kind, data.astype(np.uint8)


@pytest.mark.parametrize("case", range(CASES))
def test_random_trees_both_decoders(H, O, ctx, case):
    import torch
    from huff_coding import device as D

    rng = np.random.default_rng(1000 + case)
    kind, host = _draw(rng)
    n = host.size
    t = O.Tree.from_weights(O.weights_from_bytes(host.tobytes()))
    comp, pad = O.compress_with_tree(host.tobytes(), t)
    tree = H.HuffTree.try_from_bin(t.as_bin())
    # 1. device job: pass 1 -> host tree -> pass 2 -> restart-index decode
    x = torch.from_numpy(np.concatenate([host, np.zeros(64, np.uint8)])).cuda()
    job = H.EncodeJob(ctx, x.data_ptr(), n)
    w = job.hist()
    jt = H.HuffTree.from_weights(H.ByteWeights.from_array(w))
    assert jt.as_bin() == t.as_bin(), (case, kind)
    bits = job.bits(jt)
    out = torch.zeros((bits + 7) // 8 + 64, dtype=torch.uint8, device="cuda")
    assert job.pack(jt, out.data_ptr(), out.numel()) == bits
    torch.cuda.synchronize()
    assert out[: (bits + 7) // 8].cpu().numpy().tobytes() == comp, (case, kind)
    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    job.decode(jt, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dec[:n], x[:n]), (case, kind)
    # 2. the bare stream (no restart index) through the index-free decoder
    dc = torch.zeros(len(comp) + 64, dtype=torch.uint8, device="cuda")
    if comp:
        dc[: len(comp)] = torch.frombuffer(bytearray(comp), dtype=torch.uint8).cuda()
    got = D.decompress_dev(ctx, tree, dc.data_ptr(), len(comp), pad, dec.data_ptr(), n + 64)
    torch.cuda.synchronize()
    assert got == n and torch.equal(dec[:n], x[:n]), (case, kind, got, n)


WIDE_DTYPES = [np.int16, np.uint16, np.int32, np.uint32, np.int64, np.uint64]


@pytest.mark.parametrize("case", range(48))
def test_random_wide_alphabets(O, ctx, case):
    """wide letters: a random dtype, alphabet (1 ... 6,000 letters, small or
    full-range values), law (Zipf, equal, Fibonacci depths) and length;
    compress_with_tree byte-equal to the oracle's stream, and both the indexed
    container and its to_bytes form (no index: the sync kernels on the tree's
    shape + skip marks) decode to the input"""
    import huff_coding.wide as W

    rng = np.random.default_rng(5000 + case)
    dtype = WIDE_DTYPES[case % len(WIDE_DTYPES)]
    info = np.iinfo(dtype)
    k = int(rng.integers(1, 6000))
    if rng.random() < 0.5:
        alphabet = np.unique(rng.integers(info.min, info.max, k, dtype=dtype, endpoint=True))
    else:  # small values (4-byte letters then sit in the decoder's table entries)
        alphabet = np.unique(rng.integers(0, min(int(info.max), 1 << 20), k).astype(dtype))
    k = alphabet.size
    law = rng.integers(0, 3)
    if law == 0:
        p = 1.0 / np.arange(1, k + 1) ** rng.uniform(0.7, 1.5)
    elif law == 1:
        p = np.ones(k)
    else:
        m = min(k, 28)
        f = [1.0, 1.0]
        while len(f) < m:
            f.append(f[-1] + f[-2])
        p = np.zeros(k)
        p[:m] = f[:m]
    n = int(rng.choice([1, 3, 64, 4097, 65537, 250_001]))
    letters = alphabet[rng.choice(k, n, p=p / p.sum())]
    wmap = W.build_weights_map(letters, ctx)
    items = list(wmap.items())
    rng.shuffle(items)  # any HashMap iteration order
    t = W.WideTree.from_weights(items, dtype)
    cd = W.compress_with_tree(letters, t, ctx)
    lbits = 8 * np.dtype(dtype).itemsize
    mask = (1 << lbits) - 1
    ot = O.Tree.from_leaves([int(a) & mask for a, _ in items], [int(v) for _, v in items])
    u = letters.astype(np.int64).view(np.uint64) & np.uint64(mask) if lbits < 64 else letters.view(np.uint64)
    ocomp, opad = O.wcompress_with_tree(u, ot)
    assert cd.comp_bytes() == ocomp and cd.padding_bits() == opad, (case, dtype, k, n)
    assert np.array_equal(W.decompress(cd, ctx), letters), (case, dtype, k, n)
    back = W.WideCompressData.try_from_bytes(cd.to_bytes(), dtype)
    assert np.array_equal(W.decompress(back, ctx), letters), (case, dtype, k, n)
