"""GPU parity of the batched small-stream API (device-side
tree build, include/huffgpu.h huff_batch_hist / huff_batch_trees): for
>= 1,000 independent streams in one launch, the weights equal np.bincount
and every stream's tree bits (as_bin, tree_inner.rs:632-663) and codes equal
the oracle's HuffTree::from_weights (tree_inner.rs:281-320 with the exact
BinaryHeap tie order, oracle/huff_oracle.c)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _streams(rng, count):
    """varied small streams: sizes 0 .. 30,000, several distributions, and the
    shapes the tree build treats specially"""
    out = [b"", b"\x00" * 17, b"\x07" * 1000, bytes(range(256)) * 3, b"\x00\x01" * 50,
           bytes([255, 0, 255, 0, 3])]
    while len(out) < count:
        n = int(rng.integers(1, 30_000))
        kind = int(rng.integers(0, 4))
        if kind == 0:
            a = rng.integers(0, 256, n, dtype=np.uint8)
        elif kind == 1:
            k = int(rng.integers(2, 40))
            a = rng.integers(0, k, n).astype(np.uint8) * np.uint8(int(rng.integers(1, 6)))
        elif kind == 2:  # Zipf over a random byte permutation
            perm = rng.permutation(256).astype(np.uint8)
            p = 1.0 / np.arange(1, 257) ** float(rng.uniform(0.8, 2.0))
            a = perm[rng.choice(256, n, p=p / p.sum())]
        else:  # equal weights: the heap's tie order decides the tree
            k = int(rng.integers(2, 256))
            a = np.repeat(rng.choice(256, k, replace=False).astype(np.uint8), max(1, n // k))
            rng.shuffle(a)
        out.append(a.tobytes())
    return out


def test_batch_trees_match_oracle(H, O, ctx):
    import torch

    from huff_coding import batch

    rng = np.random.default_rng(2024)
    streams = _streams(rng, 1200)
    offs = np.zeros(len(streams) + 1, np.int64)
    offs[1:] = np.cumsum([len(x) for x in streams])
    data = torch.from_numpy(np.frombuffer(b"".join(streams) + b"\x00", np.uint8).copy()).cuda()
    hist = batch.batch_hist(ctx, data, torch.from_numpy(offs).cuda())
    t = batch.batch_trees(ctx, hist)
    torch.cuda.synchronize()
    h = hist.cpu().numpy()
    bits, nbits = t.tree_bits.cpu().numpy(), t.tree_nbits.cpu().numpy()
    codes, maxlen, status = t.codes.cpu().numpy(), t.max_len.cpu().numpy(), t.status.cpu().numpy()
    for s, x in enumerate(streams):
        want = np.bincount(np.frombuffer(x, np.uint8), minlength=256)
        assert np.array_equal(h[s], want), s
        if not x:
            assert status[s] == batch.E_EMPTY_WEIGHTS and nbits[s] == 0
            continue
        assert status[s] == 0, s
        ot = O.Tree.from_weights(O.weights_from_array(want))
        ob = ot.as_bin()
        assert nbits[s] == len(ob), s
        assert bits[s, : (len(ob) + 7) // 8].tobytes() == O.pack_bits(ob), s
        oc = ot.codes()
        assert maxlen[s] == max(len(c) for c in oc.values())
        got = {l: format(int(v) >> 8, "0%db" % (int(v) & 0xFF)) for l, v in enumerate(codes[s]) if v}
        assert got == oc, s


def test_batch_trees_deep_and_quirks(H, O, ctx):
    """weights given directly: Fibonacci weights (a code longer than the 56
    bits codes[] holds -> CODE_TOO_LONG with complete tree bits), byte 0 with
    and without bin 255 (weights.rs:423-441 re-yields byte 0 unless bin 255
    is the last non-zero one), one letter, 256 equal weights"""
    import torch

    from huff_coding import batch

    fib = [1, 1]
    while len(fib) < 70:
        fib.append(fib[-1] + fib[-2])
    rows = []
    r = np.zeros(256, np.int64)
    r[:70] = fib
    rows.append(r)
    r = np.zeros(256, np.int64)
    r[[0, 5, 9]] = [4, 2, 1]
    rows.append(r)  # byte 0 re-yielded (last non-zero bin is 9)
    r = np.zeros(256, np.int64)
    r[[0, 5, 255]] = [4, 2, 1]
    rows.append(r)  # no re-yield
    r = np.zeros(256, np.int64)
    r[77] = 5
    rows.append(r)
    rows.append(np.full(256, 3, np.int64))
    rows.append(np.zeros(256, np.int64))
    hist = torch.from_numpy(np.stack(rows * 200)).cuda()  # 1,200 streams
    t = batch.batch_trees(ctx, hist)
    torch.cuda.synchronize()
    bits, nbits, codes = t.tree_bits.cpu().numpy(), t.tree_nbits.cpu().numpy(), t.codes.cpu().numpy()
    status, maxlen = t.status.cpu().numpy(), t.max_len.cpu().numpy()
    for s in range(hist.shape[0]):
        w = rows[s % len(rows)]
        if not w.any():
            assert status[s] == batch.E_EMPTY_WEIGHTS
            continue
        ot = O.Tree.from_weights(O.weights_from_array(w))
        ob = ot.as_bin()
        assert nbits[s] == len(ob) and bits[s, : (len(ob) + 7) // 8].tobytes() == O.pack_bits(ob), s
        oc = ot.codes()
        assert maxlen[s] == max(len(c) for c in oc.values())
        deep = maxlen[s] > 56
        assert status[s] == (batch.E_CODE_TOO_LONG if deep else 0)
        got = {l: format(int(v) >> 8, "0%db" % (int(v) & 0xFF)) for l, v in enumerate(codes[s]) if v}
        assert got == {l: c for l, c in oc.items() if len(c) <= 56}, s


def test_batch_limits(H, O, ctx):
    """weights summing to 2^54 or more (the heap keys hold weight << 10) get
    HUFF_E_INVALID_ARG, the byte-0 re-yield counted; 2^54 - 1 still builds;
    descending offsets are refused before the launch"""
    import torch

    from huff_coding import batch

    rows = []
    r = np.zeros(256, np.int64)
    r[[3, 4]] = [1 << 53, 1 << 53]
    rows.append(r)  # exactly 2^54
    r = np.zeros(256, np.int64)
    r[[3, 4]] = [(1 << 53) - 1, 1 << 53]
    rows.append(r)  # 2^54 - 1: fine
    r = np.zeros(256, np.int64)
    r[[0, 5]] = [(1 << 53), (1 << 52)]
    rows.append(r)  # byte 0 re-yielded: 2^53 + 2^52 + 2^53 >= 2^54
    r = np.zeros(256, np.int64)
    r[7] = 1 << 60
    rows.append(r)  # one heavy letter
    hist = torch.from_numpy(np.stack(rows)).cuda()
    t = batch.batch_trees(ctx, hist)
    torch.cuda.synchronize()
    st = t.status.cpu().numpy()
    assert list(st) == [batch.E_INVALID_ARG, 0, batch.E_INVALID_ARG, batch.E_INVALID_ARG]
    ot = O.Tree.from_weights(O.weights_from_array(rows[1].astype(np.uint64)))
    assert t.tree_nbits.cpu().numpy()[1] == len(ot.as_bin())
    data = torch.zeros(100, dtype=torch.uint8, device="cuda")
    data[40:50] = 7
    # a descending pair is an empty stream, in the C API and the wrapper alike
    h = batch.batch_hist(ctx, data, torch.tensor([0, 50, 40, 60], dtype=torch.int64, device="cuda")).cpu().numpy()
    assert h[0, 0] == 40 and h[0, 7] == 10 and h[1].sum() == 0 and h[2, 0] == 10 and h[2, 7] == 10
    with pytest.raises(ValueError):
        batch.batch_hist(ctx, data, torch.tensor([0, -1], dtype=torch.int64, device="cuda"))
    with pytest.raises(ValueError):
        batch.batch_hist(ctx, data, torch.tensor([0, 101], dtype=torch.int64, device="cuda"))
