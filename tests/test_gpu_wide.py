"""GPU parity of the wider-letter path: compress_with_tree /
decompress for u8 ... u128 letters through the C ABI, bit-exact against the
oracle's restatement (orc_wcompress_with_tree / orc_wdecompress, which follow
comp.rs:419-451 and 487-519 over u64 letters).

128-bit letters are checked through rank relabelling: the tree built from
(rank_i, w_i) in the same order has the same shape and leaf positions, so
the compressed stream must be identical.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# around the encoder's wide chunk (16,384 letters, one wave) and the 256-run
# decoder groups
LENGTHS = [1, 2, 7, 255, 256, 257, 4095, 16383, 16384, 16385, 65535, 65536, 65537, 65536 * 3 + 1001, 400_003]


@pytest.fixture(scope="module")
def W():
    import huff_coding.wide as W

    return W


def zipf_letters(rng, n, dtype, k=3000):
    info = np.iinfo(dtype)
    alphabet = np.unique(rng.integers(info.min, info.max, k, dtype=dtype, endpoint=True))
    p = 1.0 / np.arange(1, alphabet.size + 1) ** 1.1
    p /= p.sum()
    return alphabet[rng.choice(alphabet.size, n, p=p)]


def oracle_stream(O, letters, weights_items, lbits):
    mask = (1 << lbits) - 1
    ot = O.Tree.from_leaves([int(k) & mask for k, _ in weights_items], [int(v) for _, v in weights_items])
    u = np.asarray(letters).astype(np.int64).view(np.uint64) & np.uint64(mask) if lbits < 64 else \
        np.asarray(letters).view(np.uint64)
    return O.wcompress_with_tree(u, ot), ot


@pytest.mark.parametrize("dtype", [np.uint8, np.int16, np.uint16, np.int32, np.uint64])
def test_compress_with_tree_matches_oracle(W, O, ctx, dtype):
    rng = np.random.default_rng(np.dtype(dtype).itemsize * 7 + 1)
    lbits = 8 * np.dtype(dtype).itemsize
    for n in LENGTHS:
        letters = zipf_letters(rng, n, dtype, k=50 if dtype == np.uint8 else 3000)
        wmap = W.build_weights_map(letters, ctx)
        u, c = np.unique(letters, return_counts=True)
        assert sorted(wmap.items()) == sorted(zip(u.tolist(), c.tolist()))
        items = list(wmap.items())
        rng.shuffle(items)  # any HashMap iteration order
        t = W.WideTree.from_weights(items, dtype)
        cd = W.compress_with_tree(letters, t, ctx)
        (ocomp, opad), _ = oracle_stream(O, letters, items, lbits)
        assert cd.comp_bytes() == ocomp, (dtype, n)
        assert cd.padding_bits() == opad
        assert cd.has_index()
        back = W.decompress(cd, ctx)
        assert back.dtype == np.dtype(dtype) and np.array_equal(back, letters), (dtype, n)


@pytest.mark.parametrize("marks", ["skip", "walk"])
@pytest.mark.parametrize("dtype", [np.int16, np.uint32, np.int64])
def test_index_free_decode(W, O, ctx, dtype, marks, monkeypatch):
    """a container from to_bytes has no restart index: the self-synchronising
    decoder (run on the tree's shape) + the wide decoder from its restart
    points (k_mark_lite's boundary + codes to skip, or k_mark_lds's walked
    exact points with HUFF_WIDE_MARK_WALK=1)"""
    if marks == "walk":
        monkeypatch.setenv("HUFF_WIDE_MARK_WALK", "1")
    rng = np.random.default_rng(11)
    for n in (1, 300, 65536 + 77, 250_001):
        letters = zipf_letters(rng, n, dtype)
        cd = W.compress(letters, ctx)
        raw = cd.to_bytes()
        back_cd = W.WideCompressData.try_from_bytes(raw, dtype)
        assert not back_cd.has_index()
        got = W.decompress(back_cd, ctx)
        # the oracle's bit walk over the same bytes (comp.rs:487-519)
        ot_items = list(W.build_weights_map(letters, ctx).items())
        (ocomp, opad), ot = oracle_stream(O, letters, ot_items, 8 * np.dtype(dtype).itemsize)
        assert back_cd.comp_bytes() == ocomp
        assert np.array_equal(got, letters), (dtype, n)


@pytest.mark.parametrize("top", [1 << 20, 1 << 31], ids=["letters-in-entries", "leaf-entries"])
def test_u32_table_forms(W, O, ctx, top):
    """4-byte letters: the task decoder's entries hold the letter when every
    letter is below 2^24, else a leaf index into the letters in LDS; both
    decode the indexed and the index-free container byte-exactly"""
    rng = np.random.default_rng(top % 1000 + 3)
    alphabet = np.unique(rng.integers(0, top, 3000, dtype=np.uint32))
    p = 1.0 / np.arange(1, alphabet.size + 1) ** 1.1
    letters = alphabet[rng.choice(alphabet.size, 400_003, p=p / p.sum())]
    cd = W.compress(letters, ctx)
    assert np.array_equal(W.decompress(cd, ctx), letters)
    back_cd = W.WideCompressData.try_from_bytes(cd.to_bytes(), np.uint32)
    assert not back_cd.has_index()
    assert np.array_equal(W.decompress(back_cd, ctx), letters)


def test_u128_letters(W, O, ctx):
    rng = np.random.default_rng(5)
    base = [(1 << 127) | (int(x) << 40) | 17 for x in rng.integers(0, 1 << 60, 500)] + [0, 1, (1 << 128) - 1]
    vals = list(dict.fromkeys(base))
    for n in (1, 1000, 70_001):
        idx = np.minimum(rng.geometric(0.02, n) - 1, len(vals) - 1)
        letters = W.letters_u128([vals[i] for i in idx])
        wmap = W.build_weights_map(letters, ctx)
        u, c = np.unique(idx, return_counts=True)
        assert wmap == {vals[i]: int(k) for i, k in zip(u, c)}
        items = list(wmap.items())
        rng.shuffle(items)
        t = W.WideTree.from_weights(items, W.U128)
        cd = W.compress_with_tree(letters, t, ctx)
        rank = {v: r for r, v in enumerate(vals)}
        ot = O.Tree.from_leaves([rank[k] for k, _ in items], [w for _, w in items])
        ocomp, opad = O.wcompress_with_tree(np.asarray([rank[vals[i]] for i in idx], np.uint64), ot)
        assert cd.comp_bytes() == ocomp and cd.padding_bits() == opad
        back = W.decompress(cd, ctx)
        assert back.tobytes() == letters.tobytes()
        # index-free
        back2 = W.decompress(W.WideCompressData.try_from_bytes(cd.to_bytes(), W.U128), ctx)
        assert back2.tobytes() == letters.tobytes()


def test_u128_letters_with_colliding_folds(W, O, ctx):
    """16-byte letters fold to lo ^ hi * C before hashing; eight letters
    with (hi, lo) = (i, i * C mod 2^64) all fold to 0, so no table size
    separates them: the table build re-seeds the fold (wtree.cpp) instead
    of growing without bound, and the codes stay those of the reference"""
    C = 0xC2B2AE3D27D4EB4F
    vals = [(i << 64) | ((i * C) & ((1 << 64) - 1)) for i in range(8)] + [12345, 1 << 100]
    rng = np.random.default_rng(8)
    idx = rng.integers(0, len(vals), 50_001)
    letters = W.letters_u128([vals[i] for i in idx])
    wmap = W.build_weights_map(letters, ctx)
    items = list(wmap.items())
    t = W.WideTree.from_weights(items, W.U128)
    cd = W.compress_with_tree(letters, t, ctx)
    rank = {v: r for r, v in enumerate(vals)}
    ot = O.Tree.from_leaves([rank[k] for k, _ in items], [w for _, w in items])
    ocomp, opad = O.wcompress_with_tree(np.asarray([rank[vals[i]] for i in idx], np.uint64), ot)
    assert cd.comp_bytes() == ocomp and cd.padding_bits() == opad
    assert W.decompress(cd, ctx).tobytes() == letters.tobytes()


def test_missing_letter_first_in_input_order(W, ctx):
    """comp.rs:426-432: CompressError for the first letter without a code"""
    import huff_coding as H

    t = W.WideTree.from_weights({10: 3, 20: 2, 30: 1}, np.int32)
    letters = np.array([10, 20] * 40000 + [-5, 30, 99], np.int32)
    with pytest.raises(H.CompressError) as e:
        W.compress_with_tree(letters, t, ctx)
    assert e.value.missing_letter == (-5) & 0xFFFFFFFF or e.value.missing_letter == -5
    assert "letter not found in codes" in str(e.value)


def test_single_letter_and_empty(W, ctx):
    import huff_coding as H

    letters = np.full(100_000, -12, np.int32)
    cd = W.compress(letters, ctx)
    assert cd.huff_tree().read_codes() == {-12: "0"}
    assert cd.comp_bytes() == bytes(12500) and cd.padding_bits() == 0
    assert np.array_equal(W.decompress(cd, ctx), letters)
    back = W.decompress(W.WideCompressData.try_from_bytes(cd.to_bytes(), np.int32), ctx)
    assert np.array_equal(back, letters)
    with pytest.raises(H.HuffPanic):  # from_weights of no letters panics first
        W.compress(np.zeros(0, np.int32), ctx)
    t = W.WideTree.from_weights({1: 1}, np.int32)
    with pytest.raises(H.HuffPanic):  # no bytes: CompressData::new panics
        W.compress_with_tree(np.zeros(0, np.int32), t, ctx)


@pytest.mark.parametrize("dtype", [np.uint8, np.uint16, np.int32, np.uint64])
def test_long_codes(W, O, ctx, dtype):
    """Fibonacci weights give codes up to 39 bits: u64 table values (the
    > 32-bit split in the packer) and the secondary tables in the decoder;
    the index-free decoder refuses them (> 32 bits) with CODE_TOO_LONG"""
    import huff_coding as H

    fib = [1, 1]
    while len(fib) < 40:
        fib.append(fib[-1] + fib[-2])
    items = [(100 + i, f) for i, f in enumerate(fib)]
    t = W.WideTree.from_weights(items, dtype)
    assert max(len(c) for c in t.read_codes().values()) == 39
    rng = np.random.default_rng(9)
    letters = (100 + rng.integers(0, 40, 300_000)).astype(dtype)
    cd = W.compress_with_tree(letters, t, ctx)
    (ocomp, opad), _ = oracle_stream(O, letters, items, 8 * np.dtype(dtype).itemsize)
    assert cd.comp_bytes() == ocomp and cd.padding_bits() == opad
    assert np.array_equal(W.decompress(cd, ctx), letters)
    with pytest.raises(H.HuffError) as e:
        W.decompress(W.WideCompressData.try_from_bytes(cd.to_bytes(), dtype), ctx)
    assert e.value.code == 7


@pytest.mark.parametrize("dtype", [np.uint8, np.int16, np.uint32, np.int64])
def test_codes_17_to_32_bits(W, O, ctx, dtype):
    """Fibonacci weights over 25 letters: codes up to 24 bits, so the task
    decoder refills before every code and takes level-2 entries (wdecode.hip);
    restart-index and index-free decode"""
    fib = [1, 1]
    while len(fib) < 25:
        fib.append(fib[-1] + fib[-2])
    items = [(3 + 5 * i, f) for i, f in enumerate(fib)]
    t = W.WideTree.from_weights(items, dtype)
    assert max(len(c) for c in t.read_codes().values()) == 24
    rng = np.random.default_rng(17)
    p = np.array(fib, np.float64) ** 0.5  # flatter than the weights: long codes are frequent
    letters = (3 + 5 * rng.choice(25, 300_001, p=p / p.sum())).astype(dtype)
    cd = W.compress_with_tree(letters, t, ctx)
    (ocomp, opad), _ = oracle_stream(O, letters, items, 8 * np.dtype(dtype).itemsize)
    assert cd.comp_bytes() == ocomp and cd.padding_bits() == opad
    assert np.array_equal(W.decompress(cd, ctx), letters)
    back = W.decompress(W.WideCompressData.try_from_bytes(cd.to_bytes(), dtype), ctx)
    assert np.array_equal(back, letters)


@pytest.mark.parametrize("dtype,k", [(np.uint32, 40_000), (np.uint16, 65536), (np.uint64, 20_000)])
def test_large_alphabet_table_in_hbm(W, O, ctx, dtype, k):
    """alphabets whose code table exceeds the LDS budget (kWideLdsMax):
    the encoder reads the table from L2; every u16 letter present (the
    table's empty slot key 0 is a real letter)"""
    rng = np.random.default_rng(k)
    if dtype == np.uint16:
        letters = np.concatenate([np.arange(65536, dtype=np.uint16), rng.integers(0, 65536, 200_000, dtype=np.uint16)])
        rng.shuffle(letters)
    else:
        letters = zipf_letters(rng, 300_001, dtype, k=k)
        letters[:k // 4] = np.arange(k // 4, dtype=dtype)  # 0 and other small keys
    wmap = W.build_weights_map(letters, ctx)
    items = list(wmap.items())
    t = W.WideTree.from_weights(items, dtype)
    cd = W.compress_with_tree(letters, t, ctx)
    (ocomp, opad), _ = oracle_stream(O, letters, items, 8 * np.dtype(dtype).itemsize)
    assert cd.comp_bytes() == ocomp and cd.padding_bits() == opad
    assert np.array_equal(W.decompress(cd, ctx), letters)


@pytest.mark.parametrize("dtype", [np.uint32, np.uint64, "u128"])
def test_weights_map_table_growth(W, ctx, dtype):
    """build_weights_map's HBM table starts at 2^20 slots (claims up to 3/4)
    and grows when the kernel reports it full: 1.2 M distinct letters force
    one growth; a large input over 10 letters never does (the round-3 table
    took 2 n slots whatever the alphabet). Counts equal numpy's, ascending."""
    rng = np.random.default_rng(41)
    for distinct, n in ((1_200_000, 3_000_001), (10, 8_000_001)):
        if dtype == "u128":
            keys = np.unique(rng.integers(0, 2**63, (distinct * 2, 2), dtype=np.uint64), axis=0)[:distinct]
            pairs = np.ascontiguousarray(keys[rng.integers(0, keys.shape[0], n)])  # (lo, hi) per letter
            wmap = W.build_weights_map(pairs.view(np.dtype("V16")).reshape(-1), ctx)
            u, c = np.unique(pairs[:, ::-1], axis=0, return_counts=True)  # ascending (hi, lo)
            want_keys = [int(lo) | (int(hi) << 64) for hi, lo in u]
        else:
            alphabet = np.unique(rng.integers(0, np.iinfo(dtype).max, distinct * 2, dtype=dtype))[:distinct]
            letters = alphabet[rng.integers(0, alphabet.size, n)]
            wmap = W.build_weights_map(letters, ctx)
            u, c = np.unique(letters, return_counts=True)
            want_keys = [int(x) for x in u]
        assert list(wmap.keys()) == want_keys
        assert list(wmap.values()) == [int(x) for x in c]


@pytest.mark.parametrize("dtype", [np.uint8, np.uint16, np.int32, np.int64])
def test_device_pack_any_alignment(W, O, ctx, dtype):
    """pass 2 into an output at every offset mod 16: the bytes equal the
    oracle's stream, and no byte outside [off, off + ceil(bits / 8)) changes"""
    import torch

    rng = np.random.default_rng(np.dtype(dtype).itemsize)
    n = 3 * 16384 + 77
    letters = zipf_letters(rng, n, dtype, k=200 if dtype == np.uint8 else 3000)
    items = list(W.build_weights_map(letters, ctx).items())
    t = W.WideTree.from_weights(items, dtype)
    (ocomp, opad), _ = oracle_stream(O, letters, items, 8 * np.dtype(dtype).itemsize)
    x = torch.from_numpy(letters.copy()).cuda()
    job = W.WideEncodeJob(ctx, np.dtype(dtype).itemsize, x.data_ptr(), n)
    bits = job.bits(t)
    nb = (bits + 7) // 8
    assert nb == len(ocomp)
    for off in (0, 1, 3, 4, 8, 13, 15):
        buf = torch.full((nb + 64,), 0xAB, dtype=torch.uint8, device="cuda")
        assert job.pack(t, buf.data_ptr() + off, nb) == bits
        got = buf.cpu().numpy()
        assert got[off:off + nb].tobytes() == ocomp, off
        assert (got[:off] == 0xAB).all() and (got[off + nb:] == 0xAB).all(), off
    # the restart-index decoder into a misaligned destination
    out = torch.empty(nb + 64, dtype=torch.uint8, device="cuda")
    job.pack(t, out.data_ptr(), nb)
    w = np.dtype(dtype).itemsize
    for off in (w, 16 + w):
        dec = torch.full((n * w + 64,), 0xCD, dtype=torch.uint8, device="cuda")
        job.decode(t, out.data_ptr(), dec.data_ptr() + off)
        got = dec.cpu().numpy()
        assert got[off:off + n * w].tobytes() == letters.tobytes(), off
        assert (got[:off] == 0xCD).all() and (got[off + n * w:] == 0xCD).all(), off
    # a stream packed at an odd offset decodes in place (the runtime copies a
    # misaligned stream to an aligned buffer): restart index and index-free
    for off in (1, 3, 13):
        buf = torch.zeros(nb + 64, dtype=torch.uint8, device="cuda")
        job.pack(t, buf.data_ptr() + off, nb)
        dec = torch.empty(n * w + 64, dtype=torch.uint8, device="cuda")
        job.decode(t, buf.data_ptr() + off, dec.data_ptr())
        torch.cuda.synchronize()
        assert dec[: n * w].cpu().numpy().tobytes() == letters.tobytes(), off
        dec.zero_()
        got_n = W.decompress_dev(ctx, t, buf.data_ptr() + off, nb, opad, dec.data_ptr(), n)
        torch.cuda.synchronize()
        assert got_n == n and dec[: n * w].cpu().numpy().tobytes() == letters.tobytes(), off


def test_device_job_large(W, ctx):
    """HBM-resident job: 64 Mi u16 letters, bits = sum of code lengths, pack,
    restart-index decode and index-free decode round trips"""
    import torch

    n = 64 << 20
    g = torch.Generator(device="cuda").manual_seed(3)
    # a skewed u16 alphabet: low byte uniform, high byte geometric-ish
    hi = torch.clamp(torch.empty(n, device="cuda").exponential_(0.7, generator=g).long(), max=255)
    lo = torch.randint(0, 256, (n,), device="cuda", generator=g)
    x = ((hi << 8) | lo).to(torch.int32).to(torch.int16)
    xs = x.cpu().numpy().view(np.uint16)
    u, c = np.unique(xs, return_counts=True)
    t = W.WideTree.from_weights(list(zip(u.tolist(), c.tolist())), np.uint16)
    letters, code, ln = t.code_table()
    lens = np.zeros(65536, np.uint64)
    lens[letters.astype(np.int64)] = ln
    want_bits = int((c.astype(np.uint64) * lens[u.astype(np.int64)]).sum())
    job = W.WideEncodeJob(ctx, 2, x.data_ptr(), n)
    assert job.bits(t) == want_bits
    out = torch.empty((want_bits + 31) // 32 * 4 + 16, dtype=torch.uint8, device="cuda")
    assert job.pack(t, out.data_ptr(), out.numel()) == want_bits
    dec = torch.empty(n, dtype=torch.int16, device="cuda")
    job.decode(t, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dec, x)
    dec.zero_()
    nb = (want_bits + 7) // 8
    cnt = W.decompress_dev(ctx, t, out.data_ptr(), nb, (8 - want_bits % 8) % 8, dec.data_ptr(), n)
    torch.cuda.synchronize()
    assert cnt == n and torch.equal(dec, x)


def test_index_free_dense_slow_windows(W, O, ctx, monkeypatch):
    """codes of 11-16 bits over 4,096 letters, with ~10 % of the 12-bit walk
    table's windows slow: the sync kernels' branch-free dense steps (a
    level-2 length read at every step, no refills), and with HUFF_L2_SPARSE=1
    the branching steps; both decode the index-free container exactly"""
    rng = np.random.default_rng(43)
    k = 4096
    w = np.where(np.arange(k) < 2048, 8.0, 1.0)
    letters = rng.choice(k, 400_003, p=w / w.sum()).astype(np.int16)
    u, c = np.unique(letters, return_counts=True)
    codes = O.Tree.from_leaves([int(x) for x in u], [int(x) for x in c]).codes(k)
    lens = [len(s) for s in codes.values()]
    assert 12 < max(lens) <= 16
    assert len({s[:12] for s in codes.values() if len(s) > 12}) * 64 > 1 << 12
    cd = W.compress(letters, ctx)
    raw = cd.to_bytes()
    for sparse in (False, True):
        if sparse:
            monkeypatch.setenv("HUFF_L2_SPARSE", "1")
        back_cd = W.WideCompressData.try_from_bytes(raw, np.int16)
        assert not back_cd.has_index()
        assert np.array_equal(W.decompress(back_cd, ctx), letters), sparse


def test_index_free_capacity_below_count(W, O, ctx):
    """ADVICE r5, the wide index-free path: a letter capacity below the
    decoded count fails with HUFF_E_BUFFER_TOO_SMALL and the true count,
    writes nothing past the capacity, and the same context then decodes the
    stream with a large enough buffer"""
    import ctypes as C

    import torch
    from huff_coding import _lib

    rng = np.random.default_rng(97)
    letters = zipf_letters(rng, 300_007, np.int16)
    cd = W.compress(letters, ctx)
    raw = cd.to_bytes()
    back_cd = W.WideCompressData.try_from_bytes(raw, np.int16)
    comp = np.frombuffer(back_cd.comp_bytes(), np.uint8)
    pad = back_cd.padding_bits()
    t = back_cd.huff_tree()
    n = letters.size
    dc = torch.from_numpy(np.concatenate([comp, np.zeros(64, np.uint8)])).cuda()
    out = torch.full((n + 2048,), 0x5A5A, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    L = _lib.load()
    for cap in (n - 1, n // 3, 65):
        out.fill_(0x5A5A)  # (the one-pass decoder writes the letters that fit)
        torch.cuda.synchronize()
        got = C.c_size_t()
        rc = L.huff_dev_wdecompress(ctx.h, t.h, C.c_void_p(dc.data_ptr()), comp.size, pad,
                                    C.c_void_p(out.data_ptr()), cap, C.byref(got))
        torch.cuda.synchronize()
        assert rc == _lib.E_BUFFER_TOO_SMALL and got.value == n, (cap, rc, got.value)
        res = out.cpu().numpy()
        assert (res[cap:] == 0x5A5A).all(), f"capacity {cap}: wrote past the buffer"
    assert W.decompress_dev(ctx, t, dc.data_ptr(), comp.size, pad, out.data_ptr(), n) == n
    torch.cuda.synchronize()
    res = out.cpu().numpy()
    assert np.array_equal(res[:n], letters)
    assert (res[n:] == 0x5A5A).all()
