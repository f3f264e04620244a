"""GPU parity: the HIP path through the C ABI vs the oracle, bit-exact.

Small/medium inputs are compared byte-for-byte with the faithful restatement;
BASELINE-sized inputs (1 GiB) with the oracle's table-driven checker (itself
checked against the faithful one in test_oracle_golden.py) and through
size-independent properties (encode -> decode round trip, weights sum = n).
"""
import hashlib
import os
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 15, 16, 17, 255, 4095, 4096, 4097, 65535, 65536, 65537, 131072 + 333, 1_000_003]


def oracle_bytes(O, data):
    t = O.Tree.from_weights(O.weights_from_bytes(data))
    comp, pad = O.compress_with_tree(data, t)
    return O.to_bytes(comp, pad, t), comp, pad, t


def inputs(rng):
    yield "pinned-abbccc", b"abbccc"
    yield "single", b"a"
    yield "zero-only", bytes([0])
    yield "zero-no255", bytes([0, 1, 1, 2, 0, 9])
    yield "all-256", bytes(range(256)) * 3
    for n in SIZES:
        yield f"uniform-{n}", rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    for n in (100, 70_000, 500_000):
        yield f"skew-{n}", np.minimum(rng.geometric(0.3, n), 255).astype(np.uint8).tobytes()
        yield f"two-{n}", rng.integers(0, 2, n, dtype=np.uint8).tobytes()
        yield f"const-{n}", bytes([7]) * n


def test_weights_from_bytes(H, O, ctx):
    rng = np.random.default_rng(1)
    for name, data in inputs(rng):
        g = H.ByteWeights.from_bytes(data, ctx)
        o = O.weights_from_bytes(data)
        assert (g.as_array() == o.as_array()).all(), name
        assert g.len() == o.len, name
    assert H.ByteWeights.from_bytes(b"", ctx).is_empty()


def test_pass1_repeated_and_ragged(H, O, ctx, monkeypatch):
    """pass 1 (k_hist1 + k_rows_sum + publish) run several times on one job
    and on ragged lengths: every run equals the oracle's counts, and a pack
    over the per-chunk rows is byte-exact (the rows set chunk_start)"""
    import torch
    from huff_coding import device as D

    monkeypatch.setenv("HUFF_DISABLE_FIXED8", "1")
    for n, kind, seed in [(3 * 65536 * 257 + 4095, "zipf", 11), (65536 * 5 + 1, "text", 12), (777, "uniform", 13),
                          (65536, "uniform", 14)]:
        x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        D.generate(ctx, kind, seed, x.data_ptr(), n, cdf=D.zipf_cdf(1.2) if kind == "zipf" else None)
        host = x[:n].cpu().numpy()
        want = O.fast_hist(host, 8)
        job = H.EncodeJob(ctx, x.data_ptr(), n)
        for _ in range(3):
            assert (job.hist() == want).all(), (n, kind)
        tree = H.HuffTree.from_weights(H.ByteWeights.from_array(want))
        bits = job.bits(tree)
        out = torch.zeros((bits + 7) // 8 + 64, dtype=torch.uint8, device="cuda")
        assert job.pack(tree, out.data_ptr(), out.numel()) == bits
        code, ln = O.Tree.from_weights(O.weights_from_array(want)).code_table()
        ref, rbits = O.fast_encode(host, code, ln, threads=8)
        assert rbits == bits and (out[: (bits + 7) // 8].cpu().numpy() == ref).all(), (n, kind)


def test_threaded_weights(H, O, ctx):
    rng = np.random.default_rng(2)
    cases = [bytes([0, 1] * 12), bytes([0, 1] * 5000), rng.integers(0, 200, 100_003, dtype=np.uint8).tobytes(),
             b"aaaaa", rng.integers(0, 256, 12 * 65536 + 5, dtype=np.uint8).tobytes()]
    for data in cases:
        for T in (1, 3, 12, 100):
            g = H.ByteWeights.threaded_from_bytes(data, T, ctx)
            o = O.weights_threaded(data, T)
            assert (g.as_array() == o.as_array()).all(), (len(data), T)
            assert g.len() == o.len


def test_compress_matches_oracle(H, O, ctx):
    rng = np.random.default_rng(3)
    for name, data in inputs(rng):
        want, comp, pad, _ = oracle_bytes(O, data)
        cd = H.compress(data, ctx)
        assert cd.comp_bytes() == comp, name
        assert cd.padding_bits() == pad, name
        assert cd.to_bytes() == want, name
        assert H.decompress(cd, ctx) == data, name
        # without the restart index (as read from bytes): index-free decode
        cd2 = H.CompressData.try_from_bytes(want)
        assert not cd2.has_index()
        assert H.decompress(cd2, ctx) == data, name


def test_pinned_and_derived_vectors(H, ctx, golden):
    pinned, derived = golden
    for c in pinned["to_bytes"]:
        cd = H.compress(c["input_ascii"].encode(), ctx)
        assert cd.to_bytes().hex() == c["hex"]
    for c in derived["small"] + derived["survey_crosscheck"]:
        data = bytes.fromhex(c["input_hex"])
        assert H.compress(data, ctx).to_bytes().hex() == c["to_bytes"]
    for c in pinned["roundtrips"]:
        data = c["input_ascii"].encode()
        assert H.decompress(H.compress(data, ctx), ctx) == data


def test_long_codes(H, O, ctx):
    """Fibonacci weights: codes past the 27-bit short-table limit (u64 path)"""
    f = [1, 1]
    while len(f) < 44:
        f.append(f[-1] + f[-2])
    rng = np.random.default_rng(4)
    # a buffer whose histogram is Fibonacci-shaped would be huge; instead give
    # the tree explicitly and encode bytes drawn from its letters
    w = np.zeros(256, np.uint64)
    letters = rng.choice(256, 44, replace=False)
    w[letters] = f
    t = H.HuffTree.from_weights(H.ByteWeights.from_array(w))
    ot = O.Tree.from_weights(O.weights_from_array(w))
    assert max(len(v) for v in t.read_codes().values()) > 32
    data = rng.choice(letters, 300_001).astype(np.uint8).tobytes()
    cd = H.compress_with_tree(data, t, ctx)
    comp, pad = O.compress_with_tree(data, ot)
    assert cd.comp_bytes() == comp and cd.padding_bits() == pad
    assert H.decompress(cd, ctx) == data
    assert H.decompress(H.CompressData.try_from_bytes(cd.to_bytes()), ctx) == data


def _fib_tree(H, O, nletters, seed):
    f = [1, 1]
    while len(f) < nletters:
        f.append(f[-1] + f[-2])
    rng = np.random.default_rng(seed)
    w = np.zeros(256, np.uint64)
    # letter 0 left out: its iterator quirk double-counts a
    # weight and the tree is no longer a chain
    letters = rng.choice(np.arange(1, 256), nletters, replace=False)
    w[letters] = np.array(f, dtype=np.uint64)
    return (H.HuffTree.from_weights(H.ByteWeights.from_array(w)), O.Tree.from_weights(O.weights_from_array(w)),
            letters, rng)


@pytest.mark.parametrize("nletters", [62, 75])
def test_deep_codes(H, O, ctx, nletters):
    """codes longer than 57 bits (deep.hip): 62 Fibonacci-weighted letters
    give 61-bit codes, 75 give 74-bit codes (past u64; the weights stay
    below 2^53, exact in every representation); the reference encodes
    any depth (tree_inner.rs:422-440, comp.rs:419-451). Byte-exact against the
    bit-serial oracle through the host API, the index-free decoder of a
    to_bytes container, and the device job (restart index decode)"""
    import torch

    t, ot, letters, rng = _fib_tree(H, O, nletters, 40 + nletters)
    maxlen = max(len(v) for v in ot.codes().values())
    assert maxlen > 57
    # mostly the deep letters, so every round of the packer meets long codes
    deep_letters = [k for k, v in ot.codes().items() if len(v) > 40]
    data = np.where(rng.random(200_003) < 0.5, rng.choice(deep_letters, 200_003),
                    rng.choice(letters, 200_003)).astype(np.uint8).tobytes()
    cd = H.compress_with_tree(data, t, ctx)
    comp, pad = O.compress_with_tree(data, ot)
    assert cd.comp_bytes() == comp and cd.padding_bits() == pad
    assert H.decompress(cd, ctx) == data
    assert H.decompress(H.CompressData.try_from_bytes(cd.to_bytes()), ctx) == data
    assert cd.to_bytes() == O.to_bytes(comp, pad, ot)
    # the device job at a non-zero bit base with the previous letters' tail
    n = len(data)
    x = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).cuda()
    seg = torch.empty(n - 1000 + 64, dtype=torch.uint8, device="cuda")
    seg[: n - 1000] = x[1000:]
    job = H.EncodeJob(ctx, seg.data_ptr(), n - 1000)
    job.hist()
    base = int(sum(len(ot.codes()[b]) for b in data[:1000]))
    bits = job.bits(t)
    out = torch.zeros((base % 8 + bits + 7) // 8 + 64, dtype=torch.uint8, device="cuda")
    job.pack(t, out.data_ptr(), out.numel(), bit_base=base, prev_tail=data[992:1000])
    dec = torch.empty(n - 1000 + 64, dtype=torch.uint8, device="cuda")
    job.decode(t, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    assert dec[: n - 1000].cpu().numpy().tobytes() == data[1000:]
    got = out[: (base % 8 + bits + 7) // 8].cpu().numpy().tobytes()
    assert got == comp[base // 8:]


def test_missing_letter(H, ctx):
    t = H.HuffTree.from_weights(H.ByteWeights.from_bytes(b"abb", ctx))
    with pytest.raises(H.CompressError) as e:
        H.compress_with_tree(b"abbccc", t, ctx)
    assert e.value.missing_letter == ord("c")
    rng = np.random.default_rng(5)
    data = rng.integers(0, 10, 200_000, dtype=np.uint8)
    data[150_000] = 77
    data[199_000] = 66
    t = H.HuffTree.from_weights(H.ByteWeights.from_array(np.bincount(data[:100_000], minlength=256)))
    with pytest.raises(H.CompressError) as e:
        H.compress_with_tree(data.tobytes(), t, ctx)
    assert e.value.missing_letter == 77  # the first missing letter in input order


def test_empty_inputs(H, ctx):
    with pytest.raises(H.HuffPanic, match="empty weights"):
        H.compress(b"", ctx)
    t = H.HuffTree.from_weights(H.ByteWeights.from_bytes(b"ab", ctx))
    with pytest.raises(H.HuffPanic, match="comp_bytes are empty"):
        H.compress_with_tree(b"", t, ctx)


def test_decompress_foreign_streams(H, O, ctx):
    """index-free decode of oracle-made streams, incl. odd padding, incomplete
    final codes and single-leaf trees"""
    rng = np.random.default_rng(6)
    for n in (1, 3, 100, 4099, 70_001, 400_000):
        for hi in (1, 2, 3, 9, 256):
            data = rng.integers(0, hi, n, dtype=np.uint8).tobytes()
            raw, comp, pad, t = oracle_bytes(O, data)
            assert H.decompress(H.CompressData.try_from_bytes(raw), ctx) == O.decompress(comp, pad, t)
    # arbitrary (non-encoder) payload bytes with an arbitrary padding: whatever
    # the tree walk yields, incomplete last code dropped
    t = O.Tree.from_weights(O.weights_from_bytes(b"abracadabra alakazam"))
    for n in (1, 2, 7, 300, 5000):
        payload = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for pad in (0, 3, 7):
            raw = O.to_bytes(payload, pad, t)
            assert H.decompress(H.CompressData.try_from_bytes(raw), ctx) == O.decompress(payload, pad, t)


def test_dev_decompress_foreign_streams(H, O, ctx):
    """huff_dev_decompress: device-resident streams written by the CPU
    restatement (no restart index), incl. paddings, single-letter trees,
    garbage payloads and the count-only query"""
    import torch
    from huff_coding import device as D

    rng = np.random.default_rng(13)
    cases = []
    for n in (1, 5, 1000, 65536 * 3 + 17, 700_001):
        for hi in (1, 3, 40, 256):
            cases.append(rng.integers(0, hi, n, dtype=np.uint8).tobytes())
    cases.append(np.minimum(rng.geometric(0.2, 300_000), 255).astype(np.uint8).tobytes())
    # equal counts of 8 / 64 letters: every code 3 / 6 bits, so the segment
    # length (a multiple of the lengths' gcd near 992 bits) is clamped below
    # the sample words' 1024-bit limit (indexless_sync)
    for k in (8, 64):
        cases.append(rng.permutation(np.tile(np.arange(1, k + 1, dtype=np.uint8), 400_000 // k)).tobytes())
    for data in cases:
        t = O.Tree.from_weights(O.weights_from_bytes(data))
        comp, pad = O.compress_with_tree(data, t)
        want = O.decompress(comp, pad, t)
        tree = H.HuffTree.try_from_bin(t.as_bin())
        dc = torch.zeros(len(comp) + 64, dtype=torch.uint8, device="cuda")
        dc[: len(comp)] = torch.frombuffer(bytearray(comp), dtype=torch.uint8).cuda()
        assert D.decompress_dev(ctx, tree, dc.data_ptr(), len(comp), pad, 0, 0) == len(want)
        out = torch.empty(len(want) + 64, dtype=torch.uint8, device="cuda")
        got = D.decompress_dev(ctx, tree, dc.data_ptr(), len(comp), pad, out.data_ptr(), len(want))
        torch.cuda.synchronize()
        assert got == len(want) and out[:got].cpu().numpy().tobytes() == want
    t = O.Tree.from_weights(O.weights_from_bytes(b"abracadabra alakazam"))
    tree = H.HuffTree.try_from_bin(t.as_bin())
    for n in (3, 999):
        payload = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for pad in (0, 5):
            want = O.decompress(payload, pad, t)
            dc = torch.frombuffer(bytearray(payload + bytes(64)), dtype=torch.uint8).cuda()
            out = torch.empty(len(want) + 64, dtype=torch.uint8, device="cuda")
            got = D.decompress_dev(ctx, tree, dc.data_ptr(), n, pad, out.data_ptr(), len(want) + 64)
            torch.cuda.synchronize()
            assert out[:got].cpu().numpy().tobytes() == want


@pytest.mark.parametrize("l2", [True, False], ids=["l2-lds", "l2-global"])
def test_dev_decompress_codes_past_table(H, O, ctx, l2, monkeypatch):
    """index-free decode of streams whose codes pass the 12-bit table (13-30
    bits): the sync kernels' level-2 length table in LDS, and with
    HUFF_NO_L2=1 the global secondary tables; both byte-exact vs the oracle"""
    import torch
    from huff_coding import device as D

    if not l2:
        monkeypatch.setenv("HUFF_NO_L2", "1")
    rng = np.random.default_rng(29)
    cases = [np.minimum(rng.geometric(p, n), 255).astype(np.uint8).tobytes()
             for p, n in ((0.08, 2_000_000), (0.2, 700_001), (0.35, 65536 * 5 + 3))]
    # 24 letters with Fibonacci-like counts: codes up to 23 bits
    fib = [1, 1]
    while len(fib) < 24:
        fib.append(fib[-1] + fib[-2])
    letters = np.repeat(np.arange(24, dtype=np.uint8), np.array(fib) * 3)
    cases.append(rng.permutation(letters).tobytes())
    for data in cases:
        t = O.Tree.from_weights(O.weights_from_bytes(data))
        comp, pad = O.compress_with_tree(data, t)
        want = O.decompress(comp, pad, t)
        tree = H.HuffTree.try_from_bin(t.as_bin())
        dc = torch.zeros(len(comp) + 64, dtype=torch.uint8, device="cuda")
        dc[: len(comp)] = torch.frombuffer(bytearray(comp), dtype=torch.uint8).cuda()
        out = torch.empty(len(want) + 64, dtype=torch.uint8, device="cuda")
        got = D.decompress_dev(ctx, tree, dc.data_ptr(), len(comp), pad, out.data_ptr(), len(want))
        torch.cuda.synchronize()
        assert got == len(want) and out[:got].cpu().numpy().tobytes() == want


def _device_gen(H, ctx, kind, seed, n):
    import torch
    from huff_coding import device as D

    x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    D.generate(ctx, kind, seed, x.data_ptr(), n, cdf=D.zipf_cdf(1.2) if kind == "zipf" else None)
    return x


@pytest.mark.parametrize("dec", ["auto", "10", "11"], ids=["dec-auto", "dec-fixed", "dec-checked"])
@pytest.mark.parametrize("kind,seed", [("uniform", 0x5EED0001), ("zipf", 0x5EED0002), ("text", 0x5EED0005)])
def test_device_job_medium(H, O, ctx, kind, seed, dec, monkeypatch):
    """16 MiB + ragged tail of each workload; decode through the kernel the
    runtime picks, the general decoder forced (HUFF_DEC_VARIANT=10 with the
    byte map off) and its self-checking build (11)"""
    import torch

    forced = dec != "auto"
    if forced:
        monkeypatch.setenv("HUFF_DEC_VARIANT", dec)
        monkeypatch.setenv("HUFF_DISABLE_FIXED8", "1")

    n = (1 << 24) + 12345  # 16 MiB + a ragged tail
    x = _device_gen(H, ctx, kind, seed, n)
    host = x[:n].cpu().numpy()
    gen = {"uniform": O.gen_uniform, "zipf": O.gen_zipf, "text": O.gen_text}[kind]
    assert (host == gen(seed, n)).all(), "device generator != oracle generator"
    job = H.EncodeJob(ctx, x.data_ptr(), n)
    w = job.hist()
    assert (w == O.fast_hist(host, 8)).all()
    tree = H.HuffTree.from_weights(H.ByteWeights.from_array(w))
    ot = O.Tree.from_weights(O.weights_from_array(w))
    assert tree.as_bin() == ot.as_bin()
    bits = job.bits(tree)
    out = torch.zeros((bits + 7) // 8 + 64, dtype=torch.uint8, device="cuda")
    assert job.pack(tree, out.data_ptr(), out.numel()) == bits
    torch.cuda.synchronize()
    code, ln = ot.code_table()
    want, wbits = O.fast_encode(host, code, ln, threads=8)
    got = out[: (bits + 7) // 8].cpu().numpy()
    assert wbits == bits and (got == want).all()
    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    job.decode(tree, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dec[:n], x[:n])
    if not forced:
        # a misaligned output (a tensor view at an odd offset): decoded into the
        # context's aligned buffer and copied; the bytes around it untouched
        dec.fill_(0xA5)
        job.decode(tree, out.data_ptr(), dec.data_ptr() + 3)
        torch.cuda.synchronize()
        assert torch.equal(dec[3:3 + n], x[:n])
        assert (dec[:3] == 0xA5).all() and (dec[3 + n:] == 0xA5).all()


def test_indexfree_misaligned_output(H, O, ctx):
    """huff_dev_decompress into an output pointer that is not 16-B aligned:
    the fixed-count decoder runs into an aligned buffer, then one copy"""
    import torch
    from huff_coding import device as D

    n = (1 << 22) + 77
    x = _device_gen(H, ctx, "zipf", 61, n)
    host = x[:n].cpu().numpy()
    w = O.fast_hist(host, 8)
    ot = O.Tree.from_weights(O.weights_from_array(w))
    tree = H.HuffTree.from_weights(H.ByteWeights.from_array(w))
    code, ln = ot.code_table()
    comp, bits = O.fast_encode(host, code, ln, threads=8)
    dc = torch.from_numpy(np.concatenate([comp, np.zeros(64, np.uint8)])).cuda()
    out = torch.full((n + 128,), 0x5A, dtype=torch.uint8, device="cuda")
    got = D.decompress_dev(ctx, tree, dc.data_ptr(), len(comp), (8 - bits % 8) % 8, out.data_ptr() + 5, n + 64)
    torch.cuda.synchronize()
    assert got == n
    assert torch.equal(out[5:5 + n], x[:n])
    assert (out[:5] == 0x5A).all() and (out[5 + n:] == 0x5A).all()
    # a stream at an odd address (copied to an aligned buffer first)
    dc2 = torch.zeros(len(comp) + 64, dtype=torch.uint8, device="cuda")
    dc2[3:3 + len(comp)] = dc[:len(comp)]
    out.fill_(0)
    got = D.decompress_dev(ctx, tree, dc2.data_ptr() + 3, len(comp), (8 - bits % 8) % 8, out.data_ptr(), n + 64)
    torch.cuda.synchronize()
    assert got == n and torch.equal(out[:n], x[:n])


@pytest.mark.parametrize("dec", ["auto", "11"], ids=["dec-auto", "dec-checked"])
def test_device_job_long_tail_codes(H, O, ctx, dec, monkeypatch):
    """geometric bytes: codes from 1 to > 12 bits (the multi-symbol table's
    slow path); production and the self-checking build"""
    import torch

    if dec != "auto":
        monkeypatch.setenv("HUFF_DEC_VARIANT", dec)
    rng = np.random.default_rng(77)
    n = (1 << 22) + 999
    host = np.minimum(rng.geometric(0.45, n) - 1, 255).astype(np.uint8)
    host[rng.integers(0, n, 3000)] = rng.integers(0, 256, 3000, dtype=np.uint8)  # rare letters: long codes
    x = torch.from_numpy(np.concatenate([host, np.zeros(64, np.uint8)])).cuda()
    job = H.EncodeJob(ctx, x.data_ptr(), n)
    w = job.hist()
    tree = H.HuffTree.from_weights(H.ByteWeights.from_array(w))
    _, ln = tree.code_table()
    assert ln.max() > 12
    bits = job.bits(tree)
    out = torch.zeros((bits + 7) // 8 + 64, dtype=torch.uint8, device="cuda")
    assert job.pack(tree, out.data_ptr(), out.numel()) == bits
    ot = O.Tree.from_weights(O.weights_from_array(w))
    code, oln = ot.code_table()
    want, wbits = O.fast_encode(host, code, oln, threads=8)
    torch.cuda.synchronize()
    assert wbits == bits and (out[: (bits + 7) // 8].cpu().numpy() == want).all()
    dec_t = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    job.decode(tree, out.data_ptr(), dec_t.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dec_t[:n], x[:n])


@pytest.mark.parametrize("small", ["1", "0"], ids=["small-stage", "large-stage"])
def test_decode_stage_overflow(H, O, ctx, small, monkeypatch):
    """a stream whose mean code length picks the decoders' 3 KiB stage
    (<= 5.6 bits per symbol) but with a stretch of ~8-bit codes: those tasks
    exceed the stage and decode from global memory. Indexed decode and the
    index-free decode (the skip build), against the input and the oracle's
    stream; and with HUFF_SMALL_STAGE=0 (the 4.5 KiB stage)."""
    import torch
    from huff_coding import device as D

    monkeypatch.setenv("HUFF_SMALL_STAGE", small)
    rng = np.random.default_rng(404)
    n = (1 << 22) + 4321
    host = np.minimum(rng.geometric(0.5, n) - 1, 255).astype(np.uint8)  # ~2 bits per symbol
    host[n // 3: n // 3 + 300_000] = rng.integers(0, 256, 300_000, dtype=np.uint8)  # a dense stretch
    x = torch.from_numpy(np.concatenate([host, np.zeros(64, np.uint8)])).cuda()
    job = H.EncodeJob(ctx, x.data_ptr(), n)
    w = job.hist()
    tree = H.HuffTree.from_weights(H.ByteWeights.from_array(w))
    bits = job.bits(tree)
    assert bits / n <= 5.6  # the small stage is chosen when enabled
    ot = O.Tree.from_weights(O.weights_from_array(w))
    code, ln = ot.code_table()
    assert ln[host[n // 3: n // 3 + 300_000]].mean() > 6  # the stretch's tasks exceed 3 KiB
    out = torch.zeros((bits + 7) // 8 + 64, dtype=torch.uint8, device="cuda")
    assert job.pack(tree, out.data_ptr(), out.numel()) == bits
    want, wbits = O.fast_encode(host, code, ln, threads=8)
    torch.cuda.synchronize()
    assert wbits == bits and (out[: (bits + 7) // 8].cpu().numpy() == want).all()
    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    job.decode(tree, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dec[:n], x[:n])
    dec.fill_(0)
    got = D.decompress_dev(ctx, tree, out.data_ptr(), (bits + 7) // 8, (8 - bits % 8) % 8, dec.data_ptr(), n + 64)
    torch.cuda.synchronize()
    assert got == n and torch.equal(dec[:n], x[:n])


@pytest.mark.parametrize("general", [False, True], ids=["fixed8", "general"])
def test_device_job_full_size_uniform(H, O, ctx, general, monkeypatch):
    """BASELINE config 2: 1 GiB uniform, bit-exact vs the checker + round trip.
    Every code is 8 bits here, so the byte-map kernel runs unless
    HUFF_DISABLE_FIXED8 forces the general pack/decode kernels."""
    import torch

    if general:
        monkeypatch.setenv("HUFF_DISABLE_FIXED8", "1")
    n = 1 << 30
    x = _device_gen(H, ctx, "uniform", 0x5EED0001, n)
    job = H.EncodeJob(ctx, x.data_ptr(), n)
    w = job.hist()
    assert int(w.sum()) == n
    tree = H.HuffTree.from_weights(H.ByteWeights.from_array(w))
    assert set(len(v) for v in tree.read_codes().values()) == {8}
    bits = job.bits(tree)
    assert bits == 8 * n
    out = torch.zeros(bits // 8 + 64, dtype=torch.uint8, device="cuda")
    job.pack(tree, out.data_ptr(), out.numel())
    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    job.decode(tree, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dec[:n], x[:n])
    host = x[:n].cpu().numpy()
    ot = O.Tree.from_weights(O.weights_from_array(w))
    code, ln = ot.code_table()
    want, _ = O.fast_encode(host, code, ln, threads=16)
    got = out[: n].cpu().numpy()
    assert hashlib.sha256(got.tobytes()).digest() == hashlib.sha256(want.tobytes()).digest()


def test_device_job_full_size_zipf(H, O, ctx):
    """BASELINE config 3: 1 GiB Zipf(1.2), encode + decode, bit-exact"""
    import torch

    n = 1 << 30
    x = _device_gen(H, ctx, "zipf", 0x5EED0002, n)
    job = H.EncodeJob(ctx, x.data_ptr(), n)
    w = job.hist()
    host = x[:n].cpu().numpy()
    # pass 1 on skewed bytes against an independent host count (the oracle
    # tree below is built from these weights, so a miscount would otherwise
    # be self-consistent)
    assert (w == O.fast_hist(host, 16)).all()
    tree = H.HuffTree.from_weights(H.ByteWeights.from_array(w))
    bits = job.bits(tree)
    assert 5.2 < bits / n < 5.4
    out = torch.zeros((bits + 7) // 8 + 64, dtype=torch.uint8, device="cuda")
    job.pack(tree, out.data_ptr(), out.numel())
    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    job.decode(tree, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dec[:n], x[:n])
    ot = O.Tree.from_weights(O.weights_from_array(w))
    code, ln = ot.code_table()
    want, wb = O.fast_encode(host, code, ln, threads=16)
    assert wb == bits
    got = out[: (bits + 7) // 8].cpu().numpy()
    assert (got == want).all()


def test_shard_stitching_on_one_gpu(H, O, ctx):
    """the multi-GPU data path (bit_base + prev_tail) on one device: shards
    encoded independently concatenate to the single-stream bytes"""
    import torch

    rng = np.random.default_rng(8)
    n = 3_000_017
    data = np.minimum(rng.geometric(0.2, n), 255).astype(np.uint8)
    x = torch.from_numpy(data).cuda()
    w = np.bincount(data, minlength=256).astype(np.uint64)
    tree = H.HuffTree.from_weights(H.ByteWeights.from_array(w))
    ot = O.Tree.from_weights(O.weights_from_array(w))
    code, ln = ot.code_table()
    want, total = O.fast_encode(data, code, ln, threads=8)
    bounds = [0, 1_000_003, 1_000_003 + 65536 * 7 + 5, n]
    pieces = []
    base = 0
    for r in range(3):
        lo, hi = bounds[r], bounds[r + 1]
        seg = torch.empty(hi - lo + 64, dtype=torch.uint8, device="cuda")
        seg[: hi - lo] = x[lo:hi]  # 16-B aligned copy of the shard
        job = H.EncodeJob(ctx, seg.data_ptr(), hi - lo)
        job.hist()
        bits = job.bits(tree)
        out = torch.zeros((base % 8 + bits + 7) // 8 + 64, dtype=torch.uint8, device="cuda")
        tail = data[max(0, lo - 8):lo].tobytes()
        job.pack(tree, out.data_ptr(), out.numel(), bit_base=base, prev_tail=tail)
        torch.cuda.synchronize()
        nbytes = (base % 8 + bits + 7) // 8
        own = out[:nbytes].cpu().numpy()
        # global bytes [base/8, (base+bits)/8) are this shard's; the last shard
        # also owns its zero-padded final byte
        keep = nbytes if r == 2 else (base % 8 + bits) // 8
        pieces.append(own[:keep])
        # each shard decodes its own symbols from its local stream
        dec = torch.empty(hi - lo + 64, dtype=torch.uint8, device="cuda")
        job.decode(tree, out.data_ptr(), dec.data_ptr())
        torch.cuda.synchronize()
        assert (dec[: hi - lo].cpu().numpy() == data[lo:hi]).all()
        base += bits
    got = np.concatenate(pieces)
    assert base == total and got.size == want.size and (got == want).all()


def test_back_to_back_jobs_different_trees(H, O, ctx):
    """several encode/decode jobs with different trees queued on one context
    without host synchronisation in between: the decode tables (uploaded on a
    side stream while the pack runs) must never be overwritten under a decode
    that still reads them"""
    import torch

    rng = np.random.default_rng(12)
    n = 3 * 65536 + 777
    datas = [np.minimum(rng.geometric(p, n), 255).astype(np.uint8) for p in (0.05, 0.3, 0.6, 0.12)]
    datas.append(rng.integers(0, 256, n, dtype=np.uint8))  # all-8-bit codes: byte map
    xs, outs, decs, jobs, trees = [], [], [], [], []
    for d in datas:
        x = torch.from_numpy(d).cuda()
        xs.append(x)
        job = H.EncodeJob(ctx, x.data_ptr(), n)
        jobs.append(job)
    # pass 1 for all (host waits for weights), then pass 2 + decode for all, no sync
    hists = [job.hist() for job in jobs]
    for job, w in zip(jobs, hists):
        out = torch.zeros(2 * n + 128, dtype=torch.uint8, device="cuda")
        tree, _, bits = job.pack_shards(w[None, :], 0, [b""], out.data_ptr(), out.numel())
        dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        job.decode(tree, out.data_ptr(), dec.data_ptr())
        outs.append((out, bits))
        decs.append(dec)
        trees.append(tree)
    torch.cuda.synchronize()
    for d, (out, bits), dec, w in zip(datas, outs, decs, hists):
        ot = O.Tree.from_weights(O.weights_from_array(w))
        code, ln = ot.code_table()
        want, wb = O.fast_encode(d, code, ln, threads=4)
        assert wb == bits
        assert (out[: (bits + 7) // 8].cpu().numpy() == want).all()
        assert (dec[:n].cpu().numpy() == d).all()


def test_pack_shards_on_one_gpu(H, O, ctx):
    """huff_enc_pack_shards (native tree + bit base + tail, then pack) for 4
    shards, one of them shorter than 8 bytes: the owned bytes concatenate to
    the single-stream compress_with_tree bytes"""
    import torch

    from huff_coding import mgpu

    rng = np.random.default_rng(11)
    n = 2_500_003
    data = np.minimum(rng.geometric(0.15, n), 255).astype(np.uint8)
    x = torch.from_numpy(data).cuda()
    bounds = [0, 900_001, 900_004, 1_700_000, n]
    world = len(bounds) - 1
    jobs, segs, hists, tails = [], [], [], []
    for r in range(world):
        lo, hi = bounds[r], bounds[r + 1]
        seg = torch.empty(hi - lo + 64, dtype=torch.uint8, device="cuda")
        seg[: hi - lo] = x[lo:hi]
        job = H.EncodeJob(ctx, seg.data_ptr(), hi - lo)
        hists.append(job.hist())
        tails.append(data[lo:hi][-8:].tobytes())
        jobs.append(job)
        segs.append(seg)
    hists = np.stack(hists)
    w = np.bincount(data, minlength=256).astype(np.uint64)
    ot = O.Tree.from_weights(O.weights_from_array(w))
    code, ln = ot.code_table()
    want, total = O.fast_encode(data, code, ln, threads=8)
    pieces, base_expect = [], 0
    for r in range(world):
        lo, hi = bounds[r], bounds[r + 1]
        cap = (hi - lo) * 2 + 128
        out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
        tree, base, bits = jobs[r].pack_shards(hists, r, tails, out.data_ptr(), cap)
        assert tree.as_bin() == ot.as_bin()
        assert base == base_expect
        torch.cuda.synchronize()
        pieces.append(mgpu.owned_bytes(out.cpu().numpy(), base, bits, r == world - 1))
        dec = torch.empty(hi - lo + 64, dtype=torch.uint8, device="cuda")
        jobs[r].decode(tree, out.data_ptr(), dec.data_ptr())
        torch.cuda.synchronize()
        assert (dec[: hi - lo].cpu().numpy() == data[lo:hi]).all()
        base_expect += bits
    got = np.concatenate(pieces)
    assert base_expect == total and got.size == want.size and (got == want).all()
    # a short buffer reports the bits it needs
    small = torch.zeros(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(H.HuffError) as ei:
        jobs[0].pack_shards(hists, 0, tails, small.data_ptr(), 64)
    assert ei.value.bits_needed == int(hists[0].astype(np.uint64) @ ln.astype(np.uint64))


def test_file_path_matches_cli(H, O, ctx, golden):
    rng = np.random.default_rng(9)
    with tempfile.TemporaryDirectory() as d:
        srcs = [O.gen_text(11, 3000), O.gen_text(12, 777), rng.integers(0, 256, 5000, dtype=np.uint8),
                np.array([0, 1] * 40 + [3] * 9, np.uint8), O.gen_text(99, 300_000)]
        for k, src in enumerate(srcs):
            src = bytes(src)
            p = os.path.join(d, f"f{k}")
            open(p, "wb").write(src)
            for bs in (len(src) + 10, len(src), 1000, 64, 37, 65536):
                want = O.cli_compress(src, bs)
                H.read_compress_write(p, p + ".hff", bs, ctx)
                got = open(p + ".hff", "rb").read()
                assert got == want, (k, bs)
                try:
                    want_dec = O.cli_decompress(want, bs)
                except O.OracleError as e:
                    with pytest.raises(H.CliError) as ex:
                        H.read_decompress_write(p + ".hff", p + ".out", bs, ctx)
                    assert ex.value.code == e.code
                    continue
                H.read_decompress_write(p + ".hff", p + ".out", bs, ctx)
                assert open(p + ".out", "rb").read() == want_dec, (k, bs)
        # header errors (huff/src/comp.rs:95-144)
        bad = os.path.join(d, "bad.hff")
        for blob, code in ((b"\x00\x00", 11), (b"\x80\x00\x00\x00\x02\xff\xff", 12),
                           (b"\x00\x00\x00\x00\x09\xff", 11), (b"\x00\x00\x00\x00\x02\xff\xff\x00", 12)):
            open(bad, "wb").write(blob)
            with pytest.raises(H.CliError) as ex:
                H.read_decompress_write(bad, bad + ".out", 2_000_000_000, ctx)
            assert ex.value.code == code
        empty = os.path.join(d, "empty")
        open(empty, "wb").close()
        with pytest.raises(H.HuffPanic, match="empty weights"):
            H.read_compress_write(empty, empty + ".hff", 100, ctx)


@pytest.mark.parametrize("window,piece", [(256, 4096), (1000, 5000), (4099, 65536), (65536, 1 << 20)])
def test_file_path_windows(H, O, ctx, window, piece, monkeypatch):
    """the streamed .hff path (filepath.cpp): HUFF_FILE_PIECE shrinks the
    compress pieces (a block split into pieces that pack at their bit offset
    with the previous piece's tail; pass-1 rows per ration share) and
    HUFF_FILE_WINDOW the decompress windows, so a file crosses many windows,
    each ending inside a code (carried to the next window, realigned when it
    starts inside a byte). Multi-block files (the bug-compatible stitching)
    and a tree deeper than 57 bits (deep pack, serial deep walk) included;
    outputs equal the oracle's CLI compress / decompress
    (huff/src/comp.rs:32-283)"""
    monkeypatch.setenv("HUFF_FILE_WINDOW", str(window))
    monkeypatch.setenv("HUFF_FILE_PIECE", str(piece))
    _, _, letters, rng = _fib_tree(H, O, 70, 7)
    deep = rng.choice(letters, 40_000).astype(np.uint8)
    with tempfile.TemporaryDirectory() as d:
        cases = [(O.gen_text(21, 200_000), 200_000 + 5), (O.gen_zipf(22, 150_000), 150_000),
                 (O.gen_text(23, 90_000), 7_000), (deep, 40_000)]
        for k, (src, bs) in enumerate(cases):
            src = bytes(src)
            p = os.path.join(d, f"w{k}")
            open(p, "wb").write(src)
            H.read_compress_write(p, p + ".hff", bs, ctx)
            blob = open(p + ".hff", "rb").read()
            assert blob == O.cli_compress(src, bs), k
            H.read_decompress_write(p + ".hff", p + ".out", bs, ctx)
            assert open(p + ".out", "rb").read() == O.cli_decompress(blob, bs), (k, window)


def test_file_path_large(H, O, ctx):
    """a 40 MiB file: pieces and windows of the default 64 MiB, reads and
    writes split over the I/O threads (>= 16 MiB), -b 2G (one block) and
    -b 10Mi (four stitched blocks, several pieces); byte-equal to the
    oracle's CLI compress and decompress"""
    src = O.gen_zipf(5, 40 << 20)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "big")
        src.tofile(p)
        src = src.tobytes()
        for bs in (2_000_000_000, 10 << 20):
            H.read_compress_write(p, p + ".hff", bs, ctx)
            blob = open(p + ".hff", "rb").read()
            assert blob == O.cli_compress(src, bs), bs
            H.read_decompress_write(p + ".hff", p + ".out", bs, ctx)
            got = open(p + ".out", "rb").read()
            assert got == (src if bs > len(src) else O.cli_decompress(blob, bs)), bs


def test_hist_row_and_device_exchange(H, O, ctx):
    """the sharded pass 1 without a host round trip: huff_enc_hist_row's
    device row (weights | tail bytes | count) equals the oracle, and the
    RCCL path (DeviceExchange: row -> all_gather_into_tensor -> pinned copy,
    a world-1 process group here) feeds huff_enc_pack_shards to the same bytes
    as the single-GPU encode"""
    import torch
    import torch.distributed as dist
    from huff_coding import device as D
    from huff_coding import mgpu

    row = torch.empty(258, dtype=torch.int64, device="cuda")
    for n in (0, 5, 65536 * 3 + 7, (1 << 22) + 12345):
        x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        if n:
            D.generate(ctx, "zipf", 21 + n, x.data_ptr(), n, cdf=D.zipf_cdf(1.2))
        host = x[:n].cpu().numpy()
        job = H.EncodeJob(ctx, x.data_ptr(), n)
        job.hist_row(row.data_ptr())
        torch.cuda.synchronize()
        hists, tails = mgpu.rows_to_hists(row.cpu().numpy()[None, :])
        assert (hists[0] == (O.fast_hist(host, 8) if n else 0)).all(), n
        assert tails[0] == host[-8:].tobytes(), n

    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29541")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        n = (1 << 23) + 333
        x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        D.generate(ctx, "text", 5, x.data_ptr(), n)
        host = x[:n].cpu().numpy()
        job = H.EncodeJob(ctx, x.data_ptr(), n)
        ctx.set_stream(torch.cuda.current_stream().cuda_stream)
        dx = mgpu.DeviceExchange(torch.device("cuda", 0))
        out = torch.zeros(n + 128, dtype=torch.uint8, device="cuda")
        for _ in range(2):
            hists, tails = dx(job)
            tree, base, bits = job.pack_shards(hists, 0, tails, out.data_ptr(), out.numel())
            torch.cuda.synchronize()
            code, ln = O.Tree.from_weights(O.weights_from_array(O.fast_hist(host, 8))).code_table()
            want, wbits = O.fast_encode(host, code, ln, threads=8)
            assert base == 0 and bits == wbits
            assert (out[: (bits + 7) // 8].cpu().numpy() == want).all()
            dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
            job.decode(tree, out.data_ptr(), dec.data_ptr())
            torch.cuda.synchronize()
            assert torch.equal(dec[:n], x[:n])
    finally:
        dist.destroy_process_group()


def test_enc_compress_one_call(H, O, ctx):
    """huff_enc_compress (pass 1 + tree + pass 2 in one native call) equals
    the oracle's compress_with_tree(from_weights(from_bytes)) bytes, grows
    on BUFFER_TOO_SMALL with the bits needed, and round-trips"""
    import torch
    from huff_coding import device as D

    for n, kind in [(1, "uniform"), (4097, "zipf"), ((1 << 22) + 77, "text"), ((1 << 22) + 5, "uniform")]:
        x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        D.generate(ctx, kind, 31 + n, x.data_ptr(), n, cdf=D.zipf_cdf(1.2) if kind == "zipf" else None)
        host = x[:n].cpu().numpy()
        job = H.EncodeJob(ctx, x.data_ptr(), n)
        small = torch.zeros(16, dtype=torch.uint8, device="cuda")
        if n > 64:
            with pytest.raises(H.HuffError) as e:
                job.compress(small.data_ptr(), small.numel())
            need = (e.value.bits_needed + 7) // 8
        else:
            need = n + 16
        out = torch.zeros(need + 64, dtype=torch.uint8, device="cuda")
        tree, bits = job.compress(out.data_ptr(), out.numel())
        torch.cuda.synchronize()
        ot = O.Tree.from_weights(O.weights_from_array(O.fast_hist(host, 8)))
        assert tree.as_bin() == ot.as_bin()
        code, ln = ot.code_table()
        want, wbits = O.fast_encode(host, code, ln, threads=8)
        assert bits == wbits and (out[: (bits + 7) // 8].cpu().numpy() == want).all(), (n, kind)
        dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        job.decode(tree, out.data_ptr(), dec.data_ptr())
        torch.cuda.synchronize()
        assert torch.equal(dec[:n], x[:n])


@pytest.mark.parametrize("kind", ["uniform", "zipf", "text"])
def test_pipelined_steps(H, O, ctx, kind):
    """bench.py's software pipeline: each step's pass 1 is queued between the
    previous step's pack and decode (huff_enc_hist_launch). Every compress
    and decode equals the serial one, bit for bit, and the oracle's bytes"""
    import torch
    from huff_coding import device as D

    n = (1 << 22) + 77
    x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    D.generate(ctx, kind, 7 + n, x.data_ptr(), n, cdf=D.zipf_cdf(1.2) if kind == "zipf" else None)
    host = x[:n].cpu().numpy()
    ot = O.Tree.from_weights(O.weights_from_array(O.fast_hist(host, 8)))
    code, ln = ot.code_table()
    want, wbits = O.fast_encode(host, code, ln, threads=8)
    job = H.EncodeJob(ctx, x.data_ptr(), n)
    out = torch.zeros(n + 128, dtype=torch.uint8, device="cuda")
    dec = torch.zeros(n + 64, dtype=torch.uint8, device="cuda")
    steps = 4
    for i in range(steps):
        out.zero_()
        dec.zero_()
        tree, bits = job.compress(out.data_ptr(), out.numel())
        if i + 1 < steps:
            job.hist_launch()
            job.hist_launch()  # a second launch while one is pending is a no-op
        job.decode(tree, out.data_ptr(), dec.data_ptr())
        torch.cuda.synchronize()
        assert tree.as_bin() == ot.as_bin()
        assert bits == wbits and (out[: (bits + 7) // 8].cpu().numpy() == want).all(), (kind, i)
        assert torch.equal(dec[:n], x[:n]), (kind, i)


HUFF_E_STATE = 18  # include/huffgpu.h


def test_hist_launch_one_pending_per_context(H, ctx):
    """the context's pinned weights word serves one pending pass 1: another
    job's hist/compress/hist_launch fails with HUFF_E_STATE until it is
    waited for; hist() consumes it; freeing the job releases it"""
    import torch
    from huff_coding import device as D

    n = 1 << 20
    x = torch.empty(2 * n + 64, dtype=torch.uint8, device="cuda")
    D.generate(ctx, "text", 5, x.data_ptr(), 2 * n)
    a = H.EncodeJob(ctx, x.data_ptr(), n)
    b = H.EncodeJob(ctx, x.data_ptr() + n, n)
    out = torch.zeros(n + 128, dtype=torch.uint8, device="cuda")
    a.hist_launch()
    for call in (lambda: b.hist(), lambda: b.hist_launch(), lambda: b.compress(out.data_ptr(), out.numel())):
        with pytest.raises(H.HuffError) as e:
            call()
        assert e.value.code == HUFF_E_STATE and "pending" in str(e.value)
    wa = a.hist()
    assert wa.sum() == n
    assert b.hist().sum() == n  # nothing pending any more
    b.hist_launch()
    b.close()  # huff_enc_free with its pass 1 pending
    assert a.hist().sum() == n


def test_bytemap_pack_then_bit_decoder(H, O, ctx, monkeypatch):
    """the byte-map pack leaves its arithmetic restart index unwritten; a
    decode through the bit decoders (fixed-8 disabled after the pack) must
    write it first and still return the input"""
    import torch
    from huff_coding import device as D

    for n in ((1 << 22) + 3, 65536 * 3):
        x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        D.generate(ctx, "uniform", 91 + n, x.data_ptr(), n)
        job = H.EncodeJob(ctx, x.data_ptr(), n)
        out = torch.zeros(n + 128, dtype=torch.uint8, device="cuda")
        tree, bits = job.compress(out.data_ptr(), out.numel())
        assert bits == 8 * n
        monkeypatch.setenv("HUFF_DISABLE_FIXED8", "1")
        for var in ("10", "11"):
            monkeypatch.setenv("HUFF_DEC_VARIANT", var)
            dec = torch.zeros(n + 64, dtype=torch.uint8, device="cuda")
            job.decode(tree, out.data_ptr(), dec.data_ptr())
            torch.cuda.synchronize()
            assert torch.equal(dec[:n], x[:n]), (n, var)
        monkeypatch.delenv("HUFF_DISABLE_FIXED8")
        monkeypatch.delenv("HUFF_DEC_VARIANT")


@pytest.mark.parametrize("kind", ["zipf", "uniform"])
def test_native_comm_world1_mgpu_compress(H, O, ctx, kind):
    """huff_comm (the library's RCCL communicator) + huff_mgpu_compress through
    ctypes as a world-1 group: the same bytes, tree and decode as the
    single-GPU compress, and the owned prefix is the whole stream"""
    import torch
    from huff_coding import device as D
    from huff_coding import mgpu

    n = (1 << 24) + 777
    x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    D.generate(ctx, kind, 0x5EED0002, x.data_ptr(), n, cdf=D.zipf_cdf(1.2) if kind == "zipf" else None)
    comm = mgpu.NativeComm(ctx, 1, 0, mgpu.NativeComm.unique_id())
    assert comm.observed_world() == (1, 0)  # as RCCL reports it (ncclCommCount / ncclCommUserRank)
    job = H.EncodeJob(ctx, x.data_ptr(), n)
    out = torch.zeros(n + 128, dtype=torch.uint8, device="cuda")
    tree, base, bits, owned = comm.compress(job, out.data_ptr(), out.numel())
    assert base == 0 and owned == (bits + 7) // 8
    ref_job = H.EncodeJob(ctx, x.data_ptr(), n)
    ref = torch.zeros(n + 128, dtype=torch.uint8, device="cuda")
    rtree, rbits = ref_job.compress(ref.data_ptr(), ref.numel())
    assert tree.as_bin() == rtree.as_bin() and bits == rbits
    torch.cuda.synchronize()
    assert torch.equal(out[:owned], ref[:owned])
    host = x[:n].cpu().numpy()
    ot = O.Tree.from_weights(O.weights_from_array(O.fast_hist(host, 8)))
    code, ln = ot.code_table()
    want, wb = O.fast_encode(host, code, ln, threads=8)
    assert wb == bits and (out[:owned].cpu().numpy() == want).all()
    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    job.decode(tree, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dec[:n], x[:n])
    # a short buffer reports what it needs
    small = torch.zeros(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(H.HuffError) as ei:
        comm.compress(job, small.data_ptr(), 64)
    assert ei.value.bits_needed == bits
    # a failing rank (misaligned output) still joins the collective and
    # reports its own error
    with pytest.raises(H.HuffError) as ei:
        comm.compress(job, out.data_ptr() + 3, out.numel() - 3)
    assert "aligned" in str(ei.value)
    # bench.py's pipeline: the next compress's exchange queued between a pack
    # and its decode (huff_mgpu_exchange_launch); same bytes every step
    for i in range(3):
        out.zero_()
        dec.zero_()
        t2, b2, bits2, owned2 = comm.compress(job, out.data_ptr(), out.numel())
        if i < 2:
            comm.exchange_launch(job)
            with pytest.raises(H.HuffError) as ei:  # one pending exchange per communicator
                comm.exchange_launch(job)
            assert ei.value.code == HUFF_E_STATE
        job.decode(t2, out.data_ptr(), dec.data_ptr())
        torch.cuda.synchronize()
        assert t2.as_bin() == rtree.as_bin() and bits2 == bits and owned2 == owned
        assert (out[:owned].cpu().numpy() == want).all(), i
        assert torch.equal(dec[:n], x[:n]), i
    comm.close()


def _shallow_letters(kind, n, rng):
    if kind == "u100":  # codes of 6-7 bits
        return rng.integers(0, 100, n).astype(np.uint8)
    if kind == "u256":  # all 8 bits (the padded stage)
        return rng.integers(0, 256, n).astype(np.uint8)
    if kind == "zipf64":  # 1-8 bits
        return (rng.zipf(1.3, n) % 64).astype(np.uint8)
    if kind == "dyadic":  # 1-10 bits
        p = 2.0 ** -np.arange(1, 12)
        p[-1] = p[-2]
        return rng.choice(11, n, p=p / p.sum()).astype(np.uint8)
    return (rng.integers(0, 64, n) + rng.integers(0, 64, n)).astype(np.uint8)  # "tri": up to 12 bits


@pytest.mark.parametrize("refill", ["auto", "2"])
@pytest.mark.parametrize("kind", ["u100", "u256", "zipf64", "dyadic", "tri"])
def test_shallow_trees_lookups_per_refill(H, O, ctx, kind, refill, monkeypatch):
    """trees of <= 8 / <= 10 bits decode with 4 / 3 lookups per window refill
    (decode_wave.hip decode_fixed64's R; HUFF_DEC_REFILL=2 forces two): the
    general pack matches the oracle's stream, and the restart-index decode and
    the index-free decode (its skip build) return the input, at a ragged
    size and at one with a partial task"""
    import torch
    from huff_coding import device as D

    monkeypatch.setenv("HUFF_DISABLE_FIXED8", "1")
    if refill != "auto":
        monkeypatch.setenv("HUFF_DEC_REFILL", refill)
    rng = np.random.default_rng(len(kind) * 7 + 1)
    for n in ((1 << 22) + 77, 5000):
        host = _shallow_letters(kind, n, rng)
        w = O.fast_hist(host, 8)
        ot = O.Tree.from_weights(O.weights_from_array(w))
        code, ln = ot.code_table()
        depth = int(ln[w > 0].max())
        assert depth <= {"u100": 8, "u256": 9, "zipf64": 9, "dyadic": 10, "tri": 16}[kind]
        if kind == "dyadic":
            assert depth > 8
        x = torch.from_numpy(np.concatenate([host, np.zeros(64, np.uint8)])).cuda()
        job = H.EncodeJob(ctx, x.data_ptr(), n)
        tree = H.HuffTree.from_weights(H.ByteWeights.from_array(job.hist()))
        bits = job.bits(tree)
        out = torch.zeros((bits + 7) // 8 + 64, dtype=torch.uint8, device="cuda")
        assert job.pack(tree, out.data_ptr(), out.numel()) == bits
        want, wbits = O.fast_encode(host, code, ln, threads=8)
        torch.cuda.synchronize()
        assert wbits == bits and (out[: (bits + 7) // 8].cpu().numpy() == want).all(), (kind, n)
        dec = torch.full((n + 64,), 0xEE, dtype=torch.uint8, device="cuda")
        job.decode(tree, out.data_ptr(), dec.data_ptr())
        torch.cuda.synchronize()
        assert torch.equal(dec[:n], x[:n]), (kind, n)
        dec.fill_(0xEE)
        got = D.decompress_dev(ctx, tree, out.data_ptr(), (bits + 7) // 8, (8 - bits % 8) % 8, dec.data_ptr(), n + 64)
        torch.cuda.synchronize()
        assert got == n and torch.equal(dec[:n], x[:n]), (kind, n)
