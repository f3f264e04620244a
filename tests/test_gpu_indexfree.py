"""The index-free decoder (indexless.hip + the fixed-count decoder's skip
build) against the oracle.

Streams are written by the CPU restatement (oracle/, comp.rs:419-451) with no
restart index, as the reference writes every CompressData and .hff payload,
and decoded on the device through huff_dev_decompress (comp.rs:487-519): the
speculative pass, the fix-up, the scan, the marks and the decoder.
The cases cover lanes merging with their speculative walk, codes longer than
the 12-bit table (level-2 table in LDS and the global one), heavily skewed
bytes (~1 bit per letter: many codes to skip per mark), slowly
resynchronising codes (the fix-up rounds), tiny and ragged streams,
misaligned outputs, the count-only query, garbage payloads, equality with
the self-checking build (HUFF_DEC_VARIANT=11: exact walked marks), and the
BASELINE-size streams. (Until round 4 these cases drove the opt-in split
decoder, isplit.hip, measured slower and removed in round 5; git history.)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def roundtrip(H, O, ctx, data, misalign=0):
    """oracle-encode `data`, decode it on the device, compare byte for byte
    and check that nothing past the letters was written"""
    import torch
    from huff_coding import device as D

    t = O.Tree.from_weights(O.weights_from_bytes(data))
    code, ln = t.code_table()
    host = np.frombuffer(data, np.uint8)
    comp, bits = O.fast_encode(host, code, ln, threads=8)
    pad = (8 - bits % 8) % 8
    tree = H.HuffTree.try_from_bin(t.as_bin())
    dc = torch.zeros(comp.size + 64, dtype=torch.uint8, device="cuda")
    if comp.size:
        dc[: comp.size] = torch.from_numpy(comp).cuda()
    torch.cuda.synchronize()
    n = len(data)
    assert D.decompress_dev(ctx, tree, dc.data_ptr(), comp.size, pad, 0, 0) == n
    out = torch.full((n + 80,), 0xAB, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the library runs on its own stream
    got = D.decompress_dev(ctx, tree, dc.data_ptr() if comp.size else 0, comp.size, pad,
                           out.data_ptr() + misalign, n + 16)
    torch.cuda.synchronize()
    assert got == n
    res = out.cpu().numpy()
    bad = np.nonzero(res[misalign: misalign + n] != host)[0]
    assert bad.size == 0, (bad[:10], bad.size)
    assert (res[misalign + n:] == 0xAB).all(), "wrote past the letters"
    return comp, pad, tree


def index_free_cases(O, rng):
    yield "zipf-16MiB", O.gen_zipf(0x5EED0002, (1 << 24) + 12345).tobytes()
    yield "text-16MiB", O.gen_text(0x5EED0005, (1 << 24) + 999).tobytes()
    yield "uniform40", rng.integers(0, 40, 3_000_001, dtype=np.uint8).tobytes()
    yield "geometric-long", np.minimum(rng.geometric(0.45, 2_000_003) - 1, 255).astype(np.uint8).tobytes()
    x = np.minimum(rng.geometric(0.45, 1_000_000) - 1, 255).astype(np.uint8)
    x[rng.integers(0, x.size, 3000)] = rng.integers(0, 256, 3000, dtype=np.uint8)  # codes > 12 bits
    yield "long-codes", x.tobytes()
    skew = np.where(rng.random(2_000_000) < 0.95, 0, rng.integers(1, 200, 2_000_000)).astype(np.uint8)
    yield "skewed-95", skew.tobytes()  # ~1.3 bits per letter: long skips between samples
    skew = np.where(rng.random(1_500_000) < 0.995, 7, rng.integers(0, 3, 1_500_000)).astype(np.uint8)
    yield "skewed-99.5", skew.tobytes()  # ~1 bit per letter
    runs = np.repeat(rng.integers(0, 6, 40_000, dtype=np.uint8), rng.integers(1, 300, 40_000))
    yield "runs", runs.tobytes()
    for n in (1, 2, 3, 63, 64, 65, 255, 256, 1000, 4095, 65537):
        yield f"small-{n}", rng.integers(0, 7, n, dtype=np.uint8).tobytes()
    yield "two-letters", rng.integers(0, 2, 100_001, dtype=np.uint8).tobytes()
    # near-fixed lengths {7, 8} (160 letters, equal weights) and {5, 6}:
    # resynchronise slowly, so many lanes leave their segment unmerged
    yield "lengths-7-8", rng.integers(0, 160, 2_000_001, dtype=np.uint8).tobytes()
    yield "lengths-5-6", rng.integers(0, 40, 2_000_001, dtype=np.uint8).tobytes()
    # equal counts of 8 / 64 letters: all codes 3 / 6 bits (gcd 3: S = 1023 - ...)
    for k in (8, 64):
        yield f"fixed-{k}", rng.permutation(np.tile(np.arange(1, k + 1, dtype=np.uint8), 600_000 // k)).tobytes()
    # one letter of 1-bit code beside a Fibonacci tail of codes up to ~30 bits:
    # multi-code chunks span up to 8 x 30 bits, so more than 255 one-bit codes
    # can lie between two sample slots — the slot overflows (0xFFFF) and the
    # marks fall back to the previous slot or the segment's true start
    fib = [1, 1]
    while len(fib) < 30:
        fib.append(fib[-1] + fib[-2])
    tail = np.repeat(np.arange(1, 31, dtype=np.uint8), np.array(fib))
    skew = np.full(20_000_000, 255, np.uint8)  # byte 255: ~89 %, a 1-bit code (255: no byte-0 duplicate leaf)
    skew[rng.choice(skew.size, tail.size, replace=False)] = rng.permutation(tail)
    yield "one-bit-long-tail", skew.tobytes()
    # codes up to 23 bits (Fibonacci-like counts)
    fib = [1, 1]
    while len(fib) < 24:
        fib.append(fib[-1] + fib[-2])
    letters = np.repeat(np.arange(24, dtype=np.uint8), np.array(fib) * 3)
    yield "fibonacci-24", rng.permutation(letters).tobytes()


@pytest.fixture(params=["sync", "pipeline"])
def decoder(request, monkeypatch):
    """the one-pass decoder (syncdec.hip, opt-in: HUFF_SYNC_DECODE=1) and the
    pipeline (indexless.hip, the default: HUFF_SYNC_DECODE=0) on the same cases"""
    monkeypatch.setenv("HUFF_SYNC_DECODE", "1" if request.param == "sync" else "0")
    return request.param


@pytest.fixture(scope="module")
def cases(O):
    return list(index_free_cases(O, np.random.default_rng(2024)))


def test_indexfree_matches_oracle(H, O, ctx, cases, decoder):
    for name, data in cases:
        roundtrip(H, O, ctx, data)


@pytest.mark.parametrize("l2", [True, False], ids=["l2-lds", "l2-global"])
def test_indexfree_codes_past_table(H, O, ctx, l2, monkeypatch, decoder):
    """codes of 13-23 bits: the walks' level-2 length table in LDS, and
    with HUFF_NO_L2=1 the global multi-level table"""
    if not l2:
        monkeypatch.setenv("HUFF_NO_L2", "1")
    rng = np.random.default_rng(29)
    for p, n in ((0.08, 2_000_000), (0.2, 700_001), (0.35, 65536 * 5 + 3)):
        roundtrip(H, O, ctx, np.minimum(rng.geometric(p, n), 255).astype(np.uint8).tobytes())


def test_indexfree_misaligned_output(H, O, ctx, cases, decoder):
    for name, data in cases[:4]:
        roundtrip(H, O, ctx, data[:1_000_003], misalign=3)


def test_indexfree_equals_check_build(H, O, ctx, monkeypatch):
    """the same stream through the default path (marks + skip codes) and the
    self-checking build (HUFF_DEC_VARIANT=11: walked marks, end-bit checks)"""
    import torch
    from huff_coding import device as D

    data = O.gen_zipf(0x5EED0002, 1 << 23).tobytes()
    comp, pad, tree = roundtrip(H, O, ctx, data)
    dc = torch.from_numpy(np.concatenate([comp, np.zeros(64, np.uint8)])).cuda()
    outs = []
    for flag in ("11", "0"):
        monkeypatch.setenv("HUFF_DEC_VARIANT", flag)
        out = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda")
        assert D.decompress_dev(ctx, tree, dc.data_ptr(), comp.size, pad, out.data_ptr(), len(data) + 64) == len(data)
        outs.append(out[: len(data)].clone())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


def test_indexfree_garbage_payloads(H, O, ctx, decoder):
    """random payloads under fixed trees: whatever the bits, the letters and
    the dropped final code match the reference walk"""
    import torch
    from huff_coding import device as D

    rng = np.random.default_rng(77)
    trees = [O.Tree.from_weights(O.weights_from_bytes(b"abracadabra alakazam")),
             O.Tree.from_weights(O.weights_from_bytes(O.gen_zipf(0x5EED0002, 1 << 16).tobytes()))]
    for t in trees:
        tree = H.HuffTree.try_from_bin(t.as_bin())
        for n in (1, 2, 7, 300, 5000, 123_457, 1_000_003):
            payload = rng.integers(0, 256, n, dtype=np.uint8)
            for pad in (0, 3, 7):
                want = O.decompress(payload.tobytes(), pad, t)
                dc = torch.from_numpy(np.concatenate([payload, np.zeros(64, np.uint8)])).cuda()
                out = torch.empty(len(want) + 64, dtype=torch.uint8, device="cuda")
                got = D.decompress_dev(ctx, tree, dc.data_ptr(), n, pad, out.data_ptr(), len(want) + 64)
                torch.cuda.synchronize()
                assert got == len(want) and out[:got].cpu().numpy().tobytes() == want, (n, pad)


@pytest.mark.parametrize("kind", ["zipf", "text"])
def test_indexfree_full_size_foreign_stream(H, O, ctx, kind, monkeypatch, decoder):
    """BASELINE size: the 1 GiB Zipf (configs[2]) and text streams written on
    the CPU by the oracle's table-driven encoder (no restart index, as the
    reference writes every stream: comp.rs:128-184, 487-519), decoded through
    huff_dev_decompress and compared with the input on the device"""
    import os

    import torch
    from huff_coding import device as D

    n = 1 << 30
    host = O.gen_zipf(0x5EED0002, n) if kind == "zipf" else O.gen_text(0x5EED0005, n)
    t = O.Tree.from_weights(O.weights_from_array(O.fast_hist(host, 16)))
    code, ln = t.code_table()
    comp, bits = O.fast_encode(host, code, ln, threads=min(16, os.cpu_count() or 1))
    pad = (8 - bits % 8) % 8
    tree = H.HuffTree.try_from_bin(t.as_bin())
    x = torch.from_numpy(host).cuda()
    del host
    dc = torch.zeros(comp.size + 64, dtype=torch.uint8, device="cuda")
    dc[: comp.size] = torch.from_numpy(comp).cuda()
    del comp
    out = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    out.fill_(0)
    torch.cuda.synchronize()
    got = D.decompress_dev(ctx, tree, dc.data_ptr(), dc.numel() - 64, pad, out.data_ptr(), n + 64)
    torch.cuda.synchronize()
    assert got == n
    assert torch.equal(out[:n], x)


def test_indexfree_fix_chain(H, O, ctx, monkeypatch, capfd):
    """slowly resynchronising codes (near-fixed lengths): exits that the
    speculative pass's in-workgroup fix-up and round 0 (k_fix_list) leave
    changed are followed by the one-workgroup chain (k_fix_chain); the
    diagnostics (HUFF_FIX_STATS=1) show it ran, and the letters are exact"""
    import re

    monkeypatch.setenv("HUFF_FIX_STATS", "1")
    monkeypatch.setenv("HUFF_SYNC_DECODE", "0")  # the pipeline's fix-up kernels
    rng = np.random.default_rng(31)
    chain = 0
    for k, n in ((160, 4_000_001), (40, 3_000_001), (250, 4_000_003), (129, 3_000_017)):
        roundtrip(H, O, ctx, rng.integers(0, k, n, dtype=np.uint8).tobytes())
        err = capfd.readouterr().err
        got = [int(m) for m in re.findall(r"chain fixes (\d+)", err)]
        assert got, err
        chain += sum(got)
    assert chain > 0


def test_indexfree_lead_in_phase(H, O, ctx, monkeypatch, capfd):
    """codes whose lengths share a factor (all 3 or 6 bits): the speculative
    pass's lead-in stays a multiple of it, so every lane starts in phase and
    the fix-up has nothing to do (a 128-bit lead-in with 6-bit codes once sent
    the fix-up chain through every segment)"""
    import re

    monkeypatch.setenv("HUFF_FIX_STATS", "1")
    rng = np.random.default_rng(37)
    for k in (8, 64):
        data = rng.permutation(np.tile(np.arange(1, k + 1, dtype=np.uint8), 3_000_000 // k)).tobytes()
        monkeypatch.setenv("HUFF_SYNC_DECODE", "0")
        roundtrip(H, O, ctx, data)
        err = capfd.readouterr().err
        stats = re.findall(r"listed by the speculative pass (\d+), chain fixes (\d+)", err)
        assert stats and all(a == "0" and b == "0" for a, b in stats), err
        # the one-pass decoder: segments and lead-in in phase too, so no lane
        # is re-counted (no tail jobs) and it does not fall back
        monkeypatch.setenv("HUFF_SYNC_DECODE", "1")
        roundtrip(H, O, ctx, data)
        err = capfd.readouterr().err
        stats = re.findall(r"huff sync decode: segments \d+ of \d+ bits, tail jobs (\d+), look-back waits \d+, (.*)", err)
        assert stats and all(j == "0" and w == "done" for j, w in stats), err


def test_indexfree_even_lengths_past_table(H, O, ctx, decoder):
    """every code an even length, up to 14 bits (past the 12-bit walk table):
    the long lead-in (kLeadBitsLong, kept a multiple of 2), the uniform
    level-2 length table and the refill-free slow steps (codes <= 16 bits)
    together; weights 4^k give a quaternary tree whatever the tie order"""
    rng = np.random.default_rng(41)
    letters = rng.permutation(256)[:22].astype(np.uint8)
    counts = [4 ** (7 - i) for i in range(1, 7) for _ in range(3)] + [1] * 4
    data = rng.permutation(np.repeat(letters, np.array(counts) * 300)).tobytes()
    lens = O.Tree.from_weights(O.weights_from_bytes(data)).code_table()[1]
    used = lens[letters]
    assert (used % 2 == 0).all() and used.max() == 14, used
    roundtrip(H, O, ctx, data)
    roundtrip(H, O, ctx, data[: len(data) // 3 + 7])


def test_capacity_below_count(H, O, ctx, decoder):
    """the index-free path starts k_mark_lite before the count is
    known and sizes the marks by the caller's capacity. A buffer shorter than
    the decoded count must fail with HUFF_E_BUFFER_TOO_SMALL and the true
    count, write nothing past its capacity, and leave the context able to
    decode the same stream again with a large enough buffer."""
    import ctypes as C

    import torch
    from huff_coding import _lib

    data = O.gen_zipf(0x5EED0002, (1 << 20) + 4321).tobytes()
    t = O.Tree.from_weights(O.weights_from_bytes(data))
    code, ln = t.code_table()
    host = np.frombuffer(data, np.uint8)
    comp, bits = O.fast_encode(host, code, ln, threads=8)
    pad = (8 - bits % 8) % 8
    tree = H.HuffTree.try_from_bin(t.as_bin())
    dc = torch.from_numpy(np.concatenate([comp, np.zeros(64, np.uint8)])).cuda()
    n = len(data)
    out = torch.full((n + 4096,), 0xAB, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    L = _lib.load()
    for cap in (n - 1, n // 2, 4096 + 17, 1):
        out.fill_(0xAB)  # (the one-pass decoder writes the letters that fit)
        torch.cuda.synchronize()
        got = C.c_size_t()
        rc = L.huff_dev_decompress(ctx.h, tree.h, C.c_void_p(dc.data_ptr()), comp.size, pad,
                                   C.c_void_p(out.data_ptr()), cap, C.byref(got))
        torch.cuda.synchronize()
        assert rc == _lib.E_BUFFER_TOO_SMALL and got.value == n, (cap, rc, got.value)
        res = out.cpu().numpy()
        assert (res[cap:] == 0xAB).all(), f"capacity {cap}: wrote past the buffer"
    from huff_coding import device as D

    assert D.decompress_dev(ctx, tree, dc.data_ptr(), comp.size, pad, out.data_ptr(), n) == n
    torch.cuda.synchronize()
    res = out.cpu().numpy()
    assert np.array_equal(res[:n], host)
    assert (res[n:] == 0xAB).all()


@pytest.mark.parametrize("kind,seed", [("zipf", 0x5EED0002), ("text", 0x5EED0005), ("uniform", 0x5EED0001)])
def test_dma_decoder(H, O, ctx, cases, kind, seed, monkeypatch):
    """the opt-in persistent LDS-DMA decoder (decode_wave.hip k_decode_dma,
    HUFF_DMA_DECODE=1; measured slower): the indexed decode of a
    device job (16 MiB + a ragged tail; uniform through the general kernels)
    and, for the first workload, every index-free case"""
    import torch

    monkeypatch.setenv("HUFF_DMA_DECODE", "1")
    monkeypatch.setenv("HUFF_SYNC_DECODE", "0")
    if kind == "uniform":
        monkeypatch.setenv("HUFF_DISABLE_FIXED8", "1")
    from huff_coding import device as D

    n = (1 << 24) + 12345
    x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    D.generate(ctx, kind, seed, x.data_ptr(), n, cdf=D.zipf_cdf(1.2) if kind == "zipf" else None)
    job = H.EncodeJob(ctx, x.data_ptr(), n)
    tree = H.HuffTree.from_weights(H.ByteWeights.from_array(job.hist()))
    bits = job.bits(tree)
    out = torch.zeros((bits + 7) // 8 + 64, dtype=torch.uint8, device="cuda")
    assert job.pack(tree, out.data_ptr(), out.numel()) == bits
    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    job.decode(tree, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dec[:n], x[:n])
    if kind == "zipf":
        for name, data in cases:
            roundtrip(H, O, ctx, data)
