"""k_decode_fixed's self-checking build (HUFF_DEC_VARIANT 11) and the decode guards.

The checked build runs the production decoder body with a per-lane check
that every lane's letters end exactly at the next lane's restart entry
(decode_wave.hip fx_check); a mismatch makes the runtime return
HUFF_E_CORRUPT with the task and lane. A wrong letter whose code has the
right length keeps every lane in step, so the check build also compares
per-task letter checksums recorded at encode (checksum.hip). Every decode is also compared
byte-for-byte with the input, and one test shows that the check fires on a
damaged stream.

The round-1/2 builds that decoded wrong letters (forced occupancy, spilled
bodies, the early-loads reproducer) all had a 64-bit shift whose amount sat in
the last allocated VGPR, a gfx950 hardware hazard; they are gone from the
library and `make` rejects any kernel with that instruction form
(tools/check_shift64.py, DESIGN.md §3 "The 64-bit shift hazard",
profiles/r03/shift64/).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

VARIANTS = ["11"]
IDS = ["chk"]


def _gen(H, ctx, kind, seed, n):
    import torch
    from huff_coding import device as D

    x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    D.generate(ctx, kind, seed, x.data_ptr(), n, cdf=D.zipf_cdf(1.2) if kind == "zipf" else None)
    return x


def _encode(H, x, n, ctx):
    import torch

    job = H.EncodeJob(ctx, x.data_ptr(), n)
    w = job.hist()
    tree = H.HuffTree.from_weights(H.ByteWeights.from_array(w))
    bits = job.bits(tree)
    out = torch.zeros((bits + 7) // 8 + 64, dtype=torch.uint8, device="cuda")
    assert job.pack(tree, out.data_ptr(), out.numel()) == bits
    return job, tree, out, bits


def _decode_equal(job, tree, out, x, n):
    import torch

    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    job.decode(tree, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dec[:n], x[:n])


@pytest.mark.parametrize("var", VARIANTS, ids=IDS)
@pytest.mark.parametrize("kind,seed", [("uniform", 0x5EED0001), ("zipf", 0x5EED0002), ("text", 0x5EED0005)])
def test_checked_decode_medium(H, ctx, kind, seed, var, monkeypatch):
    """16 MiB + ragged tail per workload (uniform through the general kernels)"""
    monkeypatch.setenv("HUFF_DEC_VARIANT", var)
    monkeypatch.setenv("HUFF_DISABLE_FIXED8", "1")
    n = (1 << 24) + 12345
    x = _gen(H, ctx, kind, seed, n)
    job, tree, out, _ = _encode(H, x, n, ctx)
    _decode_equal(job, tree, out, x, n)


@pytest.mark.parametrize("var", VARIANTS, ids=IDS)
def test_checked_decode_long_codes(H, ctx, var, monkeypatch):
    """codes longer than the 12-bit table (the decoder's SLOW body)"""
    import torch

    monkeypatch.setenv("HUFF_DEC_VARIANT", var)
    rng = np.random.default_rng(77)
    n = (1 << 22) + 999
    host = np.minimum(rng.geometric(0.45, n) - 1, 255).astype(np.uint8)
    host[rng.integers(0, n, 3000)] = rng.integers(0, 256, 3000, dtype=np.uint8)
    x = torch.from_numpy(np.concatenate([host, np.zeros(64, np.uint8)])).cuda()
    job, tree, out, _ = _encode(H, x, n, ctx)
    _, ln = tree.code_table()
    assert ln.max() > 12
    _decode_equal(job, tree, out, x, n)


@pytest.mark.parametrize("var", VARIANTS, ids=IDS)
def test_checked_decode_full_size_zipf(H, ctx, var, monkeypatch):
    """BASELINE configs[2] (1 GiB Zipf) through the checked build"""
    monkeypatch.setenv("HUFF_DEC_VARIANT", var)
    n = 1 << 30
    x = _gen(H, ctx, "zipf", 0x5EED0002, n)
    job, tree, out, _ = _encode(H, x, n, ctx)
    _decode_equal(job, tree, out, x, n)


@pytest.mark.parametrize("var", VARIANTS, ids=IDS)
def test_checked_indexless_decode(H, O, ctx, var, monkeypatch):
    """the index-free path (oracle-written stream, huff_dev_decompress) ends in
    the same kernel, from the restart points k_mark_lds writes"""
    import torch
    from huff_coding import device as D

    monkeypatch.setenv("HUFF_DEC_VARIANT", var)
    n = (1 << 22) + 77
    host = O.gen_text(0x5EED0005, n)
    w = O.fast_hist(host, 8)
    t = O.Tree.from_weights(O.weights_from_array(w))
    code, ln = t.code_table()
    comp, bits = O.fast_encode(host, code, ln, threads=8)
    pad = (8 - bits % 8) % 8
    tree = H.HuffTree.try_from_bin(t.as_bin())
    d_comp = torch.from_numpy(np.concatenate([comp, np.zeros(64, np.uint8)])).cuda()
    d_out = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    got = D.decompress_dev(ctx, tree, d_comp.data_ptr(), comp.size, pad, d_out.data_ptr(), n + 64)
    torch.cuda.synchronize()
    assert got == n
    assert (d_out[:n].cpu().numpy() == host).all()


def test_check_fires_on_damaged_stream(H, ctx, monkeypatch):
    """a damaged 1 KiB of a Zipf stream: some lane ends off its successor's
    restart entry, and the checked decoder reports it"""
    monkeypatch.setenv("HUFF_DEC_VARIANT", "11")
    n = 1 << 22
    x = _gen(H, ctx, "zipf", 0x5EED0002, n)
    job, tree, out, bits = _encode(H, x, n, ctx)
    out[100_000:101_024] = 0xFF
    import torch

    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    with pytest.raises(H.HuffError) as ei:
        job.decode(tree, out.data_ptr(), dec.data_ptr())
    assert ei.value.code == 19 and "self-check" in str(ei.value)


def test_checksum_sees_wrong_letter_of_right_length(H, ctx, monkeypatch):
    """16 letters of equal weight: every code has 4 bits, so one flipped bit
    of the stream turns one letter into another and leaves every lane in
    step (the end-bit check passes). The check build's letter checksums
    (checksum.hip: per 4,096-letter task, sum and position-weighted sum of
    the input, recorded by pack) see it and name the task."""
    import torch

    monkeypatch.setenv("HUFF_DEC_VARIANT", "11")
    monkeypatch.setenv("HUFF_DISABLE_FIXED8", "1")
    rng = np.random.default_rng(5)
    # equal counts of letters 1..16: a full tree of depth 4 (letter 0 would
    # add the reference's re-yielded byte-0 leaf, weights.rs:396-441)
    n = (1 << 21) + 336
    host = rng.permutation(np.tile(np.arange(1, 17, dtype=np.uint8), n // 16))
    x = torch.from_numpy(np.concatenate([host, np.zeros(64, np.uint8)])).cuda()
    job, tree, out, bits = _encode(H, x, n, ctx)
    _, ln = tree.code_table()
    assert set(ln[1:17].tolist()) == {4} and ln[17:].max() == 0
    _decode_equal(job, tree, out, x, n)  # intact: both checks pass
    byte = 3 * 2048 + 5  # letters 12,298-12,299: task 3
    out[byte] ^= 0x10
    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    with pytest.raises(H.HuffError) as ei:
        job.decode(tree, out.data_ptr(), dec.data_ptr())
    assert ei.value.code == 19 and "letter checksums differ in 1 task" in str(ei.value)
    assert "first: task 3" in str(ei.value)


def test_decode_refuses_other_tree(H, ctx):
    """huffgpu.h: huff_enc_decode needs the tree the stream was packed with
    (ADVICE r1): another tree is HUFF_E_STATE, not garbage"""
    import torch

    n = 1 << 20
    x = _gen(H, ctx, "zipf", 0x5EED0002, n)
    job, tree, out, _ = _encode(H, x, n, ctx)
    y = _gen(H, ctx, "text", 0x5EED0005, n)
    other = H.HuffTree.from_weights(H.ByteWeights.from_array(H.EncodeJob(ctx, y.data_ptr(), n).hist()))
    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    with pytest.raises(H.HuffError) as ei:
        job.decode(other, out.data_ptr(), dec.data_ptr())
    assert ei.value.code == 18
    job.decode(tree, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dec[:n], x[:n])
