"""The single-pass index-free decoder (ifdec.hip) against the oracle.

Streams are written by the CPU restatement (oracle/, comp.rs:419-451) with no
restart index, as the reference writes every CompressData and .hff payload,
and decoded on the device through huff_dev_decompress (comp.rs:487-519).
The cases cover the decoder's paths: the common merge of each lane's walk
with its speculative path, codes longer than the 12-bit table, lanes with
more than 64 letters, blocks whose letters exceed the LDS image, tiny
segments (HUFF_IFD_SEG) that force slow lanes, in-block re-walks and the
multi-kernel fallback, misaligned outputs, and the count-only query.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _roundtrip(H, O, ctx, data, misalign=0):
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
    assert (res[misalign: misalign + n] == host).all(), np.nonzero(res[misalign: misalign + n] != host)[0][:10]
    assert (res[misalign + n:] == 0xAB).all(), "wrote past the letters"
    return comp, pad, tree


def _cases(O, rng):
    yield "zipf-16MiB", O.gen_zipf(0x5EED0002, (1 << 24) + 12345).tobytes()
    yield "text-16MiB", O.gen_text(0x5EED0005, (1 << 24) + 999).tobytes()
    yield "uniform40", rng.integers(0, 40, 3_000_001, dtype=np.uint8).tobytes()
    yield "geometric-long", np.minimum(rng.geometric(0.45, 2_000_003) - 1, 255).astype(np.uint8).tobytes()
    x = np.minimum(rng.geometric(0.45, 1_000_000) - 1, 255).astype(np.uint8)
    x[rng.integers(0, x.size, 3000)] = rng.integers(0, 256, 3000, dtype=np.uint8)  # codes > 12 bits
    yield "long-codes", x.tobytes()
    skew = np.where(rng.random(2_000_000) < 0.95, 0, rng.integers(1, 200, 2_000_000)).astype(np.uint8)
    yield "skewed-95", skew.tobytes()  # lanes past 64 letters, blocks past the image
    runs = np.repeat(rng.integers(0, 6, 40_000, dtype=np.uint8), rng.integers(1, 300, 40_000))
    yield "runs", runs.tobytes()
    for n in (1, 2, 3, 63, 64, 65, 255, 256, 1000, 4095, 65537):
        yield f"small-{n}", rng.integers(0, 7, n, dtype=np.uint8).tobytes()
    yield "two-letters", rng.integers(0, 2, 100_001, dtype=np.uint8).tobytes()


@pytest.fixture(scope="module")
def cases(O):
    return list(_cases(O, np.random.default_rng(2024)))


@pytest.mark.parametrize("mode", ["1", "2"], ids=["gated", "forced"])
def test_ifd_matches_oracle(H, O, ctx, cases, mode, monkeypatch):
    """mode 1: the runtime's choice (slowly resynchronising codes take the
    multi-kernel path); mode 2: every stream through the single pass"""
    monkeypatch.setenv("HUFF_IFD", mode)
    for name, data in cases:
        _roundtrip(H, O, ctx, data)


@pytest.mark.parametrize("seg", ["16", "24", "40", "97", "400"])
def test_ifd_forced_segments(H, O, ctx, cases, seg, monkeypatch):
    """tiny segments: most lanes do not resynchronise inside their segment
    (slow lanes, re-walks, broken anchors -> the multi-kernel fallback);
    large ones: lanes past 64 letters"""
    monkeypatch.setenv("HUFF_IFD_SEG", seg)
    monkeypatch.setenv("HUFF_IFD", "2")  # the single pass even for slowly resynchronising codes
    for name, data in cases:
        if len(data) > 4_000_000:
            continue
        _roundtrip(H, O, ctx, data)


def test_ifd_misaligned_output(H, O, ctx, cases, monkeypatch):
    monkeypatch.setenv("HUFF_IFD", "2")
    for name, data in cases[:3]:
        _roundtrip(H, O, ctx, data[:1_000_003], misalign=3)


def test_ifd_equals_multikernel_path(H, O, ctx, monkeypatch):
    """the same stream through HUFF_IFD=0 (indexless.hip) and the single pass"""
    import torch
    from huff_coding import device as D

    data = O.gen_zipf(0x5EED0002, 1 << 23).tobytes()
    comp, pad, tree = _roundtrip(H, O, ctx, data)
    dc = torch.from_numpy(np.concatenate([comp, np.zeros(64, np.uint8)])).cuda()
    outs = []
    for flag in ("2", "0"):
        monkeypatch.setenv("HUFF_IFD", flag)
        out = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda")
        assert D.decompress_dev(ctx, tree, dc.data_ptr(), comp.size, pad, out.data_ptr(), len(data) + 64) == len(data)
        outs.append(out[: len(data)].clone())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("mode", ["0", "2"], ids=["multikernel", "single-pass"])
def test_ifd_garbage_payloads(H, O, ctx, mode, monkeypatch):
    """random payloads under a fixed tree: whatever the bits, the letters and
    the dropped final code match the reference walk"""
    import torch
    from huff_coding import device as D

    monkeypatch.setenv("HUFF_IFD", mode)
    rng = np.random.default_rng(5)
    t = O.Tree.from_weights(O.weights_from_bytes(O.gen_text(0x5EED0005, 1 << 16).tobytes()))
    tree = H.HuffTree.try_from_bin(t.as_bin())
    for n in (5, 777, 100_003, 2_000_000):
        payload = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for pad in (0, 3, 7):
            want = O.decompress(payload, pad, t)
            dc = torch.frombuffer(bytearray(payload + bytes(64)), dtype=torch.uint8).cuda()
            out = torch.empty(len(want) + 64, dtype=torch.uint8, device="cuda")
            got = D.decompress_dev(ctx, tree, dc.data_ptr(), n, pad, out.data_ptr(), len(want) + 64)
            torch.cuda.synchronize()
            assert got == len(want) and out[:got].cpu().numpy().tobytes() == want
