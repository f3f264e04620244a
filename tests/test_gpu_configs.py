"""BASELINE configs[3] and configs[4] on one GPU, bit-exact against the oracle.

configs[3]: 16 GiB uniform bytes, 8 shards of 2 GiB.
configs[4]: 64 GiB text (the documented enwik8 stand-in), 8 shards of 8 GiB.

The multi-GPU path is contiguous shards + one exchange of per-shard weights
+ an exclusive sum of shard bits (huff/src/comp.rs:177-227 for the
reference's block stitching). On one GPU the shards are jobs over slices of
one stream generated on the device by offset, passed through the same native
huff_enc_pack_shards a rank calls. Checked here:
  * 8 contiguous shards of a 1 GiB uniform stream and of a 1 GiB text stream:
    the concatenated owned bytes == oracle fast_encode of the whole stream;
  * one FULL per-GPU shard of each config at its real, non-zero bit base
    (rank 3 of configs[3]: 2 GiB; rank 5 of configs[4]: 8 GiB, a base that is
    not byte aligned): packed bytes == oracle fast_encode of the shard at that
    bit offset, and decode == input.
The weights of all 8 shards are the real ones (each shard generated and
histogrammed on the device), so the tree and the bit bases are those of the
full 16 GiB / 64 GiB streams.
"""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEEDS = {"uniform": 0x5EED0003, "text": 0x5EED0005}


def _gen(ctx, kind, n, offset, buf=None):
    import torch
    from huff_coding import device as D

    x = buf if buf is not None else torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    D.generate(ctx, kind, SEEDS[kind], x.data_ptr(), n, offset=offset)
    return x


def _all_shard_hists(H, ctx, kind, shard, world):
    """per-shard weights and last-8-byte tails of the whole stream, generated
    shard by shard through one device buffer"""
    hists, tails = [], []
    x = None
    for r in range(world):
        x = _gen(ctx, kind, shard, r * shard, x)
        job = H.EncodeJob(ctx, x.data_ptr(), shard)
        hists.append(job.hist())
        tails.append(x[shard - 8: shard].cpu().numpy().tobytes())
        job.close()
    return np.stack(hists), tails, x


@pytest.mark.parametrize("kind", ["uniform", "text"])
def test_eight_shards_concatenate_to_single_stream(H, O, ctx, kind):
    """1 GiB split into 8 contiguous shards: concatenation == whole-stream encode"""
    import torch
    from huff_coding import mgpu

    world, n = 8, 1 << 30
    shard = n // world
    x = _gen(ctx, kind, n, 0)
    host = x[:n].cpu().numpy()
    jobs, hists, tails = [], [], []
    for r in range(world):
        jobs.append(H.EncodeJob(ctx, x.data_ptr() + r * shard, shard))
        hists.append(jobs[r].hist())
        tails.append(host[(r + 1) * shard - 8:(r + 1) * shard].tobytes())
    hists = np.stack(hists)
    w = hists.sum(axis=0, dtype=np.uint64)
    assert (w == O.fast_hist(host, 16)).all()
    ot = O.Tree.from_weights(O.weights_from_array(w))
    code, ln = ot.code_table()
    want, total = O.fast_encode(host, code, ln, threads=16)
    pieces, base_expect = [], 0
    out = torch.zeros(shard * 2 + 128, dtype=torch.uint8, device="cuda")
    dec = torch.empty(shard + 64, dtype=torch.uint8, device="cuda")
    for r in range(world):
        tree, base, bits = jobs[r].pack_shards(hists, r, tails, out.data_ptr(), out.numel())
        assert tree.as_bin() == ot.as_bin() and base == base_expect
        torch.cuda.synchronize()
        pieces.append(mgpu.owned_bytes(out[: (base % 8 + bits + 7) // 8].cpu().numpy(), base, bits, r == world - 1))
        jobs[r].decode(tree, out.data_ptr(), dec.data_ptr())
        torch.cuda.synchronize()
        assert torch.equal(dec[:shard], x[r * shard:(r + 1) * shard])
        base_expect += bits
    got = np.concatenate(pieces)
    assert base_expect == total and got.size == want.size
    assert hashlib.sha256(got.tobytes()).digest() == hashlib.sha256(want.tobytes()).digest()


@pytest.mark.parametrize("kind,shard_log2,rank", [("uniform", 31, 3), ("text", 33, 5)],
                         ids=["configs3-2GiB-rank3", "configs4-8GiB-rank5"])
def test_full_size_shard_at_its_bit_base(H, O, ctx, kind, shard_log2, rank):
    """one whole per-GPU shard of configs[3] / configs[4] packed at its real
    bit base (from all 8 shards' weights) and decoded"""
    import torch

    world = 8
    shard = 1 << shard_log2
    hists, tails, buf = _all_shard_hists(H, ctx, kind, shard, world)
    x = _gen(ctx, kind, shard, rank * shard, buf)
    job = H.EncodeJob(ctx, x.data_ptr(), shard)
    assert (job.hist() == hists[rank]).all()
    w = hists.sum(axis=0, dtype=np.uint64)
    ot = O.Tree.from_weights(O.weights_from_array(w))
    code, ln = ot.code_table()
    per = hists.astype(np.uint64) @ ln.astype(np.uint64)
    bits_r = int(per[rank])
    cap = (7 + bits_r + 7) // 8 + 128
    out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    tree, base, bits = job.pack_shards(hists, rank, tails, out.data_ptr(), cap)
    assert tree.as_bin() == ot.as_bin()
    assert base == int(per[:rank].sum()) and bits == bits_r and base > 0
    if kind == "text":
        assert base % 8 != 0  # the shard's first byte is shared with rank - 1
    nbytes = (base % 8 + bits + 7) // 8
    torch.cuda.synchronize()
    got = out[:nbytes].cpu().numpy()
    host = x[:shard].cpu().numpy()
    want, wb = O.fast_encode(host, code, ln, threads=16, bit_base=base % 8)
    assert wb == bits and want.size == nbytes
    # byte 0: the shard's bits are its low 8 - base%8 bits (the high ones are
    # rank - 1's, which pack_shards completes from the previous tails)
    mask = (1 << (8 - base % 8)) - 1
    assert (int(got[0]) & mask) == (int(want[0]) & mask)
    assert hashlib.sha256(got[1:].tobytes()).digest() == hashlib.sha256(want[1:].tobytes()).digest()
    b = base % 8
    if b:  # the leading b bits are the last b bits of rank - 1's stream: its last 8 letters' codes
        prev = np.frombuffer(tails[rank - 1], np.uint8)
        pw, pb = O.fast_encode(prev, code, ln, threads=1)
        val = int.from_bytes(pw.tobytes(), "big") >> (pw.size * 8 - pb)
        assert pb >= b and (int(got[0]) >> (8 - b)) == (val & ((1 << b) - 1))
    del got, want, host
    dec = torch.empty(shard + 64, dtype=torch.uint8, device="cuda")
    job.decode(tree, out.data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dec[:shard], x[:shard])
