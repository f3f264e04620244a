"""Multi-rank sharding logic (huff_coding/mgpu.py) on CPU with
the gloo backend, world sizes 2 and 3.

Each rank owns a contiguous shard of one global input (ragged sizes, one
shard shorter than 8 bytes, one empty). The GPU pack is stood in for by the
oracle's table-driven encoder reproducing exactly what huff_enc_pack writes:
the global stream from byte bit_base // 8, whose first byte also carries the
previous shards' last bits (recomputed from prev_tail). The test checks that
  - every rank builds the same tree from the exchanged weights,
  - the concatenation of owned_bytes() over ranks equals compress_with_tree
    over the whole input (oracle), and the padding matches.
The real kernel's handling of bit_base/prev_tail is covered on the GPU by
test_gpu_parity.py::test_shard_stitching_on_one_gpu.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _global_input(seed):
    rng = np.random.default_rng(seed)
    sizes = [5000, 3, 0, 777, 12345][: 5]
    alphabet = np.frombuffer(b"etaoin shrdlu\n\x00\xff", np.uint8)
    p = rng.random(alphabet.size) ** 3
    p /= p.sum()
    return rng.choice(alphabet, size=sum(sizes), p=p).astype(np.uint8), sizes


def _shard_sizes(total, world, seed):
    rng = np.random.default_rng(seed + world)
    cuts = np.sort(rng.integers(0, total, world - 1))
    if world >= 3:
        cuts[0] = cuts[1] - 3 if cuts[1] >= 3 else cuts[0]  # a shard shorter than 8 bytes
    edges = [0, *cuts.tolist(), total]
    return [edges[i + 1] - edges[i] for i in range(world)], edges


def fake_pack(O, shard, code, ln, bit_base, prev_tail):
    """the bytes huff_enc_pack writes at d_out for this shard"""
    r = bit_base % 8
    pt = np.frombuffer(prev_tail, np.uint8)
    P = int(sum(int(ln[b]) for b in pt))
    assert P >= r
    s0 = (r - P) % 8
    data = np.concatenate([pt, shard]).astype(np.uint8)
    if data.size == 0:
        return np.zeros(0, np.uint8)
    enc, _ = O.fast_encode(data, code, ln, threads=1, bit_base=s0)
    return enc[(s0 + P - r) // 8:]


def _worker(rank, world, port, seed, q):
    sys.path[:0] = [os.path.join(ROOT, "huff-encoding_amd"), os.path.join(ROOT, "oracle")]
    import torch.distributed as dist

    import huff_coding as H
    import oracle as O
    from huff_coding import mgpu

    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        x, _ = _global_input(seed)
        sizes, edges = _shard_sizes(x.size, world, seed)
        shard = x[edges[rank]: edges[rank + 1]]
        w = O.fast_hist(shard, 1) if shard.size else np.zeros(256, np.uint64)
        hists, tails = mgpu.exchange(w, shard[-8:].tobytes())
        tree = H.HuffTree.from_weights(H.ByteWeights.from_array(hists.sum(axis=0, dtype=np.uint64)))
        code, ln = tree.code_table()
        pl = mgpu.plan(hists, tails, ln, rank)
        local = fake_pack(O, shard, code, ln, pl.bit_base, pl.prev_tail)
        mine = mgpu.owned_bytes(local, pl.bit_base, pl.bits, rank == world - 1)
        got = [None] * world
        dist.all_gather_object(got, (mine.tobytes(), tree.as_bin(), pl.bit_base, pl.bits))
        if rank == 0:
            q.put(("ok", got))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put(("err", f"rank {rank}: {type(e).__name__}: {e}"))
        raise


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_stream_equals_single_stream(world, O, H):
    import torch.multiprocessing as mp

    seed = 1234
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    status, got = q.get(timeout=180)
    for p in procs:
        p.join(60)
    assert status == "ok", got
    assert all(p.exitcode == 0 for p in procs)

    x, _ = _global_input(seed)
    t = O.Tree.from_weights(O.weights_from_array(O.fast_hist(x, 1)))
    want, pad = O.compress_with_tree(x.tobytes(), t)
    assert len({g[1] for g in got}) == 1, "ranks built different trees"
    assert got[0][1] == H.HuffTree.from_weights(H.ByteWeights.from_array(O.fast_hist(x, 1))).as_bin()
    stream = b"".join(g[0] for g in got)
    assert stream == want
    end = got[-1][2] + got[-1][3]
    assert (8 - end % 8) % 8 == pad
    # bit bases are the exclusive scan of per-rank bits
    assert [g[2] for g in got] == list(np.cumsum([0] + [g[3] for g in got[:-1]]))
