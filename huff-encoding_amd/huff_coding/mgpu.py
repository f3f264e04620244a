"""Multi-GPU sharding of the encode/decode path.

One process per GPU. The input is cut into contiguous shards (rank r owns
bytes [r*n, (r+1)*n) of the global stream). Per step:

  1. every rank runs hist256 on its shard (pass 1);
  2. ONE collective: all_gather of a 258 x int64 row per rank = its 256
     weights + its last <= 8 input bytes + their count (RCCL over xGMI on GPUs,
     gloo in the CPU tests). Every rank now has every rank's histogram;
  3. every rank builds the identical HuffTree from the summed weights on the
     host (the tree is a deterministic function of the weights);
  4. rank r's first bit is O_r = sum_{q<r} bits_q with bits_q = h_q . len —
     no second collective; the 8 bytes before the shard (previous ranks'
     tails) let the shard's first, shared byte be completed locally;
  5. pack at bit_base O_r, then decode locally from the shard's own stream.

The concatenation over ranks of owned_bytes() is byte-identical to
compress_with_tree over the whole input (the last rank owns the zero-padded
final byte). Messages are 2 KiB per rank: latency-bound, not link-bound.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist


@dataclass
class ShardPlan:
    hists: np.ndarray         # [world, 256] u64 per-rank weights
    weights: np.ndarray       # [256] u64 global weights
    bit_base: int             # O_r
    bits: int                 # this rank's bits
    per_rank_bits: np.ndarray
    prev_tail: bytes          # <= 8 input bytes right before this shard


def exchange(weights: np.ndarray, tail, device: Optional[torch.device] = None, group=None):
    """all_gather of [weights(256) | tail bytes | tail length] -> (hists, tails).

    `tail` is the shard's last <= 8 input bytes: host bytes, or a uint8
    tensor already on `device` (then it never leaves the GPU before the
    collective)."""
    world = dist.get_world_size(group)
    row = np.zeros(258, np.int64)
    row[:256] = np.asarray(weights, np.uint64).view(np.int64)
    dev_tail = isinstance(tail, torch.Tensor)
    if dev_tail:
        tail = tail[-8:]
        row[257] = tail.numel()
    else:
        t = bytes(tail[-8:])
        row[256] = np.frombuffer(t.ljust(8, b"\0"), np.int64)[0]
        row[257] = len(t)
    rt = torch.from_numpy(row)
    if device is not None:
        rt = rt.to(device, non_blocking=False)
    if dev_tail and tail.numel():
        rt.view(torch.uint8)[256 * 8: 256 * 8 + tail.numel()] = tail
    rows = [torch.empty_like(rt) for _ in range(world)]
    dist.all_gather(rows, rt, group=group)
    return rows_to_hists(torch.stack(rows).cpu().numpy())


def rows_to_hists(allr: np.ndarray):
    """[world, 258] int64 rows (exchange layout) -> (hists u64 [world, 256], tails)"""
    hists = allr[:, :256].view(np.uint64).copy()
    tails = [allr[q, 256:257].view(np.uint8)[: int(allr[q, 257])].tobytes() for q in range(allr.shape[0])]
    return hists, tails


class DeviceExchange:
    """The sharded pass 1 with the row built on the GPU (huff_enc_hist_row)
    and all-gathered by RCCL in stream order: hist kernels -> row kernel ->
    all_gather_into_tensor -> one copy of the world x 258 rows into pinned
    host memory -> ONE host wait. No host round trip precedes the collective
    (compare exchange(), which reads the weights back first)."""

    def __init__(self, device: torch.device, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.row = torch.empty(258, dtype=torch.int64, device=device)
        self.rows = torch.empty(self.world * 258, dtype=torch.int64, device=device)
        self.host = torch.empty(self.world * 258, dtype=torch.int64, pin_memory=True)
        self.done = torch.cuda.Event()

    def __call__(self, job):
        job.hist_row(self.row.data_ptr())  # on the context stream = torch's current stream
        dist.all_gather_into_tensor(self.rows, self.row, group=self.group)
        self.host.copy_(self.rows, non_blocking=True)
        self.done.record()
        self.done.synchronize()
        return rows_to_hists(self.host.numpy().reshape(self.world, 258))


def pack_rows(job, rows: np.ndarray, rank: int, d_out: int, out_cap: int):
    """huff_mgpu_pack_rows: the native host half of huff_mgpu_compress over
    rows the caller gathered itself ([world, 258] int64, each rank's
    huff_enc_hist_row output, rank order) -> (HuffTree, bit_base, bits,
    owned_bytes); a short buffer raises HuffError with .bits_needed /
    .bit_base"""
    import ctypes as C

    from ._lib import load

    from . import HuffError, HuffTree, _check

    rows = np.ascontiguousarray(rows, np.int64)
    world = rows.shape[0]
    tree_h = C.c_void_p()
    base, bits, owned = C.c_uint64(), C.c_uint64(), C.c_uint64()
    rc = load().huff_mgpu_pack_rows(job.h, rows.ctypes.data_as(C.c_void_p), world, rank, C.c_void_p(d_out), out_cap,
                                    C.byref(tree_h), C.byref(base), C.byref(bits), C.byref(owned))
    try:
        _check(rc)
    except HuffError as e:
        e.bits_needed = bits.value
        e.bit_base = base.value
        raise
    return HuffTree(tree_h), base.value, bits.value, owned.value


def plan(hists: np.ndarray, tails: List[bytes], code_len: np.ndarray, rank: int) -> ShardPlan:
    per = hists.astype(np.uint64) @ np.asarray(code_len, np.uint64)
    before = b"".join(tails[:rank])
    return ShardPlan(hists=hists, weights=hists.sum(axis=0, dtype=np.uint64), bit_base=int(per[:rank].sum()),
                     bits=int(per[rank]), per_rank_bits=per, prev_tail=before[-8:])


def owned_bytes(local: np.ndarray, bit_base: int, bits: int, is_last: bool) -> np.ndarray:
    """the bytes of the global stream this rank contributes: its local stream
    starts at global byte bit_base//8; the partial final byte belongs to the
    next rank (which completes it), except on the last rank"""
    end = bit_base % 8 + bits
    keep = (end + 7) // 8 if is_last else end // 8
    return local[:keep]


def encode_shard_plan(job, shard_tail: bytes, rank: int, device=None, group=None, tree_from_weights=None):
    """steps 1-4: hist, exchange, tree, offsets. Returns (tree, plan)."""
    if tree_from_weights is None:
        from . import ByteWeights, HuffTree

        def tree_from_weights(w):
            return HuffTree.from_weights(ByteWeights.from_array(w))
    w = job.hist()
    hists, tails = exchange(w, shard_tail, device=device, group=group)
    tree = tree_from_weights(hists.sum(axis=0, dtype=np.uint64))
    _, ln = tree.code_table()
    return tree, plan(hists, tails, ln, rank)


class NativeComm:
    """The library's own RCCL communicator (huff_comm, include/huffgpu.h) and
    the one-call sharded compress a Rust/C host would bind. rank 0 makes the
    id (unique_id()); the caller distributes its 128 bytes (here: through the
    torch.distributed process group that launched the ranks)."""

    ID_BYTES = 128

    def __init__(self, ctx, world: int, rank: int, uid: bytes):
        import ctypes as C

        from ._lib import load

        from . import _check

        if len(uid) != self.ID_BYTES:
            raise ValueError("RCCL unique id must be 128 bytes")
        self.ctx, self.world, self.rank = ctx, world, rank
        self.h = C.c_void_p()
        self._id = C.create_string_buffer(bytes(uid), self.ID_BYTES)
        _check(load().huff_comm_init(ctx.h, self._id, world, rank, C.byref(self.h)))

    @staticmethod
    def unique_id() -> bytes:
        import ctypes as C

        from ._lib import load

        from . import _check

        buf = C.create_string_buffer(NativeComm.ID_BYTES)
        _check(load().huff_comm_unique_id(buf))
        return buf.raw

    @classmethod
    def from_process_group(cls, ctx, group=None):
        """every rank of the torch.distributed group joins one huff_comm"""
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        return cls(ctx, world, rank, obj[0])

    def observed_world(self):
        """(world, rank) as RCCL itself reports them (ncclCommCount /
        ncclCommUserRank through huff_comm_world)"""
        import ctypes as C

        from ._lib import load

        from . import _check

        w, r = C.c_int(), C.c_int()
        _check(load().huff_comm_world(self.h, C.byref(w), C.byref(r)))
        return w.value, r.value

    def exchange_launch(self, job):
        """huff_mgpu_exchange_launch: the exchange of the job's next compress
        queued now (every rank at the same point); that compress then only
        waits for the gathered rows"""
        from ._lib import load

        from . import _check

        _check(load().huff_mgpu_exchange_launch(self.h, job.h))

    def compress(self, job, d_out: int, out_cap: int):
        """huff_mgpu_compress: (HuffTree, bit_base, bits, owned_bytes); a short
        buffer raises HuffError with .bits_needed / .bit_base"""
        import ctypes as C

        from ._lib import load

        from . import HuffError, HuffTree, _check

        tree_h = C.c_void_p()
        base, bits, owned = C.c_uint64(), C.c_uint64(), C.c_uint64()
        rc = load().huff_mgpu_compress(self.h, job.h, C.c_void_p(d_out), out_cap, C.byref(tree_h), C.byref(base),
                                       C.byref(bits), C.byref(owned))
        try:
            _check(rc)
        except HuffError as e:
            e.bits_needed = bits.value
            e.bit_base = base.value
            raise
        return HuffTree(tree_h), base.value, bits.value, owned.value

    def close(self):
        from ._lib import load

        if getattr(self, "h", None):
            load().huff_comm_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
