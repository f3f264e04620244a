"""Many small byte streams at once (include/huffgpu.h
huff_batch_hist / huff_batch_trees): the byte weights and the HuffTree of
every stream of a batch, each in one launch, bit-exact with
HuffTree::from_weights (tree_inner.rs:281-320) stream by stream.

Device tensors in, device tensors out:

    hist = batch_hist(ctx, data_u8, offsets_u64)          # [S, 256] u64
    t = batch_trees(ctx, hist)                             # BatchTrees
    t.tree_bits[s, : (t.tree_nbits[s] + 7) // 8]          # as_bin, MSB first
    t.codes[s, letter] == code << 8 | len                  # 0: no code
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import torch

from . import _lib
from ._lib import load

TREE_BITS_MAX_BYTES = 322  # HUFF_TREE_BITS_MAX_BYTES


def _check(rc: int):
    from . import _check as chk

    chk(rc)


def batch_hist(ctx, data: torch.Tensor, offsets: torch.Tensor) -> torch.Tensor:
    """[S, 256] u64 (as int64) weights of data[offsets[s]:offsets[s+1]]; a
    descending pair (offsets[s+1] < offsets[s]) is an empty stream, as
    huff_batch_hist defines it (include/huffgpu.h)"""
    assert data.is_cuda and data.dtype == torch.uint8 and data.is_contiguous()
    assert offsets.is_cuda and offsets.dtype == torch.int64 and offsets.is_contiguous()
    ns = offsets.numel() - 1
    if ns > 0:  # every offset inside the data, so no stream reads past it (one device reduction, one host read)
        ok = (offsets.min() >= 0) & (offsets.max() <= data.numel())
        if not bool(ok.item()):
            raise ValueError("offsets must lie in [0, data.numel()]")
    hist = torch.empty((max(ns, 0), 256), dtype=torch.int64, device=data.device)
    _check(load().huff_batch_hist(ctx.h, C.c_void_p(data.data_ptr()), C.c_void_p(offsets.data_ptr()), ns,
                                  C.c_void_p(hist.data_ptr())))
    return hist


@dataclass
class BatchTrees:
    tree_bits: torch.Tensor   # [S, TREE_BITS_MAX_BYTES] u8
    tree_nbits: torch.Tensor  # [S] int32
    codes: torch.Tensor       # [S, 256] int64: code << 8 | len
    max_len: torch.Tensor     # [S] int32
    status: torch.Tensor      # [S] int32: 0, E_EMPTY_WEIGHTS, E_CODE_TOO_LONG or E_INVALID_ARG (weights >= 2^54)


def batch_trees(ctx, hist: torch.Tensor) -> BatchTrees:
    assert hist.is_cuda and hist.dtype == torch.int64 and hist.is_contiguous() and hist.shape[1:] == (256,)
    ns = hist.shape[0]
    dev = hist.device
    r = BatchTrees(torch.zeros((ns, TREE_BITS_MAX_BYTES), dtype=torch.uint8, device=dev),
                   torch.zeros(ns, dtype=torch.int32, device=dev), torch.empty((ns, 256), dtype=torch.int64, device=dev),
                   torch.zeros(ns, dtype=torch.int32, device=dev), torch.zeros(ns, dtype=torch.int32, device=dev))
    _check(load().huff_batch_trees(ctx.h, C.c_void_p(hist.data_ptr()), ns, C.c_void_p(r.tree_bits.data_ptr()),
                                   TREE_BITS_MAX_BYTES, C.c_void_p(r.tree_nbits.data_ptr()),
                                   C.c_void_p(r.codes.data_ptr()), C.c_void_p(r.max_len.data_ptr()),
                                   C.c_void_p(r.status.data_ptr())))
    return r


E_EMPTY_WEIGHTS = _lib.E_EMPTY_WEIGHTS
E_CODE_TOO_LONG = _lib.E_CODE_TOO_LONG
E_INVALID_ARG = _lib.E_INVALID_ARG
