"""Device-resident encode/decode jobs (huff_enc_* in include/huffgpu.h).

Inputs already live in HBM (a torch tensor's data_ptr() or a huff_dev_alloc
pointer). Used by bench.py and the multi-GPU path; the reference-named API in
__init__ stages host buffers through the same kernels.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _lib
from ._lib import load


def _check(rc):
    from . import _check as chk

    chk(rc)


class EncodeJob:
    """hist256 -> (host) HuffTree -> pack -> (restart-index) decode over one buffer."""

    def __init__(self, ctx, d_in: int, n: int):
        self.ctx = ctx
        self.n = n
        self.h = C.c_void_p()
        _check(load().huff_enc_create(ctx.h, C.c_void_p(d_in), n, C.byref(self.h)))

    def close(self):
        if getattr(self, "h", None):
            load().huff_enc_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def hist(self) -> np.ndarray:
        """pass 1: the 256 weights (u64) of the job's bytes"""
        w = np.empty(256, np.uint64)
        _check(load().huff_enc_hist(self.h, w.ctypes.data))
        return w

    def hist_launch(self):
        """pass 1 queued ahead, not waited for: the next hist()/compress() of
        this job only waits for its weights (huff_enc_hist_launch). Queued
        between a job's pack and its decode, the host tree build of the next
        compress overlaps that decode."""
        _check(load().huff_enc_hist_launch(self.h))

    def hist_row(self, d_row: int):
        """pass 1 enqueued without a host wait: 258 int64 at d_row (device) =
        [weights(256) | last <= 8 input bytes, little-endian | their count]"""
        _check(load().huff_enc_hist_row(self.h, C.c_void_p(d_row)))

    def bits(self, tree) -> int:
        v = C.c_uint64()
        _check(load().huff_enc_bits(self.h, tree.h, C.byref(v)))
        return v.value

    def pack(self, tree, d_out: int, out_cap: int, bit_base: int = 0, prev_tail: Optional[bytes] = None) -> int:
        """pass 2: writes ceil((bit_base%8 + bits)/8) bytes at d_out; returns bits"""
        v = C.c_uint64()
        pt = prev_tail or b""
        buf = C.create_string_buffer(pt, len(pt)) if pt else None
        _check(load().huff_enc_pack(self.h, tree.h, bit_base, buf, len(pt), C.c_void_p(d_out), out_cap,
                                    C.byref(v)))
        return v.value

    def pack_shards(self, hists: np.ndarray, rank: int, tails, d_out: int, out_cap: int):
        """pass 2 for shard `rank` of len(hists) shards: tree of the summed
        weights, bit base and shared-byte tail computed natively, then pack.
        Returns (HuffTree, bit_base, bits). Raises HuffError(BUFFER_TOO_SMALL)
        with .bits_needed when out_cap is short."""
        from . import HuffError, HuffTree

        h = np.ascontiguousarray(hists, dtype=np.uint64)
        world = h.shape[0]
        tp = lp = None
        if rank:  # the tails of the shards before this one
            tb = np.zeros(world * 8, np.uint8)
            tl = np.zeros(world, np.uint8)
            for q, t in enumerate(tails[:rank]):
                t = bytes(t[-8:])
                tb[q * 8: q * 8 + len(t)] = np.frombuffer(t, np.uint8)
                tl[q] = len(t)
            tp, lp = tb.ctypes.data, tl.ctypes.data
        tree_h = C.c_void_p()
        base = C.c_uint64()
        bits = C.c_uint64()
        rc = load().huff_enc_pack_shards(self.h, h.ctypes.data, world, rank, tp, lp, d_out, out_cap,
                                         C.byref(tree_h), C.byref(base), C.byref(bits))
        try:
            _check(rc)
        except HuffError as e:
            e.bits_needed = bits.value
            e.bit_base = base.value
            raise
        return HuffTree(tree_h), base.value, bits.value

    def compress(self, d_out: int, out_cap: int):
        """compress() of the resident buffer in one native call: pass 1, the
        tree of its weights, pass 2 at bit 0. Returns (HuffTree, bits);
        HuffError(BUFFER_TOO_SMALL) carries .bits_needed"""
        from . import HuffError, HuffTree

        tree_h = C.c_void_p()
        bits = C.c_uint64()
        rc = load().huff_enc_compress(self.h, C.c_void_p(d_out), out_cap, C.byref(tree_h), C.byref(bits))
        try:
            _check(rc)
        except HuffError as e:
            e.bits_needed = bits.value
            e.bit_base = 0
            raise
        return HuffTree(tree_h), bits.value

    def decode(self, tree, d_comp: int, d_out: int):
        """block-parallel decode of this job's pack output via its restart index"""
        _check(load().huff_enc_decode(self.h, tree.h, C.c_void_p(d_comp), C.c_void_p(d_out)))


def decompress_dev(ctx, tree, d_comp: int, comp_bytes: int, padding: int, d_out: int, out_cap: int) -> int:
    """comp.rs:487-519 on a device-resident stream with no restart index
    (self-synchronising decode); returns the number of letters written"""
    n = C.c_size_t()
    rc = load().huff_dev_decompress(ctx.h, tree.h, C.c_void_p(d_comp), comp_bytes, padding,
                                    C.c_void_p(d_out) if d_out else None, out_cap, C.byref(n))
    if not d_out and rc == _lib.E_BUFFER_TOO_SMALL:  # count-only query
        return n.value
    _check(rc)
    return n.value


def generate(ctx, kind: str, seed: int, d_out: int, n: int, offset: int = 0, cdf: Optional[np.ndarray] = None):
    """synthetic input in HBM: kind 'uniform' | 'zipf' | 'text' (cdf for zipf)"""
    k = {"uniform": 0, "zipf": 1, "text": 2}[kind]
    cp = None
    if k == 1:
        cdf = np.ascontiguousarray(cdf, np.uint64)
        cp = cdf.ctypes.data_as(C.POINTER(C.c_uint64))
    _check(load().huff_dev_generate(ctx.h, k, seed, offset, cp, C.c_void_p(d_out), n))


def calibrate(ctx, d_src: int, d_dst: int, n: int, iters: int = 5):
    """measured HBM ceilings of this GPU (not a reference function): best-of-
    iters GB/s of a streaming read of n bytes and of a streaming copy (2n
    bytes moved); d_src / d_dst 16-B aligned device buffers of >= n bytes"""
    r, c = C.c_double(), C.c_double()
    _check(load().huff_dev_calibrate(ctx.h, C.c_void_p(d_src), C.c_void_p(d_dst), n, iters, C.byref(r), C.byref(c)))
    return r.value, c.value


def zipf_cdf(alpha: float = 1.2) -> np.ndarray:
    """P(rank k) ~ k^-alpha, k=1..256, byte = k-1; cdf[k-1] = floor(2^64 * P(<=k))
    (same definition as oracle/huff_oracle.c orc_zipf_cdf; an input table)."""
    import math

    p = [math.pow(float(k), -alpha) for k in range(1, 257)]
    s = 0.0
    for v in p:  # sequential, in the same order as the C definition
        s += v
    acc = 0.0
    cdf = np.zeros(256, np.uint64)
    for i in range(256):
        acc += p[i] / s
        scaled = acc * 18446744073709551616.0
        cdf[i] = np.uint64(0xFFFFFFFFFFFFFFFF) if scaled >= 18446744073709551615.0 else np.uint64(int(scaled))
    cdf[255] = np.uint64(0xFFFFFFFFFFFFFFFF)
    return cdf


class DeviceBuffer:
    """hipMalloc'd bytes owned by a context (for callers without torch)."""

    def __init__(self, ctx, nbytes: int):
        self.ctx = ctx
        self.nbytes = nbytes
        self.p = C.c_void_p()
        _check(load().huff_dev_alloc(ctx.h, nbytes, C.byref(self.p)))

    @property
    def ptr(self) -> int:
        return self.p.value

    def upload(self, data: np.ndarray):
        a = np.ascontiguousarray(data, np.uint8)
        _check(load().huff_memcpy_htod(self.ctx.h, self.p, a.ctypes.data_as(C.c_void_p), a.size))

    def download(self, n: Optional[int] = None) -> np.ndarray:
        n = self.nbytes if n is None else n
        out = np.empty(n, np.uint8)
        _check(load().huff_memcpy_dtoh(self.ctx.h, out.ctypes.data_as(C.c_void_p), self.p, n))
        return out

    def free(self):
        if self.p:
            load().huff_dev_free(self.ctx.h, self.p)
            self.p = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
