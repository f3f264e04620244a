"""huff_coding — MI355X-native drop-in for the byte path of k-xlsx/huff-encoding.

Python mirror of the reference crate's prelude (huff_coding/src/prelude.rs:1-23)
for the u8 alphabet, over the C ABI in include/huffgpu.h:

    ByteWeights        weights.rs:174-443   (counting = hist256 GPU kernel)
    HuffTree           tree/tree_inner.rs   (host, reference tie order)
    CompressData       comp.rs:40-300
    compress_with_tree comp.rs:419-451      (GPU encode)
    compress           comp.rs:353-356      (deterministic ByteWeights path, see below)
    decompress         comp.rs:487-519      (GPU decode)
    read_compress_write / read_decompress_write   huff/src/comp.rs:32-157

Errors: the reference's Result errors are raised as CompressError /
FromBinError / CompressedDataFromBytesError; its panics as HuffPanic with the
reference's panic message. `compress` differs from the reference on purpose:
the reference builds weights with a RandomState HashMap (weights.rs:82-84), so
its trees differ from run to run under ties; here `compress` is
`compress_with_tree(bytes, HuffTree.from_weights(ByteWeights.from_bytes(bytes)))`,
the deterministic path.
"""
from __future__ import annotations

import ctypes as C
import threading
from typing import Dict, Iterator, Optional, Tuple

import numpy as np

from . import _lib
from ._lib import load

__all__ = [
    "ByteWeights", "HuffTree", "HuffBranch", "HuffLeaf", "CompressData", "compress", "compress_with_tree", "decompress",
    "read_compress_write", "read_decompress_write", "parse_block_size", "Context", "EncodeJob",
    "HuffError", "HuffPanic", "CompressError", "FromBinError", "CompressedDataFromBytesError",
]


# --------------------------------------------------------------------------
# errors
# --------------------------------------------------------------------------
class HuffError(Exception):
    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code
        self.message = message


class HuffPanic(HuffError):
    """A reference panic (empty weights, empty comp bytes, padding > 7, ...)."""


class CompressError(HuffError):
    """comp.rs:562-590: letter not found in codes."""

    def __init__(self, code: int, message: str, missing_letter: int):
        super().__init__(code, f"{message} ({missing_letter})")
        self.missing_letter = missing_letter


class FromBinError(HuffError):
    """tree_inner.rs:673-700"""


class CompressedDataFromBytesError(HuffError):
    """comp.rs:530-554"""


class CliError(HuffError):
    """huff/src/error.rs ErrorKind (MissingHeaderInfo, InvalidHeaderInfo, Io, InvalidInput)."""


_PANICS = {_lib.E_EMPTY_WEIGHTS, _lib.E_EMPTY_COMP, _lib.E_PADDING, _lib.E_TREE_LEN}
_CLI = {_lib.E_IO, _lib.E_MISSING_HEADER, _lib.E_INVALID_HEADER, _lib.E_UNRECOGNIZED}


def branch_code(fn, h, node: int) -> Optional[str]:
    """leaf.rs:70-73 through huff_branch_code / huff_wbranch_code: the code as
    a '0'/'1' string, None for a root with children; a code longer than the
    first buffer (a deep try_from_bin tree) is read again at its reported size"""
    cap = 512
    while True:
        bits = (C.c_uint8 * cap)()
        n, has_code = C.c_size_t(), C.c_int()
        rc = fn(h, node, bits, cap, C.byref(n), C.byref(has_code))
        if rc == _lib.E_BUFFER_TOO_SMALL and n.value > cap:
            cap = n.value
            continue
        _check(rc)
        return "".join(str(bits[k]) for k in range(n.value)) if has_code.value else None


def _check(rc: int):
    if rc == _lib.HUFF_OK:
        return
    msg = _lib.last_error()
    if rc == _lib.E_MISSING_LETTER:
        raise CompressError(rc, msg, int(load().huff_last_missing_letter()))
    if rc == _lib.E_FROM_BIN:
        raise FromBinError(rc, msg)
    if rc == _lib.E_FROM_BYTES:
        raise CompressedDataFromBytesError(rc, msg)
    if rc in _PANICS:
        raise HuffPanic(rc, msg)
    if rc in _CLI:
        raise CliError(rc, msg)
    raise HuffError(rc, msg)


def _buf(data) -> Tuple[object, int, int]:
    """(keepalive, address, length) of a bytes-like or uint8 array"""
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data, dtype=np.uint8)
        return a, a.ctypes.data, a.size
    b = bytes(data)
    cb = C.create_string_buffer(b, len(b)) if b else None
    return cb, (C.addressof(cb) if cb is not None else 0), len(b)


# --------------------------------------------------------------------------
# context
# --------------------------------------------------------------------------
class Context:
    """One HIP stream + device workspace (huff_ctx). One per thread."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        _check(load().huff_ctx_create(device, C.byref(h)))
        self.h = h
        self.device = device

    def set_stream(self, stream_handle: Optional[int]):
        _check(load().huff_ctx_set_stream(self.h, C.c_void_p(stream_handle) if stream_handle else None))

    def synchronize(self):
        _check(load().huff_ctx_synchronize(self.h))

    def set_timing(self, on: bool = True):
        _check(load().huff_ctx_set_timing(self.h, 1 if on else 0))

    def kernel_time(self, name: str):
        """(total ms, launches) of a kernel since the last reset_timing()"""
        ms = C.c_double()
        n = C.c_uint64()
        _check(load().huff_ctx_kernel_time(self.h, name.encode(), C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def reset_timing(self):
        _check(load().huff_ctx_reset_timing(self.h))

    def close(self):
        if getattr(self, "h", None):
            load().huff_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_tls = threading.local()


def default_context() -> Context:
    ctx = getattr(_tls, "ctx", None)
    if ctx is None:
        import os

        ctx = Context(int(os.environ.get("HUFF_DEVICE", os.environ.get("LOCAL_RANK", "0"))))
        _tls.ctx = ctx
    return ctx


# --------------------------------------------------------------------------
# ByteWeights
# --------------------------------------------------------------------------
class _CW(C.Structure):
    _fields_ = [("weights", C.c_uint64 * 256), ("len", C.c_uint64)]


class ByteWeights:
    """weights.rs:174-178 {weights: [usize; 256], len}"""

    def __init__(self):
        self._c = _CW()

    @staticmethod
    def new() -> "ByteWeights":
        return ByteWeights()

    @staticmethod
    def from_bytes(data, ctx: Optional[Context] = None) -> "ByteWeights":
        """weights.rs:265-279, counted by the hist256 GPU kernel"""
        ctx = ctx or default_context()
        keep, addr, n = _buf(data)
        bw = ByteWeights()
        _check(load().huff_weights_from_bytes(ctx.h, addr, n, C.byref(bw._c)))
        return bw

    @staticmethod
    def threaded_from_bytes(data, thread_num: int, ctx: Optional[Context] = None) -> "ByteWeights":
        """weights.rs:293-319 (ration split + merge order, quirk included)"""
        ctx = ctx or default_context()
        keep, addr, n = _buf(data)
        bw = ByteWeights()
        _check(load().huff_weights_threaded_from_bytes(ctx.h, addr, n, thread_num, C.byref(bw._c)))
        return bw

    @staticmethod
    def from_array(counts) -> "ByteWeights":
        a = np.ascontiguousarray(np.asarray(counts, dtype=np.uint64))
        if a.shape != (256,):
            raise ValueError("ByteWeights needs 256 counts")
        bw = ByteWeights()
        C.memmove(bw._c.weights, a.ctypes.data, 256 * 8)
        bw._c.len = int(np.count_nonzero(a))
        return bw

    def get(self, byte: int) -> Optional[int]:
        v = self._c.weights[byte]
        return None if v == 0 else int(v)

    def len(self) -> int:
        return int(self._c.len)

    def is_empty(self) -> bool:
        return self._c.len == 0

    def as_array(self) -> np.ndarray:
        return np.ctypeslib.as_array(self._c.weights).copy()

    def __iter__(self) -> Iterator[Tuple[int, int]]:
        l = (C.c_uint8 * 257)()
        w = (C.c_uint64 * 257)()
        n = load().huff_weights_iter(C.byref(self._c), l, w)
        return iter([(int(l[k]), int(w[k])) for k in range(n)])

    def add_byte_weights(self, other: "ByteWeights"):
        load().huff_weights_add(C.byref(self._c), C.byref(other._c))

    def __iadd__(self, other: "ByteWeights"):
        self.add_byte_weights(other)
        return self

    def __add__(self, other: "ByteWeights") -> "ByteWeights":
        r = ByteWeights()
        C.memmove(C.byref(r._c), C.byref(self._c), C.sizeof(_CW))
        r.add_byte_weights(other)
        return r

    def __eq__(self, other) -> bool:  # weights.rs:216-220: weights only
        return isinstance(other, ByteWeights) and list(self._c.weights) == list(other._c.weights)


# --------------------------------------------------------------------------
# HuffTree
# --------------------------------------------------------------------------
class HuffTree:
    def __init__(self, handle):
        self.h = handle

    def __del__(self):
        try:
            if getattr(self, "h", None):
                load().huff_tree_free(self.h)
                self.h = None
        except Exception:
            pass

    @staticmethod
    def from_weights(weights: ByteWeights) -> "HuffTree":
        h = C.c_void_p()
        _check(load().huff_tree_from_weights(C.byref(weights._c), C.byref(h)))
        return HuffTree(h)

    @staticmethod
    def try_from_bin(bits: str) -> "HuffTree":
        """bits as a '0'/'1' string (bitvec order)"""
        packed = bytearray((len(bits) + 7) // 8)
        for k, ch in enumerate(bits):
            if ch == "1":
                packed[k // 8] |= 0x80 >> (k % 8)
        keep, addr, _ = _buf(bytes(packed))
        h = C.c_void_p()
        _check(load().huff_tree_try_from_bin(addr, len(bits), C.byref(h)))
        return HuffTree(h)

    def clone(self) -> "HuffTree":
        h = C.c_void_p()
        _check(load().huff_tree_clone(self.h, C.byref(h)))
        return HuffTree(h)

    def read_codes(self) -> Dict[int, str]:
        """tree_inner.rs:356-419 -> {byte: '0101'}"""
        out = {}
        L = load()
        bits = (C.c_uint8 * 512)()
        n = C.c_size_t()
        for b in range(256):
            _check(L.huff_tree_code_bits(self.h, b, bits, 512, C.byref(n)))
            if n.value:
                out[b] = "".join(str(bits[k]) for k in range(n.value))
        return out

    def code_table(self):
        """(u64 code right-aligned, u8 len) per byte"""
        code = np.zeros(256, np.uint64)
        ln = np.zeros(256, np.uint8)
        _check(load().huff_tree_read_codes(self.h, code.ctypes.data_as(C.POINTER(C.c_uint64)),
                                           ln.ctypes.data_as(C.POINTER(C.c_uint8))))
        return code, ln

    def as_bin(self) -> str:
        """tree_inner.rs:632-668 as a '0'/'1' string"""
        n = C.c_size_t()
        buf = (C.c_uint8 * 512)()
        _check(load().huff_tree_as_bin(self.h, buf, 512, C.byref(n)))
        return "".join("1" if (buf[k // 8] >> (7 - k % 8)) & 1 else "0" for k in range(n.value))

    def num_leaves(self) -> int:
        return int(load().huff_tree_num_leaves(self.h))

    def root_weight(self) -> int:
        return int(load().huff_tree_root_weight(self.h))

    def root(self) -> "HuffBranch":
        """tree_inner.rs:322-325"""
        b = C.c_int32()
        _check(load().huff_tree_root(self.h, C.byref(b)))
        return HuffBranch(self, b.value)


class HuffLeaf:
    """leaf.rs:25-79 as read from a tree branch: letter (None for a joint
    branch), weight, code (a '0'/'1' string, None for a joint root)"""

    def __init__(self, letter: Optional[int], weight: int, code: Optional[str]):
        self._letter, self._weight, self._code = letter, weight, code

    def letter(self) -> Optional[int]:
        return self._letter

    def weight(self) -> int:
        return self._weight

    def code(self) -> Optional[str]:
        return self._code


class HuffBranch:
    """branch.rs:157-279 over the library's tree: a node id valid while the
    tree lives (the branch keeps the tree alive)"""

    def __init__(self, tree: "HuffTree", node: int):
        self._tree, self._node = tree, node

    def _children(self):
        lft, rgt = C.c_int32(), C.c_int32()
        _check(load().huff_branch_children(self._tree.h, self._node, C.byref(lft), C.byref(rgt)))
        return lft.value, rgt.value

    def leaf(self) -> HuffLeaf:
        L = load()
        has, letter, weight = C.c_int(), C.c_uint8(), C.c_uint64()
        _check(L.huff_branch_leaf(self._tree.h, self._node, C.byref(has), C.byref(letter), C.byref(weight)))
        code = branch_code(L.huff_branch_code, self._tree.h, self._node)
        return HuffLeaf(int(letter.value) if has.value else None, int(weight.value), code)

    def left_child(self) -> Optional["HuffBranch"]:
        lft, _ = self._children()
        return HuffBranch(self._tree, lft) if lft >= 0 else None

    def right_child(self) -> Optional["HuffBranch"]:
        _, rgt = self._children()
        return HuffBranch(self._tree, rgt) if rgt >= 0 else None

    def has_children(self) -> bool:
        return self._children()[0] >= 0

    def children_iter(self):
        """branch.rs:247-250: None, or an iterator over (left, right)"""
        lft, rgt = self._children()
        if lft < 0:
            return None
        return iter((HuffBranch(self._tree, lft), HuffBranch(self._tree, rgt)))


def bitvec_str(bits: str) -> str:
    """bitvec's Display: '[10011000, 11100110, ...]'"""
    return "[" + ", ".join(bits[k:k + 8] for k in range(0, len(bits), 8)) + "]"


# --------------------------------------------------------------------------
# CompressData
# --------------------------------------------------------------------------
class CompressData:
    def __init__(self, handle):
        self.h = handle

    def __del__(self):
        try:
            if getattr(self, "h", None):
                load().huff_cd_free(self.h)
                self.h = None
        except Exception:
            pass

    @staticmethod
    def new(comp_bytes: bytes, padding_bits: int, huff_tree: HuffTree) -> "CompressData":
        """comp.rs:55-68 (panics become HuffPanic)"""
        keep, addr, n = _buf(comp_bytes)
        h = C.c_void_p()
        _check(load().huff_cd_new(addr, n, padding_bits, huff_tree.h, C.byref(h)))
        return CompressData(h)

    def comp_bytes(self) -> bytes:
        p = C.POINTER(C.c_uint8)()
        n = C.c_size_t()
        _check(load().huff_cd_comp_bytes(self.h, C.byref(p), C.byref(n)))
        return C.string_at(p, n.value) if n.value else b""

    def padding_bits(self) -> int:
        return int(load().huff_cd_padding(self.h))

    def huff_tree(self) -> HuffTree:
        t = load().huff_cd_tree(self.h)
        h = C.c_void_p()
        _check(load().huff_tree_clone(t, C.byref(h)))
        return HuffTree(h)

    def has_index(self) -> bool:
        return bool(load().huff_cd_has_index(self.h))

    def to_bytes(self) -> bytes:
        """comp.rs:279-300"""
        n = C.c_size_t()
        rc = load().huff_cd_to_bytes(self.h, None, 0, C.byref(n))
        if rc not in (_lib.HUFF_OK, _lib.E_BUFFER_TOO_SMALL):
            _check(rc)
        buf = (C.c_uint8 * max(n.value, 1))()
        _check(load().huff_cd_to_bytes(self.h, buf, n.value, C.byref(n)))
        return bytes(buf[: n.value])

    @staticmethod
    def try_from_bytes(data) -> "CompressData":
        """comp.rs:128-184"""
        keep, addr, n = _buf(data)
        h = C.c_void_p()
        _check(load().huff_cd_try_from_bytes(addr, n, C.byref(h)))
        return CompressData(h)


def compress_with_tree(letters, huff_tree: HuffTree, ctx: Optional[Context] = None) -> CompressData:
    """comp.rs:419-451 on the GPU (the tree is borrowed, not consumed)."""
    ctx = ctx or default_context()
    keep, addr, n = _buf(letters)
    h = C.c_void_p()
    _check(load().huff_compress_with_tree(ctx.h, addr, n, huff_tree.h, C.byref(h)))
    return CompressData(h)


def compress(letters, ctx: Optional[Context] = None) -> CompressData:
    """ByteWeights -> HuffTree -> compress_with_tree (deterministic; see module doc)."""
    ctx = ctx or default_context()
    keep, addr, n = _buf(letters)
    h = C.c_void_p()
    _check(load().huff_compress_bytes(ctx.h, addr, n, C.byref(h)))
    return CompressData(h)


def decompress(comp_data: CompressData, ctx: Optional[Context] = None) -> bytes:
    """comp.rs:487-519 on the GPU (restart-index decode when the data came from
    this encoder, self-synchronising index-free decode otherwise)."""
    ctx = ctx or default_context()
    n = C.c_size_t()
    rc = load().huff_decompress(ctx.h, comp_data.h, None, 0, C.byref(n))
    if rc not in (_lib.HUFF_OK, _lib.E_BUFFER_TOO_SMALL):
        _check(rc)
    if rc == _lib.HUFF_OK and n.value == 0:
        return b""
    out = np.empty(max(n.value, 1), np.uint8)
    _check(load().huff_decompress(ctx.h, comp_data.h, out.ctypes.data_as(C.POINTER(C.c_uint8)), out.size,
                                  C.byref(n)))
    return out[: n.value].tobytes()


# --------------------------------------------------------------------------
# huff CLI file path
# --------------------------------------------------------------------------
def parse_block_size(s: str) -> int:
    """huff/src/cli.rs:79-114"""
    v = C.c_size_t()
    _check(load().huff_parse_block_size(s.encode(), C.byref(v)))
    return v.value


def read_compress_write(src: str, dst: str, block_size: int = 2_000_000_000, ctx: Optional[Context] = None):
    """huff/src/comp.rs:32-74"""
    ctx = ctx or default_context()
    _check(load().huff_file_compress(ctx.h, src.encode(), dst.encode(), block_size))


def read_decompress_write(src: str, dst: str, block_size: int = 2_000_000_000, ctx: Optional[Context] = None):
    """huff/src/comp.rs:79-157"""
    ctx = ctx or default_context()
    _check(load().huff_file_decompress(ctx.h, src.encode(), dst.encode(), block_size))


from .device import EncodeJob  # noqa: E402  (device-resident jobs)
