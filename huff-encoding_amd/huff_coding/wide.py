"""HuffTree<L> / compress / decompress for the reference's wider integer
letters (include/huffgpu_wide.h; SURVEY.md §8f-3, letter.rs:41-60).

A letter type is a numpy integer dtype (int8 ... uint64) or one of the
128-bit names "u128" / "i128" (arrays of dtype V16, 16 little-endian bytes
per letter). Letters are handled as their bit patterns, as the reference's
to_be_bytes / from_be_bytes are bit copies; Python-side letter values are
ints of the type's range.

    w = build_weights_map(letters)              # {letter: count}, ascending
    t = WideTree.from_weights(w, letters.dtype) # iteration order of `w`
    cd = compress_with_tree(letters, t)
    assert (decompress(cd) == letters).all()
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Iterable, Optional, Tuple, Union

import numpy as np

from . import _lib
from ._lib import load

U128 = "u128"
I128 = "i128"


def _check(rc: int):
    if rc == _lib.E_MISSING_LETTER:
        buf = (C.c_uint8 * 16)()
        w = C.c_uint32()
        load().huff_last_missing_wletter(buf, C.byref(w))
        from . import CompressError

        raise CompressError(rc, _lib.last_error(), int.from_bytes(bytes(buf[: w.value]), "little"))
    from . import _check as chk

    chk(rc)


class LetterType:
    """width in bytes, signedness, numpy storage dtype"""

    def __init__(self, dtype):
        if isinstance(dtype, str) and dtype in (U128, I128):
            self.width, self.signed, self.np = 16, dtype == I128, np.dtype("V16")
            self.name = dtype
        else:
            d = np.dtype(dtype)
            if d.kind not in "iu" or d.itemsize not in (1, 2, 4, 8):
                raise TypeError(f"{d} is not an integer letter type (letter.rs:56-60)")
            self.width, self.signed, self.np = d.itemsize, d.kind == "i", d.newbyteorder("<")
            self.name = d.name

    def to_int(self, raw: bytes) -> int:
        return int.from_bytes(raw, "little", signed=self.signed)

    def to_raw(self, v: int) -> bytes:
        return int(v).to_bytes(self.width, "little", signed=self.signed)

    def array(self, letters) -> np.ndarray:
        """contiguous storage array of the letters"""
        if isinstance(letters, np.ndarray) and letters.dtype == self.np:
            return np.ascontiguousarray(letters)
        if self.width == 16:
            return np.frombuffer(b"".join(self.to_raw(v) for v in letters), self.np).copy()
        return np.ascontiguousarray(np.asarray(letters, dtype=self.np))

    def values(self, arr: np.ndarray) -> list:
        if self.width == 16:
            return [self.to_int(arr[i].tobytes()) for i in range(arr.size)]
        return [int(v) for v in arr]


def letters_u128(values: Iterable[int], signed: bool = False) -> np.ndarray:
    """a V16 array of 128-bit letters from Python ints"""
    return LetterType(I128 if signed else U128).array(list(values))


def _ltype_of(letters) -> LetterType:
    if isinstance(letters, np.ndarray):
        if letters.dtype == np.dtype("V16"):
            return LetterType(U128)
        return LetterType(letters.dtype)
    raise TypeError("letters must be a numpy integer array (or V16 for 128-bit letters)")


class WideTree:
    """HuffTree<L> (tree_inner.rs) for an integer letter type L"""

    def __init__(self, handle, ltype: LetterType):
        self.h = handle
        self.ltype = ltype

    def __del__(self):
        try:
            if getattr(self, "h", None):
                load().huff_wtree_free(self.h)
                self.h = None
        except Exception:
            pass

    @staticmethod
    def from_weights(weights: Union[Dict[int, int], Iterable[Tuple[int, int]]], dtype) -> "WideTree":
        """tree_inner.rs:281-320 over the weights in their iteration order"""
        lt = LetterType(dtype)
        items = list(weights.items()) if isinstance(weights, dict) else list(weights)
        letters = lt.array([k for k, _ in items])
        w = np.asarray([v for _, v in items] or [0], np.uint64)
        h = C.c_void_p()
        _check(load().huff_wtree_from_weights(lt.width, letters.ctypes.data if items else None,
                                              w.ctypes.data, len(items), C.byref(h)))
        return WideTree(h, lt)

    @staticmethod
    def try_from_bin(bits: str, dtype) -> "WideTree":
        """tree_inner.rs:522-604 (bits as a '0'/'1' string)"""
        lt = LetterType(dtype)
        packed = bytearray((len(bits) + 7) // 8 or 1)
        for k, ch in enumerate(bits):
            if ch == "1":
                packed[k // 8] |= 0x80 >> (k % 8)
        buf = (C.c_uint8 * len(packed)).from_buffer(packed)
        h = C.c_void_p()
        _check(load().huff_wtree_try_from_bin(lt.width, buf, len(bits), C.byref(h)))
        return WideTree(h, lt)

    def clone(self) -> "WideTree":
        h = C.c_void_p()
        _check(load().huff_wtree_clone(self.h, C.byref(h)))
        return WideTree(h, self.ltype)

    def num_leaves(self) -> int:
        return int(load().huff_wtree_num_leaves(self.h))

    def code_table(self):
        """(letters storage array, u64 codes right-aligned, u8 lens), ascending letter"""
        n = C.c_size_t()
        rc = load().huff_wtree_read_codes(self.h, None, None, None, 0, C.byref(n))
        if rc not in (_lib.HUFF_OK, _lib.E_BUFFER_TOO_SMALL):
            _check(rc)
        lt = self.ltype
        letters = np.zeros(n.value, lt.np) if lt.width < 16 else np.zeros(n.value, np.dtype("V16"))
        code = np.zeros(n.value, np.uint64)
        ln = np.zeros(n.value, np.uint8)
        _check(load().huff_wtree_read_codes(self.h, letters.ctypes.data, code.ctypes.data_as(C.POINTER(C.c_uint64)),
                                            ln.ctypes.data_as(C.POINTER(C.c_uint8)), n.value, C.byref(n)))
        return letters, code, ln

    def read_codes(self) -> Dict[int, str]:
        """tree_inner.rs:356-419 -> {letter: '0101'}"""
        letters, code, ln = self.code_table()
        vals = self.ltype.values(letters)
        return {v: format(int(c), f"0{int(l)}b") for v, c, l in zip(vals, code, ln)}

    def as_bin(self) -> str:
        """tree_inner.rs:632-668 as a '0'/'1' string"""
        n = C.c_size_t()
        _check(load().huff_wtree_as_bin(self.h, None, 0, C.byref(n)))
        buf = (C.c_uint8 * max((n.value + 7) // 8, 1))()
        _check(load().huff_wtree_as_bin(self.h, buf, len(buf), C.byref(n)))
        return "".join("1" if (buf[k // 8] >> (7 - k % 8)) & 1 else "0" for k in range(n.value))

    def root(self) -> "WideBranch":
        """tree_inner.rs:322-325"""
        b = C.c_int32()
        _check(load().huff_wtree_root(self.h, C.byref(b)))
        return WideBranch(self, b.value)


class WideBranch:
    """HuffBranch<L> (branch.rs:157-279) of a WideTree; leaf() gives a
    huff_coding.HuffLeaf whose letter is the integer value of L"""

    def __init__(self, tree: WideTree, node: int):
        self._tree, self._node = tree, node

    def _children(self):
        lft, rgt = C.c_int32(), C.c_int32()
        _check(load().huff_wbranch_children(self._tree.h, self._node, C.byref(lft), C.byref(rgt)))
        return lft.value, rgt.value

    def leaf(self):
        from . import HuffLeaf

        L = load()
        lt = self._tree.ltype
        has, weight = C.c_int(), C.c_uint64()
        raw = (C.c_uint8 * lt.width)()
        _check(L.huff_wbranch_leaf(self._tree.h, self._node, C.byref(has), raw, C.byref(weight)))
        from . import branch_code

        code = branch_code(L.huff_wbranch_code, self._tree.h, self._node)
        letter = lt.to_int(bytes(raw)) if has.value else None
        return HuffLeaf(letter, int(weight.value), code)

    def left_child(self) -> Optional["WideBranch"]:
        lft, _ = self._children()
        return WideBranch(self._tree, lft) if lft >= 0 else None

    def right_child(self) -> Optional["WideBranch"]:
        _, rgt = self._children()
        return WideBranch(self._tree, rgt) if rgt >= 0 else None

    def has_children(self) -> bool:
        return self._children()[0] >= 0

    def children_iter(self):
        """branch.rs:247-250: None, or an iterator over (left, right)"""
        lft, rgt = self._children()
        if lft < 0:
            return None
        return iter((WideBranch(self._tree, lft), WideBranch(self._tree, rgt)))


class WideCompressData:
    """CompressData<L> (comp.rs:40-300)"""

    def __init__(self, handle, ltype: LetterType):
        self.h = handle
        self.ltype = ltype

    def __del__(self):
        try:
            if getattr(self, "h", None):
                load().huff_wcd_free(self.h)
                self.h = None
        except Exception:
            pass

    @staticmethod
    def new(comp_bytes: bytes, padding_bits: int, huff_tree: WideTree) -> "WideCompressData":
        b = bytes(comp_bytes)
        buf = C.create_string_buffer(b, len(b)) if b else None
        h = C.c_void_p()
        _check(load().huff_wcd_new(buf, len(b), padding_bits, huff_tree.h, C.byref(h)))
        return WideCompressData(h, huff_tree.ltype)

    def comp_bytes(self) -> bytes:
        p = C.POINTER(C.c_uint8)()
        n = C.c_size_t()
        _check(load().huff_wcd_comp_bytes(self.h, C.byref(p), C.byref(n)))
        return C.string_at(p, n.value) if n.value else b""

    def padding_bits(self) -> int:
        return int(load().huff_wcd_padding(self.h))

    def huff_tree(self) -> WideTree:
        h = C.c_void_p()
        _check(load().huff_wtree_clone(load().huff_wcd_tree(self.h), C.byref(h)))
        return WideTree(h, self.ltype)

    def has_index(self) -> bool:
        return bool(load().huff_wcd_has_index(self.h))

    def to_bytes(self) -> bytes:
        n = C.c_size_t()
        rc = load().huff_wcd_to_bytes(self.h, None, 0, C.byref(n))
        if rc not in (_lib.HUFF_OK, _lib.E_BUFFER_TOO_SMALL):
            _check(rc)
        buf = (C.c_uint8 * max(n.value, 1))()
        _check(load().huff_wcd_to_bytes(self.h, buf, n.value, C.byref(n)))
        return bytes(buf[: n.value])

    @staticmethod
    def try_from_bytes(data: bytes, dtype) -> "WideCompressData":
        lt = LetterType(dtype)
        b = bytes(data)
        buf = C.create_string_buffer(b, len(b)) if b else None
        h = C.c_void_p()
        _check(load().huff_wcd_try_from_bytes(lt.width, buf, len(b), C.byref(h)))
        return WideCompressData(h, lt)


def _ctx(ctx):
    from . import default_context

    return ctx or default_context()


def build_weights_map(letters: np.ndarray, ctx=None) -> Dict[int, int]:
    """weights.rs:82-123 on the GPU: {letter: count}, ascending letter bit pattern"""
    lt = _ltype_of(letters)
    a = lt.array(letters)
    n = C.c_size_t()
    rc = load().huff_wweights_map(_ctx(ctx).h, lt.width, a.ctypes.data if a.size else None, a.size, None, None, 0,
                                  C.byref(n))
    if rc not in (_lib.HUFF_OK, _lib.E_BUFFER_TOO_SMALL):
        _check(rc)
    u = np.zeros(n.value, a.dtype)
    w = np.zeros(n.value, np.uint64)
    _check(load().huff_wweights_map(_ctx(ctx).h, lt.width, a.ctypes.data if a.size else None, a.size, u.ctypes.data,
                                    w.ctypes.data_as(C.POINTER(C.c_uint64)), n.value, C.byref(n)))
    return dict(zip(lt.values(u), (int(x) for x in w)))


def compress_with_tree(letters: np.ndarray, huff_tree: WideTree, ctx=None) -> WideCompressData:
    """comp.rs:419-451 on the GPU (the tree is borrowed)"""
    a = huff_tree.ltype.array(letters)
    h = C.c_void_p()
    _check(load().huff_wcompress_with_tree(_ctx(ctx).h, a.ctypes.data if a.size else None, a.size, huff_tree.h,
                                           C.byref(h)))
    return WideCompressData(h, huff_tree.ltype)


def compress(letters: np.ndarray, ctx=None) -> WideCompressData:
    """comp.rs:353-359 (weights in build_weights_map's ascending order)"""
    lt = _ltype_of(letters)
    a = lt.array(letters)
    h = C.c_void_p()
    _check(load().huff_wcompress(_ctx(ctx).h, lt.width, a.ctypes.data if a.size else None, a.size, C.byref(h)))
    return WideCompressData(h, lt)


def decompress(comp_data: WideCompressData, ctx=None) -> np.ndarray:
    """comp.rs:487-519 on the GPU -> array of the letter type"""
    lt = comp_data.ltype
    n = C.c_size_t()
    rc = load().huff_wdecompress(_ctx(ctx).h, comp_data.h, None, 0, C.byref(n))
    if rc not in (_lib.HUFF_OK, _lib.E_BUFFER_TOO_SMALL):
        _check(rc)
    out = np.zeros(n.value, lt.np)
    if n.value == 0:
        return out
    _check(load().huff_wdecompress(_ctx(ctx).h, comp_data.h, out.ctypes.data, n.value, C.byref(n)))
    return out[: n.value]


class WideEncodeJob:
    """device-resident job over letters in HBM (huff_wenc_*)"""

    def __init__(self, ctx, width: int, d_in: int, n: int):
        self.ctx = ctx
        self.n = n
        self.width = width
        self.h = C.c_void_p()
        _check(load().huff_wenc_create(ctx.h, width, C.c_void_p(d_in), n, C.byref(self.h)))

    def close(self):
        if getattr(self, "h", None):
            load().huff_wenc_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def bits(self, tree: WideTree) -> int:
        v = C.c_uint64()
        _check(load().huff_wenc_bits(self.h, tree.h, C.byref(v)))
        return v.value

    def pack(self, tree: WideTree, d_out: int, out_cap: int) -> int:
        v = C.c_uint64()
        _check(load().huff_wenc_pack(self.h, tree.h, C.c_void_p(d_out), out_cap, C.byref(v)))
        return v.value

    def decode(self, tree: WideTree, d_comp: int, d_out: int):
        _check(load().huff_wenc_decode(self.h, tree.h, C.c_void_p(d_comp), C.c_void_p(d_out)))


def decompress_dev(ctx, tree: WideTree, d_comp: int, comp_bytes: int, padding: int, d_out: int,
                   out_cap_letters: int) -> int:
    """comp.rs:487-519 on a device stream without a restart index -> letters written"""
    n = C.c_size_t()
    rc = load().huff_dev_wdecompress(ctx.h, tree.h, C.c_void_p(d_comp), comp_bytes, padding,
                                     C.c_void_p(d_out) if d_out else None, out_cap_letters, C.byref(n))
    if not d_out and rc == _lib.E_BUFFER_TOO_SMALL:
        return n.value
    _check(rc)
    return n.value
