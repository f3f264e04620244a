"""ctypes view of the CPU oracle (oracle/huff_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker or the timed CPU restatement of
the reference. The product package (huff-encoding_amd/) never imports it.

The restatement follows k-xlsx/huff-encoding (see huff_oracle.c for the
file:line of every function). Parity status: pinned by the reference's own
doctest/test known answers (tests/golden/reference_pinned.json).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle.so")

OK = 0
E_EMPTY_WEIGHTS = 2
E_MISSING_LETTER = 3
E_FROM_BIN = 4
E_FROM_BYTES = 5
E_BUFFER = 6
E_MISSING_HEADER = 11
E_INVALID_HEADER = 12
E_EMPTY_COMP = 14
E_PADDING = 15
E_TREE_LEN = 16


class OracleError(Exception):
    def __init__(self, code: int, msg: str = ""):
        super().__init__(f"oracle error {code}: {msg}")
        self.code = code
        self.msg = msg


def build() -> str:
    """Compile the oracle with its Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        u8p = C.POINTER(C.c_uint8)
        u64p = C.POINTER(C.c_uint64)
        sz = C.c_size_t
        L.orc_weights_from_bytes.argtypes = [u8p, sz, C.c_void_p]
        L.orc_weights_iter.argtypes = [C.c_void_p, u8p, u64p]
        L.orc_weights_iter.restype = sz
        L.orc_weights_add.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_weights_threaded.argtypes = [u8p, sz, sz, C.c_void_p]
        L.orc_tree_from_leaves.argtypes = [u64p, u64p, sz]
        L.orc_tree_from_leaves.restype = C.c_void_p
        L.orc_tree_from_weights.argtypes = [C.c_void_p]
        L.orc_tree_from_weights.restype = C.c_void_p
        L.orc_tree_free.argtypes = [C.c_void_p]
        L.orc_tree_num_leaves.argtypes = [C.c_void_p]
        L.orc_tree_num_leaves.restype = sz
        L.orc_tree_codes.argtypes = [C.c_void_p, C.c_uint32, u8p, sz, C.POINTER(C.c_uint32)]
        L.orc_tree_codes.restype = C.c_uint32
        L.orc_tree_as_bin.argtypes = [C.c_void_p, C.c_uint32, u8p]
        L.orc_tree_as_bin.restype = sz
        L.orc_tree_try_from_bin.argtypes = [u8p, sz, C.c_uint32, C.POINTER(C.c_void_p), C.POINTER(C.c_char_p)]
        L.orc_compress_with_tree.argtypes = [u8p, sz, C.c_void_p, u8p, sz, C.POINTER(sz), u8p, u8p]
        L.orc_compressed_bits.argtypes = [u8p, sz, C.c_void_p]
        L.orc_compressed_bits.restype = C.c_uint64
        L.orc_decompress.argtypes = [u8p, sz, C.c_uint8, C.c_void_p, u8p, sz]
        L.orc_decompress.restype = sz
        L.orc_to_bytes.argtypes = [u8p, sz, C.c_uint8, C.c_void_p, u8p, sz]
        L.orc_to_bytes.restype = sz
        L.orc_try_from_bytes.argtypes = [u8p, sz, C.POINTER(C.c_void_p), u8p, C.POINTER(sz), C.POINTER(sz), C.POINTER(C.c_char_p)]
        L.orc_cli_compress.argtypes = [u8p, sz, sz, u8p, sz, C.POINTER(sz)]
        L.orc_cli_decompress.argtypes = [u8p, sz, sz, u8p, sz, C.POINTER(sz)]
        L.orc_offset_bytes.argtypes = [u8p, sz, sz, u8p]
        L.orc_offset_bytes.restype = sz
        L.orc_fast_encode.argtypes = [u8p, sz, u64p, u8p, C.c_int, C.c_uint64, u8p, sz, C.POINTER(C.c_uint64)]
        L.orc_fast_hist.argtypes = [u8p, sz, C.c_int, u64p]
        L.orc_wcompress_with_tree.argtypes = [u64p, sz, C.c_void_p, u8p, sz, C.POINTER(sz), u8p, C.POINTER(sz)]
        L.orc_wdecompress.argtypes = [u8p, sz, C.c_uint8, C.c_void_p, u64p, sz]
        L.orc_wdecompress.restype = sz
        L.orc_fast_encode_idx.argtypes = [u8p, sz, u64p, u8p, C.c_int, C.c_uint64, u8p, sz,
                                          C.POINTER(C.c_uint64), u64p]
        L.orc_fast_decode.argtypes = [u8p, sz, C.c_void_p, sz, C.c_int, u64p, u8p]
        L.orc_splitmix64.argtypes = [C.c_uint64, C.c_uint64]
        L.orc_splitmix64.restype = C.c_uint64
        L.orc_gen_uniform.argtypes = [C.c_uint64, C.c_uint64, sz, u8p]
        L.orc_zipf_cdf.argtypes = [C.c_double, u64p]
        L.orc_gen_zipf.argtypes = [C.c_uint64, C.c_uint64, sz, u64p, u8p]
        L.orc_gen_text.argtypes = [C.c_uint64, C.c_uint64, sz, u8p]
        L.orc_now.restype = C.c_double
        _lib = L
    return _lib


def _u8(a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return a, a.ctypes.data_as(C.POINTER(C.c_uint8))


def _as_bytes(data) -> np.ndarray:
    if isinstance(data, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(data), dtype=np.uint8)
    return np.ascontiguousarray(data, dtype=np.uint8)


class Weights(C.Structure):
    """weights.rs:174-178 ByteWeights {weights: [usize;256], len}"""
    _fields_ = [("w", C.c_uint64 * 256), ("len", C.c_uint64)]

    def get(self, b: int):
        v = self.w[b]
        return None if v == 0 else v

    def as_array(self) -> np.ndarray:
        return np.ctypeslib.as_array(self.w).copy()

    def iter(self):
        l = np.zeros(257, np.uint8)
        w = np.zeros(257, np.uint64)
        n = lib().orc_weights_iter(C.byref(self), l.ctypes.data_as(C.POINTER(C.c_uint8)),
                                   w.ctypes.data_as(C.POINTER(C.c_uint64)))
        return [(int(l[i]), int(w[i])) for i in range(n)]

    def __iadd__(self, other: "Weights"):
        lib().orc_weights_add(C.byref(self), C.byref(other))
        return self


def weights_from_bytes(data) -> Weights:
    a, p = _u8(_as_bytes(data))
    w = Weights()
    lib().orc_weights_from_bytes(p, a.size, C.byref(w))
    return w


def weights_threaded(data, thread_num: int) -> Weights:
    a, p = _u8(_as_bytes(data))
    w = Weights()
    lib().orc_weights_threaded(p, a.size, thread_num, C.byref(w))
    return w


def weights_from_array(arr) -> Weights:
    w = Weights()
    for i, v in enumerate(arr):
        w.w[i] = int(v)
    w.len = int(sum(1 for v in arr if v))
    return w


class Tree:
    """tree_inner.rs HuffTree (u8 letters unless built from_leaves)."""

    def __init__(self, handle):
        self.h = handle

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_tree_free(self.h)
            self.h = None

    @staticmethod
    def from_weights(w: Weights) -> "Tree":
        h = lib().orc_tree_from_weights(C.byref(w))
        if not h:
            raise OracleError(E_EMPTY_WEIGHTS, "provided empty weights")
        return Tree(h)

    @staticmethod
    def from_leaves(letters, weights) -> "Tree":
        n = len(letters)
        if n == 0:
            raise OracleError(E_EMPTY_WEIGHTS, "provided empty weights")
        la = np.asarray(letters, np.uint64)
        wa = np.asarray(weights, np.uint64)
        h = lib().orc_tree_from_leaves(la.ctypes.data_as(C.POINTER(C.c_uint64)),
                                       wa.ctypes.data_as(C.POINTER(C.c_uint64)), n)
        return Tree(h)

    def num_leaves(self) -> int:
        return lib().orc_tree_num_leaves(self.h)

    def codes(self, nletters: int = 256) -> dict:
        stride = 512
        bits = np.zeros(nletters * stride, np.uint8)
        lens = np.zeros(nletters, np.uint32)
        lib().orc_tree_codes(self.h, nletters, bits.ctypes.data_as(C.POINTER(C.c_uint8)), stride,
                             lens.ctypes.data_as(C.POINTER(C.c_uint32)))
        out = {}
        for l in range(nletters):
            if lens[l]:
                out[l] = "".join(str(int(b)) for b in bits[l * stride: l * stride + lens[l]])
        return out

    def code_table(self):
        """(code u64 right-aligned, len u8) arrays for the fast checker."""
        c = self.codes()
        code = np.zeros(256, np.uint64)
        ln = np.zeros(256, np.uint8)
        for k, s in c.items():
            code[k] = int(s, 2)
            ln[k] = len(s)
        return code, ln

    def as_bin(self, letter_bits: int = 8) -> str:
        n = lib().orc_tree_as_bin(self.h, letter_bits, None)
        b = np.zeros(max(n, 1), np.uint8)
        lib().orc_tree_as_bin(self.h, letter_bits, b.ctypes.data_as(C.POINTER(C.c_uint8)))
        return "".join(str(int(x)) for x in b[:n])

    @staticmethod
    def try_from_bin(bits: str, letter_bits: int = 8) -> "Tree":
        a = np.array([1 if ch == "1" else 0 for ch in bits] or [0], np.uint8)
        h = C.c_void_p()
        msg = C.c_char_p()
        e = lib().orc_tree_try_from_bin(a.ctypes.data_as(C.POINTER(C.c_uint8)), len(bits), letter_bits,
                                        C.byref(h), C.byref(msg))
        if e:
            raise OracleError(e, msg.value.decode() if msg.value else "")
        return Tree(h.value)


def bitvec_str(bits: str) -> str:
    """bitvec Display: groups of 8 separated by ', ' inside brackets."""
    return "[" + ", ".join(bits[i:i + 8] for i in range(0, len(bits), 8)) + "]"


def pack_bits(bits: str) -> bytes:
    out = bytearray((len(bits) + 7) // 8)
    for i, ch in enumerate(bits):
        if ch == "1":
            out[i // 8] |= 0x80 >> (i % 8)
    return bytes(out)


def compress_with_tree(data, tree: Tree):
    """comp.rs:419-451 -> (comp_bytes, padding)"""
    a, p = _u8(_as_bytes(data))
    nbits = lib().orc_compressed_bits(p, a.size, tree.h)
    cap = nbits // 8 + 2
    out = np.zeros(cap, np.uint8)
    olen = C.c_size_t()
    pad = C.c_uint8()
    miss = C.c_uint8()
    e = lib().orc_compress_with_tree(p, a.size, tree.h, out.ctypes.data_as(C.POINTER(C.c_uint8)), cap,
                                     C.byref(olen), C.byref(pad), C.byref(miss))
    if e == E_MISSING_LETTER:
        raise OracleError(e, f"letter not found in codes ({miss.value})")
    if e:
        raise OracleError(e)
    return out[: olen.value].tobytes(), pad.value


def decompress(comp: bytes, padding: int, tree: Tree) -> bytes:
    a, p = _u8(_as_bytes(comp))
    n = lib().orc_decompress(p, a.size, padding, tree.h, None, 0)
    out = np.zeros(max(n, 1), np.uint8)
    lib().orc_decompress(p, a.size, padding, tree.h, out.ctypes.data_as(C.POINTER(C.c_uint8)), n)
    return out[:n].tobytes()


def wcompress_with_tree(letters, tree: Tree):
    """comp.rs:419-451 over integer letters (<= 64 bits, as u64 bit patterns)
    -> (comp_bytes, padding); OracleError(E_MISSING_LETTER) carries .index"""
    a = np.ascontiguousarray(np.asarray(letters).astype(np.uint64))
    cap = 8 * a.size * 8 + 16  # codes of any length the tests build
    out = np.zeros(cap, np.uint8)
    olen = C.c_size_t()
    pad = C.c_uint8()
    miss = C.c_size_t()
    e = lib().orc_wcompress_with_tree(a.ctypes.data_as(C.POINTER(C.c_uint64)), a.size, tree.h,
                                      out.ctypes.data_as(C.POINTER(C.c_uint8)), cap, C.byref(olen), C.byref(pad),
                                      C.byref(miss))
    if e:
        err = OracleError(e, "letter not found in codes" if e == E_MISSING_LETTER else "")
        err.index = miss.value
        raise err
    return out[:olen.value].tobytes(), pad.value


def wdecompress(comp: bytes, padding: int, tree: Tree) -> np.ndarray:
    """comp.rs:487-519 over integer letters -> u64 array"""
    a, p = _u8(_as_bytes(comp))
    n = lib().orc_wdecompress(p, a.size, padding, tree.h, None, 0)
    out = np.zeros(max(n, 1), np.uint64)
    lib().orc_wdecompress(p, a.size, padding, tree.h, out.ctypes.data_as(C.POINTER(C.c_uint64)), n)
    return out[:n]


def to_bytes(comp: bytes, padding: int, tree: Tree) -> bytes:
    a, p = _u8(_as_bytes(comp))
    n = lib().orc_to_bytes(p, a.size, padding, tree.h, None, 0)
    out = np.zeros(n, np.uint8)
    lib().orc_to_bytes(p, a.size, padding, tree.h, out.ctypes.data_as(C.POINTER(C.c_uint8)), n)
    return out.tobytes()


def try_from_bytes(data):
    a, p = _u8(_as_bytes(data))
    h = C.c_void_p()
    pad = C.c_uint8()
    off = C.c_size_t()
    ln = C.c_size_t()
    msg = C.c_char_p()
    e = lib().orc_try_from_bytes(p, a.size, C.byref(h), C.byref(pad), C.byref(off), C.byref(ln), C.byref(msg))
    if e:
        raise OracleError(e, msg.value.decode() if msg.value else "")
    return a[off.value: off.value + ln.value].tobytes(), pad.value, Tree(h.value)


def cli_compress(data, block_size: int) -> bytes:
    a, p = _u8(_as_bytes(data))
    olen = C.c_size_t()
    e = lib().orc_cli_compress(p, a.size, block_size, None, 0, C.byref(olen))
    if e:
        raise OracleError(e)
    out = np.zeros(olen.value, np.uint8)
    e = lib().orc_cli_compress(p, a.size, block_size, out.ctypes.data_as(C.POINTER(C.c_uint8)), olen.value,
                               C.byref(olen))
    if e:
        raise OracleError(e)
    return out.tobytes()


def cli_decompress(data, block_size: int) -> bytes:
    a, p = _u8(_as_bytes(data))
    olen = C.c_size_t()
    e = lib().orc_cli_decompress(p, a.size, block_size, None, 0, C.byref(olen))
    if e:
        raise OracleError(e)
    out = np.zeros(max(olen.value, 1), np.uint8)
    e = lib().orc_cli_decompress(p, a.size, block_size, out.ctypes.data_as(C.POINTER(C.c_uint8)), olen.value,
                                 C.byref(olen))
    if e:
        raise OracleError(e)
    return out[: olen.value].tobytes()


def offset_bytes(data, shift: int) -> bytes:
    a, p = _u8(_as_bytes(data))
    out = np.zeros(a.size + shift // 8 + 2, np.uint8)
    n = lib().orc_offset_bytes(p, a.size, shift, out.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out[:n].tobytes()


def fast_encode(data: np.ndarray, code: np.ndarray, ln: np.ndarray, threads: int = 8, bit_base: int = 0,
                out: np.ndarray | None = None):
    a, p = _u8(data)
    total = int(np.dot(np.bincount(a, minlength=256).astype(np.uint64), ln.astype(np.uint64))) if a.size < (1 << 16) else None
    if out is None:
        if total is None:
            w = fast_hist(a, threads)
            total = int(np.dot(w.astype(np.uint64), ln.astype(np.uint64)))
        out = np.zeros((bit_base + total + 7) // 8 + 1, np.uint8)
    tb = C.c_uint64()
    code = np.ascontiguousarray(code, np.uint64)
    ln = np.ascontiguousarray(ln, np.uint8)
    e = lib().orc_fast_encode(p, a.size, code.ctypes.data_as(C.POINTER(C.c_uint64)),
                              ln.ctypes.data_as(C.POINTER(C.c_uint8)), threads, bit_base,
                              out.ctypes.data_as(C.POINTER(C.c_uint8)), out.size, C.byref(tb))
    if e:
        raise OracleError(e)
    nbytes = (bit_base + tb.value + 7) // 8
    return out[:nbytes], tb.value


def fast_roundtrip(data: np.ndarray, threads: int = 8):
    """table-driven CPU path on all `threads`: histogram, tree, encode,
    decode (over the encoder's job split). Returns (comp, decoded, t_enc,
    t_dec) in seconds. The "cpu-fast" reference of SURVEY §8d."""
    a, p = _u8(data)
    t0 = now()
    w = fast_hist(a, threads)
    tree = Tree.from_weights(weights_from_array(w))
    code, ln = tree.code_table()
    total = int(np.dot(w.astype(np.uint64), ln.astype(np.uint64)))
    out = np.empty((total + 7) // 8 + 1, np.uint8)
    tb = C.c_uint64()
    starts = np.zeros(max(threads, 1), np.uint64)
    e = lib().orc_fast_encode_idx(p, a.size, code.ctypes.data_as(C.POINTER(C.c_uint64)),
                                  ln.ctypes.data_as(C.POINTER(C.c_uint8)), threads, 0,
                                  out.ctypes.data_as(C.POINTER(C.c_uint8)), out.size, C.byref(tb),
                                  starts.ctypes.data_as(C.POINTER(C.c_uint64)))
    if e:
        raise OracleError(e)
    t1 = now()
    nbytes = (tb.value + 7) // 8
    back = np.empty(a.size, np.uint8)
    lib().orc_fast_decode(out.ctypes.data_as(C.POINTER(C.c_uint8)), nbytes, tree.h, a.size, threads,
                          starts.ctypes.data_as(C.POINTER(C.c_uint64)), back.ctypes.data_as(C.POINTER(C.c_uint8)))
    t2 = now()
    return out[:nbytes], back, t1 - t0, t2 - t1


def fast_hist(data: np.ndarray, threads: int = 8) -> np.ndarray:
    a, p = _u8(data)
    w = np.zeros(256, np.uint64)
    lib().orc_fast_hist(p, a.size, threads, w.ctypes.data_as(C.POINTER(C.c_uint64)))
    return w


def gen_uniform(seed: int, n: int, offset: int = 0) -> np.ndarray:
    out = np.zeros(n, np.uint8)
    lib().orc_gen_uniform(seed, offset, n, out.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out


def zipf_cdf(alpha: float = 1.2) -> np.ndarray:
    cdf = np.zeros(256, np.uint64)
    lib().orc_zipf_cdf(alpha, cdf.ctypes.data_as(C.POINTER(C.c_uint64)))
    return cdf


def gen_zipf(seed: int, n: int, alpha: float = 1.2, offset: int = 0) -> np.ndarray:
    cdf = zipf_cdf(alpha)
    out = np.zeros(n, np.uint8)
    lib().orc_gen_zipf(seed, offset, n, cdf.ctypes.data_as(C.POINTER(C.c_uint64)),
                       out.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out


def gen_text(seed: int, n: int, offset: int = 0) -> np.ndarray:
    out = np.zeros(n, np.uint8)
    lib().orc_gen_text(seed, offset, n, out.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out


def now() -> float:
    return lib().orc_now()
