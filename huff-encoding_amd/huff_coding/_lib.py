"""Loader for the in-tree C ABI library (lib/libhuffgpu.so, include/huffgpu.h).

PyTorch, when present, is imported first: it ships its own HIP runtime under
the same soname (libamdhip64.so.7); loading torch first makes the codec bind to
that single runtime so torch tensors, streams and RCCL share it with us.
There is no CPU fallback: a missing library or GPU raises.
"""
from __future__ import annotations

import ctypes as C
import os

try:  # plumbing only: device memory, streams, torch.distributed
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_PKG, "lib", "libhuffgpu.so")
# A/B measurements load an alternative in-tree build (e.g. lib/ab/libhuffgpu.so)
if os.environ.get("HUFF_LIB_AB"):
    LIB_PATH = os.path.join(_PKG, "lib", os.environ["HUFF_LIB_AB"], "libhuffgpu.so")

HUFF_OK = 0
E_INVALID_ARG = 1
E_EMPTY_WEIGHTS = 2
E_MISSING_LETTER = 3
E_FROM_BIN = 4
E_FROM_BYTES = 5
E_BUFFER_TOO_SMALL = 6
E_CODE_TOO_LONG = 7
E_HIP = 8
E_IO = 9
E_UNRECOGNIZED = 10
E_MISSING_HEADER = 11
E_INVALID_HEADER = 12
E_TIMEOUT = 13
E_EMPTY_COMP = 14
E_PADDING = 15
E_TREE_LEN = 16
E_NO_DEVICE = 17
E_STATE = 18
E_CORRUPT = 19

# every exported function: (name, restype, argtypes)
u8p = C.POINTER(C.c_uint8)
u64p = C.POINTER(C.c_uint64)
vp = C.c_void_p
sz = C.c_size_t
szp = C.POINTER(C.c_size_t)
i = C.c_int

SIGNATURES = [
    ("huff_last_error", C.c_char_p, []),
    ("huff_last_missing_letter", C.c_uint8, []),
    ("huff_version", C.c_char_p, []),
    ("huff_ctx_create", i, [i, C.POINTER(vp)]),
    ("huff_ctx_destroy", i, [vp]),
    ("huff_ctx_set_stream", i, [vp, vp]),
    ("huff_ctx_synchronize", i, [vp]),
    ("huff_ctx_device", i, [vp]),
    ("huff_ctx_set_timing", i, [vp, i]),
    ("huff_ctx_kernel_time", i, [vp, C.c_char_p, C.POINTER(C.c_double), u64p]),
    ("huff_ctx_reset_timing", i, [vp]),
    ("huff_weights_new", None, [vp]),
    ("huff_weights_from_bytes", i, [vp, vp, sz, vp]),
    ("huff_weights_threaded_from_bytes", i, [vp, vp, sz, sz, vp]),
    ("huff_weights_add", None, [vp, vp]),
    ("huff_weights_iter", sz, [vp, u8p, u64p]),
    ("huff_tree_from_weights", i, [vp, C.POINTER(vp)]),
    ("huff_tree_clone", i, [vp, C.POINTER(vp)]),
    ("huff_tree_free", None, [vp]),
    ("huff_tree_num_leaves", sz, [vp]),
    ("huff_tree_root_weight", C.c_uint64, [vp]),
    ("huff_tree_read_codes", i, [vp, u64p, u8p]),
    ("huff_tree_code_bits", i, [vp, C.c_uint8, u8p, sz, szp]),
    ("huff_tree_as_bin", i, [vp, u8p, sz, szp]),
    ("huff_tree_try_from_bin", i, [vp, sz, C.POINTER(vp)]),
    ("huff_tree_root", i, [vp, C.POINTER(C.c_int32)]),
    ("huff_branch_children", i, [vp, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    ("huff_branch_leaf", i, [vp, C.c_int32, C.POINTER(i), u8p, u64p]),
    ("huff_branch_code", i, [vp, C.c_int32, u8p, sz, szp, C.POINTER(i)]),
    ("huff_cd_new", i, [vp, sz, C.c_uint8, vp, C.POINTER(vp)]),
    ("huff_cd_free", None, [vp]),
    ("huff_cd_comp_bytes", i, [vp, C.POINTER(u8p), szp]),
    ("huff_cd_padding", C.c_uint8, [vp]),
    ("huff_cd_tree", vp, [vp]),
    ("huff_cd_has_index", i, [vp]),
    ("huff_cd_to_bytes", i, [vp, u8p, sz, szp]),
    ("huff_cd_try_from_bytes", i, [vp, sz, C.POINTER(vp)]),
    ("huff_compress_with_tree", i, [vp, vp, sz, vp, C.POINTER(vp)]),
    ("huff_compress_bytes", i, [vp, vp, sz, C.POINTER(vp)]),
    ("huff_decompress", i, [vp, vp, u8p, sz, szp]),
    ("huff_enc_create", i, [vp, vp, sz, C.POINTER(vp)]),
    ("huff_enc_free", None, [vp]),
    ("huff_enc_hist", i, [vp, vp]),
    ("huff_enc_hist_row", i, [vp, vp]),
    ("huff_enc_hist_launch", i, [vp]),
    ("huff_enc_bits", i, [vp, vp, u64p]),
    ("huff_enc_pack", i, [vp, vp, C.c_uint64, vp, sz, vp, sz, u64p]),
    ("huff_enc_pack_shards", i, [vp, vp, C.c_uint32, C.c_uint32, vp, vp, vp, sz, C.POINTER(vp), u64p, u64p]),
    ("huff_enc_compress", i, [vp, vp, sz, C.POINTER(vp), u64p]),
    ("huff_enc_decode", i, [vp, vp, vp, vp]),
    ("huff_dev_decompress", i, [vp, vp, vp, sz, C.c_uint8, vp, sz, szp]),
    ("huff_batch_hist", i, [vp, vp, vp, C.c_uint32, vp]),
    ("huff_batch_trees", i, [vp, vp, C.c_uint32, vp, sz, vp, vp, vp, vp]),
    ("huff_comm_unique_id", i, [vp]),
    ("huff_comm_init", i, [vp, vp, i, i, C.POINTER(vp)]),
    ("huff_comm_free", None, [vp]),
    ("huff_comm_world", i, [vp, C.POINTER(i), C.POINTER(i)]),
    ("huff_mgpu_compress", i, [vp, vp, vp, sz, C.POINTER(vp), u64p, u64p, u64p]),
    ("huff_mgpu_exchange_launch", i, [vp, vp]),
    ("huff_mgpu_pack_rows", i, [vp, vp, i, i, vp, sz, C.POINTER(vp), u64p, u64p, u64p]),
    ("huff_dev_generate", i, [vp, i, C.c_uint64, C.c_uint64, u64p, vp, sz]),
    ("huff_dev_calibrate", i, [vp, vp, vp, sz, i, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    ("huff_dev_alloc", i, [vp, sz, C.POINTER(vp)]),
    ("huff_dev_free", i, [vp, vp]),
    ("huff_memcpy_htod", i, [vp, vp, vp, sz]),
    ("huff_memcpy_dtoh", i, [vp, vp, vp, sz]),
    ("huff_file_compress", i, [vp, C.c_char_p, C.c_char_p, sz]),
    ("huff_file_decompress", i, [vp, C.c_char_p, C.c_char_p, sz]),
    ("huff_parse_block_size", i, [C.c_char_p, szp]),
    # include/huffgpu_wide.h
    ("huff_wtree_from_weights", i, [C.c_uint32, vp, vp, sz, C.POINTER(vp)]),
    ("huff_wtree_clone", i, [vp, C.POINTER(vp)]),
    ("huff_wtree_free", None, [vp]),
    ("huff_wtree_width", C.c_uint32, [vp]),
    ("huff_wtree_num_leaves", sz, [vp]),
    ("huff_wtree_read_codes", i, [vp, vp, vp, vp, sz, szp]),
    ("huff_wtree_as_bin", i, [vp, vp, sz, szp]),
    ("huff_wtree_try_from_bin", i, [C.c_uint32, vp, sz, C.POINTER(vp)]),
    ("huff_wtree_root", i, [vp, C.POINTER(C.c_int32)]),
    ("huff_wbranch_children", i, [vp, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    ("huff_wbranch_leaf", i, [vp, C.c_int32, C.POINTER(i), vp, u64p]),
    ("huff_wbranch_code", i, [vp, C.c_int32, u8p, sz, szp, C.POINTER(i)]),
    ("huff_wweights_map", i, [vp, C.c_uint32, vp, sz, vp, vp, sz, szp]),
    ("huff_wcd_new", i, [vp, sz, C.c_uint8, vp, C.POINTER(vp)]),
    ("huff_wcd_free", None, [vp]),
    ("huff_wcd_comp_bytes", i, [vp, C.POINTER(u8p), szp]),
    ("huff_wcd_padding", C.c_uint8, [vp]),
    ("huff_wcd_tree", vp, [vp]),
    ("huff_wcd_has_index", i, [vp]),
    ("huff_wcd_to_bytes", i, [vp, vp, sz, szp]),
    ("huff_wcd_try_from_bytes", i, [C.c_uint32, vp, sz, C.POINTER(vp)]),
    ("huff_wcompress_with_tree", i, [vp, vp, sz, vp, C.POINTER(vp)]),
    ("huff_wcompress", i, [vp, C.c_uint32, vp, sz, C.POINTER(vp)]),
    ("huff_wdecompress", i, [vp, vp, vp, sz, szp]),
    ("huff_last_missing_wletter", i, [vp, C.POINTER(C.c_uint32)]),
    ("huff_wenc_create", i, [vp, C.c_uint32, vp, sz, C.POINTER(vp)]),
    ("huff_wenc_free", None, [vp]),
    ("huff_wenc_bits", i, [vp, vp, vp]),
    ("huff_wenc_pack", i, [vp, vp, vp, sz, vp]),
    ("huff_wenc_decode", i, [vp, vp, vp, vp]),
    ("huff_dev_wdecompress", i, [vp, vp, vp, sz, C.c_uint8, vp, sz, szp]),
]

_lib = None


def load():
    """Load libhuffgpu.so (build it first with `make -C huff-encoding_amd`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run `make -C huff-encoding_amd` (the codec has no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    m = load().huff_last_error()
    return m.decode() if m else ""
