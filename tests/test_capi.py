"""The C ABI boundary: the library loads and exports every symbol the header
declares, and GPU entry points fail loudly (no CPU fallback) without a GPU."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in sorted(os.listdir(os.path.join(ROOT, "include")))
           if h.endswith(".h")]
LIB = os.path.join(ROOT, "huff-encoding_amd", "lib", "libhuffgpu.so")


def declared():
    src = "".join(open(h).read() for h in HEADERS)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(huff_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared()
    assert len(names) >= 45
    for must in ("huff_weights_from_bytes", "huff_tree_from_weights", "huff_compress_with_tree",
                 "huff_decompress", "huff_cd_to_bytes", "huff_cd_try_from_bytes", "huff_enc_pack",
                 "huff_file_compress", "huff_file_decompress", "huff_wtree_from_weights",
                 "huff_wcompress_with_tree", "huff_wdecompress", "huff_wweights_map"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    import huff_coding._lib as L

    bound = {name for name, _, _ in L.SIGNATURES}
    assert set(declared()) == bound


def test_no_gpu_fails_loudly(H):
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(H.HuffError) as e:
        H.Context(0)
    assert e.value.code == 17  # HUFF_E_NO_DEVICE
    with pytest.raises(H.HuffError):
        H.compress(b"abbccc")


def test_host_cpp_tests():
    """C++ test binary mirroring the reference's own tests (tree_init.rs,
    tree_bin.rs, weights doctests) against the product host code."""
    import subprocess

    pkg = os.path.join(ROOT, "huff-encoding_amd")
    subprocess.run(["make", "-s", "-C", pkg, os.path.join(pkg, "build", "test_host")], check=True)
    r = subprocess.run([os.path.join(pkg, "build", "test_host")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout


def test_host_cpp_tests_under_sanitizers():
    """the same host tests built with AddressSanitizer + UBSan (host code only:
    GPU sanitizers are not available on the pool): no leak, overflow or UB
    report, every check passing"""
    import shutil
    import subprocess

    if shutil.which("g++") is None:
        pytest.skip("no g++")
    pkg = os.path.join(ROOT, "huff-encoding_amd")
    subprocess.run(["make", "-s", "-C", pkg, "asan"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([os.path.join(pkg, "build", "test_host_asan")], capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout and "runtime error" not in r.stderr
