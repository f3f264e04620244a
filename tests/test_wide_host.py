"""Wider integer letters: the host half of HuffTree<L>
(from_weights, read_codes, as_bin, try_from_bin, CompressData containers)
through the C ABI, against the reference's known answers and the oracle.
No GPU needed."""
import itertools

import numpy as np
import pytest


@pytest.fixture(scope="module")
def W():
    import huff_coding.wide as W

    return W


def test_tree_init_known_answer_every_order(W):
    """tests/tree_init.rs:8-47: six letters with weights 5,9,12,13,16,45; the
    codes are pinned for every HashMap iteration order (no weight ties)"""
    w = {0: 5, 1: 9, 2: 12, 3: 13, 4: 16, 5: 45}
    want = {0: "1100", 1: "1101", 2: "100", 3: "101", 4: "111", 5: "0"}
    for perm in itertools.permutations(range(6)):
        t = W.WideTree.from_weights([(k, w[k]) for k in perm], np.int32)
        assert t.read_codes() == want


def test_lib_rs_char_codes_every_order(W):
    """lib.rs:39-50: a x3, b x2, c x1 -> a=0, b=11, c=10 in every order"""
    for perm in itertools.permutations([(ord("a"), 3), (ord("b"), 2), (ord("c"), 1)]):
        t = W.WideTree.from_weights(list(perm), np.uint32)
        assert t.read_codes() == {ord("a"): "0", ord("b"): "11", ord("c"): "10"}


def test_single_branch(W):
    """tests/tree_init.rs:51-64: one letter (-12) is the root with code 0"""
    t = W.WideTree.from_weights({-12: 78}, np.int32)
    assert t.read_codes() == {-12: "0"}
    assert t.num_leaves() == 1


def test_empty_weights_error(W):
    """tests/tree_init.rs:66-69 should_panic 'provided empty weights'"""
    import huff_coding as H

    with pytest.raises(H.HuffPanic) as e:
        W.WideTree.from_weights({}, np.uint16)
    assert "provided empty weights" in str(e.value)


def test_u128_from_u8_bin_is_too_small(W):
    """tree_inner.rs:500-509 and tests/tree_bin.rs:17-27: a u8 tree's bits do
    not make a HuffTree<u128>; tree_inner.rs:516: [0, 1] is too small"""
    import huff_coding as H

    t8_bits = "10011000111001100001001100010"  # tree_inner.rs:621-628, abbccc
    with pytest.raises(H.FromBinError) as e:
        W.WideTree.try_from_bin(t8_bits, W.U128)
    assert "too small" in str(e.value)
    with pytest.raises(H.FromBinError):
        W.WideTree.try_from_bin("01", W.U128)
    with pytest.raises(H.FromBinError) as e:  # tests/tree_bin.rs:29-32: empty
        W.WideTree.try_from_bin("", np.uint8)
    # a u8 tree with extra bits is "too big"
    with pytest.raises(H.FromBinError) as e:
        W.WideTree.try_from_bin(t8_bits + "0", np.uint8)
    assert "too big" in str(e.value)


def test_u8_width_matches_byte_tree_bin(W):
    """tree_inner.rs:621-628: HuffTree<u8> bits for abbccc, built from the
    same (letter, weight) sequence ByteWeights iterates"""
    t = W.WideTree.from_weights([(ord("a"), 1), (ord("b"), 2), (ord("c"), 3)], np.uint8)
    assert t.as_bin() == "10011000111001100001001100010"


@pytest.mark.parametrize("dtype,lbits", [(np.int16, 16), (np.uint32, 32), (np.int64, 64)])
def test_random_trees_match_oracle(W, O, dtype, lbits):
    """from_weights / read_codes / as_bin / try_from_bin vs the oracle's
    restatement on random weight lists with many ties"""
    rng = np.random.default_rng(lbits)
    info = np.iinfo(dtype)
    for trial in range(25):
        k = int(rng.integers(1, 400))
        letters = np.unique(rng.integers(info.min, info.max, k, dtype=dtype, endpoint=True))
        rng.shuffle(letters)
        weights = rng.integers(1, 6, letters.size)  # ties on purpose
        t = W.WideTree.from_weights(list(zip(letters.tolist(), weights.tolist())), dtype)
        ot = O.Tree.from_leaves(letters.astype(np.int64).view(np.uint64) & np.uint64((1 << lbits) - 1)
                                if lbits < 64 else letters.view(np.uint64), weights)
        bits = t.as_bin()
        assert bits == ot.as_bin(lbits)
        t2 = W.WideTree.try_from_bin(bits, dtype)
        assert t2.read_codes() == t.read_codes()
        assert t2.as_bin() == bits


def test_read_codes_overwrite_from_bin(W):
    """read_codes (tree_inner.rs:356-419): a letter present twice (a tree from
    bits) keeps the later leaf's code in preorder"""
    # joint(joint(leaf 7, leaf 9), leaf 7) for u16
    leaf = lambda v: "0" + format(v, "016b")  # noqa: E731
    bits = "1" + "1" + leaf(7) + leaf(9) + leaf(7)
    t = W.WideTree.try_from_bin(bits, np.uint16)
    assert t.read_codes() == {7: "1", 9: "01"}


def test_u128_letters_roundtrip_bits(W):
    vals = [0, 1, (1 << 127) + 5, (1 << 64) + 3, 12345678901234567890123]
    w = [(v, i + 1) for i, v in enumerate(vals)]
    t = W.WideTree.from_weights(w, W.U128)
    bits = t.as_bin()
    assert len(bits) == 2 * len(vals) - 1 + 128 * len(vals)
    t2 = W.WideTree.try_from_bin(bits, W.U128)
    assert t2.read_codes() == t.read_codes()
    assert set(t.read_codes()) == set(vals)


def test_container_roundtrip_and_errors(W):
    """CompressData<L>::to_bytes / try_from_bytes (comp.rs:128-184, 279-300)"""
    import huff_coding as H

    t = W.WideTree.from_weights({-100: 1, -101: 2, -102: 3}, np.int32)
    cd = W.WideCompressData.new(b"\xbc\x00", 7, t)
    raw = cd.to_bytes()
    back = W.WideCompressData.try_from_bytes(raw, np.int32)
    assert back.comp_bytes() == b"\xbc\x00" and back.padding_bits() == 7
    assert back.huff_tree().read_codes() == t.read_codes()
    assert not back.has_index()
    with pytest.raises(H.CompressedDataFromBytesError):  # a u32 tree is no u64 tree
        W.WideCompressData.try_from_bytes(raw, np.int64)
    with pytest.raises(H.HuffPanic):
        W.WideCompressData.new(b"", 0, t)
    with pytest.raises(H.HuffPanic):
        W.WideCompressData.new(b"\x00", 8, t)


def test_deep_tree_leaf_codes(W):
    """a try_from_bin tree deeper than the first code buffer (a
    caterpillar of 5,000 u16 letters: depth 4,999) gives every leaf its full
    code through HuffBranch::leaf (leaf.rs:70-73), as the reference does,
    and walking every leaf stays linear (parent links, not a DFS per code)"""
    import time

    k = 5000
    bits = "".join("10" + format(i, "016b") for i in range(k - 1)) + "0" + format(k - 1, "016b")
    t = W.WideTree.try_from_bin(bits, np.uint16)
    b = t.root()
    t0 = time.perf_counter()
    for depth in range(k - 1):
        leaf = b.left_child().leaf()
        assert leaf.letter() == depth and leaf.code() == "1" * depth + "0"
        b = b.right_child()
    assert b.leaf().letter() == k - 1 and b.leaf().code() == "1" * (k - 1)
    assert time.perf_counter() - t0 < 30
