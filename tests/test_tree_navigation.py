"""Walking the tree through the C ABI (huff_tree_root, huff_branch_children,
huff_branch_leaf, huff_branch_code) against the oracle, on the CPU.

The reference exposes the tree as HuffTree::root (tree_inner.rs:322-325),
HuffBranch::leaf / left_child / right_child / has_children / children_iter
(branch.rs:207-279) and HuffLeaf::letter / weight / code (leaf.rs:61-73),
with codes set on every branch below the root (tree_inner.rs:422-440) and a
single-leaf root coded [0] (tree_inner.rs:310-315). A walk of the product's
tree must serialise to the oracle's as_bin (the reference's own preorder
walk over children_iter, tree_inner.rs:632-668), give every branch its path
as its code, and carry weights that add up (leaf weights = the letters'
weights; 0 after try_from_bin, tree_inner.rs:446-447).
"""
import numpy as np
import pytest

from test_host_parity import KINDS, random_weights


def tree_of(H, data: bytes):
    """HuffTree::from_weights of the bytes' counts (counted on the host: no GPU here)"""
    w = np.bincount(np.frombuffer(data, np.uint8), minlength=256).astype(np.uint64)
    return H.HuffTree.from_weights(H.ByteWeights.from_array(w))


def walk(b, path, out):
    """preorder over children_iter: as_bin bits, and per branch its record"""
    leaf = b.leaf()
    out.append((path, leaf.letter(), leaf.weight(), leaf.code(), b.has_children()))
    it = b.children_iter()
    if it is None:
        assert b.left_child() is None and b.right_child() is None and leaf.letter() is not None
        return "0" + format(leaf.letter(), "08b")
    assert leaf.letter() is None
    lft, rgt = list(it)
    assert b.left_child().leaf().code() == lft.leaf().code() and b.right_child().leaf().code() == rgt.leaf().code()
    return "1" + walk(lft, path + "0", out) + walk(rgt, path + "1", out)


@pytest.mark.parametrize("kind", KINDS)
def test_walk_matches_oracle(H, O, kind):
    rng = np.random.default_rng(7 + KINDS.index(kind))
    for _ in range(25):
        w = random_weights(rng, kind)
        t = H.HuffTree.from_weights(H.ByteWeights.from_array(w))
        ot = O.Tree.from_weights(O.weights_from_array(w))
        recs = []
        assert walk(t.root(), "", recs) == ot.as_bin()
        root_path, _, root_w, root_code, root_kids = recs[0]
        assert root_w == t.root_weight()
        assert root_code == (None if root_kids else "0")
        by_path = {p: (letter, wt) for p, letter, wt, _, _ in recs}
        for p, letter, wt, code, kids in recs[1:]:
            assert code == p  # every branch below the root carries its path
            if kids:
                assert wt == by_path[p + "0"][1] + by_path[p + "1"][1]
            else:
                # a letter's leaf weight is its weight, except the duplicated
                # byte-0 leaf of the iterator quirk (weights.rs:423-441), which
                # carries byte 0's weight again
                assert wt == int(w[letter])
        assert sum(1 for r in recs if not r[4]) == t.num_leaves()
        # read_codes keeps the later leaf of a duplicated letter (overwrite)
        codes = {}
        for p, letter, _, _, kids in recs:
            if not kids:
                codes[letter] = p if p else "0"
        assert codes == t.read_codes() == ot.codes()
        # the same walk over a tree read back from its bits: weights 0
        t2 = H.HuffTree.try_from_bin(t.as_bin())
        recs2 = []
        assert walk(t2.root(), "", recs2) == ot.as_bin()
        assert all(r[2] == 0 for r in recs2)
        assert [(r[0], r[1], r[3]) for r in recs2] == [(r[0], r[1], r[3]) for r in recs]


def test_known_answer_ghhiii(H):
    """tree_inner.rs:356-419 read_codes doc: 'ghhiii' -> i 0, h 11, g 10"""
    t = tree_of(H, b"ghhiii")
    root = t.root()
    assert root.has_children() and root.leaf().letter() is None and root.leaf().code() is None
    assert root.leaf().weight() == 6
    i, joint = root.left_child(), root.right_child()
    assert (i.leaf().letter(), i.leaf().weight(), i.leaf().code()) == (ord("i"), 3, "0")
    assert (joint.leaf().letter(), joint.leaf().weight(), joint.leaf().code()) == (None, 3, "1")
    g, h = joint.children_iter()
    assert (g.leaf().letter(), g.leaf().weight(), g.leaf().code()) == (ord("g"), 1, "10")
    assert (h.leaf().letter(), h.leaf().weight(), h.leaf().code()) == (ord("h"), 2, "11")
    assert i.children_iter() is None and not i.has_children()


def test_single_leaf_root(H):
    """tree_inner.rs:310-315: a one-letter tree's root is its leaf, code [0]"""
    t = tree_of(H, b"zzzz")
    root = t.root()
    assert not root.has_children() and root.children_iter() is None
    leaf = root.leaf()
    assert (leaf.letter(), leaf.weight(), leaf.code()) == (ord("z"), 4, "0")


def test_bad_branch_ids(H):
    """ids the tree does not hold and a null tree: HUFF_E_INVALID_ARG (1); a
    short bit buffer: HUFF_E_BUFFER_TOO_SMALL with the length it needs"""
    import ctypes as C

    from huff_coding import _lib

    L = _lib.load()
    t = tree_of(H, b"abbccc")
    lft, rgt = C.c_int32(), C.c_int32()
    for bad in (-1, -7, 100000):
        assert L.huff_branch_children(t.h, bad, C.byref(lft), C.byref(rgt)) == 1
        assert L.huff_branch_leaf(t.h, bad, None, None, None) == 1
    b = C.c_int32()
    assert L.huff_tree_root(None, C.byref(b)) == 1
    leaf = t.root().left_child()
    while leaf.has_children():
        leaf = leaf.left_child()
    n, has = C.c_size_t(), C.c_int()
    code = leaf.leaf().code()
    assert len(code) >= 1
    assert L.huff_branch_code(t.h, leaf._node, None, 0, C.byref(n), C.byref(has)) not in (0, 1)
    assert n.value == len(code)


def wwalk(b, lt, path, out):
    """the wide tree's preorder walk: as_bin with W*8 letter bits (big-endian
    two's complement, letter.rs as_be_bytes)"""
    leaf = b.leaf()
    out.append((path, leaf.letter(), leaf.weight(), leaf.code(), b.has_children()))
    it = b.children_iter()
    if it is None:
        raw = int(leaf.letter()).to_bytes(lt.width, "big", signed=lt.signed)
        return "0" + "".join(format(x, "08b") for x in raw)
    lft, rgt = list(it)
    return "1" + wwalk(lft, lt, path + "0", out) + wwalk(rgt, lt, path + "1", out)


@pytest.mark.parametrize("dtype,lbits", [(np.int16, 16), (np.uint32, 32), (np.int64, 64)])
def test_wide_walk_matches_oracle(O, dtype, lbits):
    """HuffTree<L>::root and its branches for wider letters (letter.rs:41-60)
    against the oracle's as_bin; leaf weights are the letters' weights, joint
    weights the sums, codes the paths; a tree read back from bits: weights 0"""
    import huff_coding.wide as W

    rng = np.random.default_rng(100 + lbits)
    info = np.iinfo(dtype)
    for _ in range(15):
        k = int(rng.integers(1, 300))
        letters = np.unique(rng.integers(info.min, info.max, k, dtype=dtype, endpoint=True))
        rng.shuffle(letters)
        weights = rng.integers(1, 6, letters.size)
        wmap = dict(zip(letters.tolist(), weights.tolist()))
        t = W.WideTree.from_weights(list(wmap.items()), dtype)
        ot = O.Tree.from_leaves(letters.astype(np.int64).view(np.uint64) & np.uint64((1 << lbits) - 1)
                                if lbits < 64 else letters.view(np.uint64), weights)
        recs = []
        assert wwalk(t.root(), t.ltype, "", recs) == ot.as_bin(lbits)
        assert recs[0][3] == (None if recs[0][4] else "0")
        by_path = {p: wt for p, _, wt, _, _ in recs}
        for p, letter, wt, code, kids in recs[1:]:
            assert code == p
            assert wt == (by_path[p + "0"] + by_path[p + "1"] if kids else wmap[letter])
        assert recs[0][2] == int(weights.sum())
        t2 = W.WideTree.try_from_bin(t.as_bin(), dtype)
        recs2 = []
        assert wwalk(t2.root(), t2.ltype, "", recs2) == ot.as_bin(lbits)
        assert all(r[2] == 0 for r in recs2)
