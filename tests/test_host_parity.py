"""Product host logic (C++ behind the C ABI) vs the oracle, on the CPU.

Covers everything of the hot path that runs on the host by design: the
ByteWeights iterator/merge quirks, the HuffTree build with the reference's
BinaryHeap tie order, read_codes overwrite semantics, tree <-> bits and the
CompressData byte container. No GPU call is made here.
"""
import numpy as np
import pytest


def random_weights(rng, kind):
    w = np.zeros(256, np.uint64)
    if kind == "sparse":
        idx = rng.choice(256, size=rng.integers(1, 12), replace=False)
        w[idx] = rng.integers(1, 50, idx.size)
    elif kind == "ties":
        idx = rng.choice(256, size=rng.integers(2, 200), replace=False)
        w[idx] = rng.integers(1, 4, idx.size)  # massive ties
    elif kind == "full":
        w[:] = rng.integers(1, 1 << 40, 256)
    elif kind == "fib":
        f = [1, 1]
        while len(f) < 40:
            f.append(f[-1] + f[-2])
        idx = rng.choice(256, size=40, replace=False)
        w[idx] = f
    elif kind == "zero_no255":  # §C.1 duplicate leaf of byte 0
        idx = rng.choice(np.arange(1, 255), size=rng.integers(0, 20), replace=False)
        w[idx] = rng.integers(1, 9, idx.size)
        w[0] = rng.integers(1, 9)
    return w


KINDS = ["sparse", "ties", "full", "fib", "zero_no255"]


@pytest.mark.parametrize("kind", KINDS)
def test_tree_matches_oracle(H, O, kind):
    rng = np.random.default_rng(hash(kind) % 1000)
    for _ in range(40):
        w = random_weights(rng, kind)
        bw = H.ByteWeights.from_array(w)
        ow = O.weights_from_array(w)
        assert list(bw) == ow.iter()
        t = H.HuffTree.from_weights(bw)
        ot = O.Tree.from_weights(ow)
        assert t.read_codes() == ot.codes()
        assert t.as_bin() == ot.as_bin()
        assert t.num_leaves() == ot.num_leaves()
        assert t.root_weight() == int(w.sum()) + (int(w[0]) if (w[0] and not w[255]) else 0)
        t2 = H.HuffTree.try_from_bin(t.as_bin())
        assert t2.read_codes() == t.read_codes()
        assert t2.root_weight() == 0  # weights are not serialised (tree_inner.rs:137-144)


def test_known_answers_through_product(H, golden):
    pinned, _ = golden
    for c in pinned["codes"]:
        data = c["input_ascii"].encode()
        t = H.HuffTree.from_weights(H.ByteWeights.from_array(np.bincount(np.frombuffer(data, np.uint8), minlength=256)))
        assert {chr(k): v for k, v in t.read_codes().items()} == c["codes"]
    for c in pinned["tree_bits"]:
        data = c["input_ascii"].encode() if "input_ascii" in c else bytes.fromhex(c["input_hex"])
        t = H.HuffTree.from_weights(H.ByteWeights.from_array(np.bincount(np.frombuffer(data, np.uint8), minlength=256)))
        assert H.bitvec_str(t.as_bin()) == c["bits"]


def test_weights_add_quirk(H, O):
    rng = np.random.default_rng(5)
    for _ in range(200):
        a = random_weights(rng, rng.choice(KINDS))
        b = random_weights(rng, rng.choice(KINDS))
        if rng.random() < 0.2:
            a[:] = 0
        x = H.ByteWeights.from_array(a)
        x += H.ByteWeights.from_array(b)
        y = O.weights_from_array(a)
        y += O.weights_from_array(b)
        assert (x.as_array() == y.as_array()).all()
        assert x.len() == y.len


def test_empty_weights(H):
    with pytest.raises(H.HuffPanic) as e:
        H.HuffTree.from_weights(H.ByteWeights.new())
    assert "provided empty weights" in str(e.value)


def test_try_from_bin_errors(H):
    with pytest.raises(H.FromBinError) as e:
        H.HuffTree.try_from_bin("")
    assert "too small" in str(e.value)
    with pytest.raises(H.FromBinError) as e:
        H.HuffTree.try_from_bin("0" + "01100001" + "1")
    assert "too big" in str(e.value)
    with pytest.raises(H.FromBinError):
        H.HuffTree.try_from_bin("1" + "0" + "0110")
    # deep chain of joints (no recursion in the product parser)
    with pytest.raises(H.FromBinError):
        H.HuffTree.try_from_bin("1" * 5000)


def test_container_roundtrip_and_errors(H, O):
    rng = np.random.default_rng(9)
    for _ in range(50):
        w = random_weights(rng, rng.choice(KINDS))
        t = H.HuffTree.from_weights(H.ByteWeights.from_array(w))
        comp = bytes(rng.integers(0, 256, rng.integers(1, 40), dtype=np.uint8))
        pad = int(rng.integers(0, 8))
        cd = H.CompressData.new(comp, pad, t)
        raw = cd.to_bytes()
        ot = O.Tree.from_weights(O.weights_from_array(w))
        assert raw == O.to_bytes(comp, pad, ot)
        cd2 = H.CompressData.try_from_bytes(raw)
        assert cd2.comp_bytes() == comp and cd2.padding_bits() == pad
        assert cd2.huff_tree().read_codes() == t.read_codes()
        assert not cd2.has_index()
    # errors / panics (comp.rs:128-184, 55-68)
    with pytest.raises(H.CompressedDataFromBytesError, match="slice is empty"):
        H.CompressData.try_from_bytes(b"")
    with pytest.raises(H.CompressedDataFromBytesError, match="tree length"):
        H.CompressData.try_from_bytes(b"\x00\x00\x00")
    with pytest.raises(H.HuffPanic, match="at least 2"):
        H.CompressData.try_from_bytes(b"\x00\x00\x00\x00\x01\xff")
    with pytest.raises(H.CompressedDataFromBytesError, match="too short to read tree"):
        H.CompressData.try_from_bytes(b"\x00\x00\x00\x00\x09\xff")
    with pytest.raises(H.CompressedDataFromBytesError, match="invalid tree"):
        H.CompressData.try_from_bytes(b"\x00\x00\x00\x00\x02\xff\xff\x00")
    good = bytes.fromhex("370000000498e61310bc00")
    with pytest.raises(H.HuffPanic, match="comp_bytes are empty"):
        H.CompressData.try_from_bytes(good[:9])
    with pytest.raises(H.HuffPanic, match="padding bits"):
        H.CompressData.try_from_bytes(bytes([0x3F]) + good[1:])
    t = H.CompressData.try_from_bytes(good).huff_tree()
    with pytest.raises(H.HuffPanic):
        H.CompressData.new(b"", 0, t)
    with pytest.raises(H.HuffPanic):
        H.CompressData.new(b"\x00", 8, t)


def test_ration_bounds_via_oracle_semantics(O):
    """utils.rs:6-28: the last ration takes the remainder; n < T -> one ration"""
    data = bytes([0, 1] * 12)
    assert O.weights_threaded(data, 12).w[0] == 23      # §C.2 double count
    assert O.weights_threaded(data, 100).w[0] == 12     # one ration: no merge


def test_parse_block_size(H):
    assert H.parse_block_size("2G") == 2_000_000_000
    assert H.parse_block_size("64ki") == 65536
    assert H.parse_block_size("3Mi") == 3 * 1048576
    assert H.parse_block_size("12") == 12
    assert H.parse_block_size("5k") == 5000
    for bad in ("0", "", "k", "12x", "1.5G", "99999999999999999999999"):
        with pytest.raises(H.HuffError):
            H.parse_block_size(bad)
