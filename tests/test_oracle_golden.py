"""Pin the CPU oracle against the reference's own known answers.

Every assertion here comes from reference_pinned.json, i.e. from a doctest or
test of k-xlsx/huff-encoding (file:line in each case). This is what licenses
the oracle as the checker for the GPU path.
"""
import numpy as np
import pytest


def asc(s: str) -> bytes:
    return s.encode("latin-1")


def case_input(c) -> bytes:
    return asc(c["input_ascii"]) if "input_ascii" in c else bytes.fromhex(c["input_hex"])


def test_codes(O, golden):
    pinned, _ = golden
    for c in pinned["codes"]:
        t = O.Tree.from_weights(O.weights_from_bytes(case_input(c)))
        codes = t.codes()
        assert {chr(k): v for k, v in codes.items()} == c["codes"], c["source"]


def test_tree_bits(O, golden):
    pinned, _ = golden
    for c in pinned["tree_bits"]:
        t = O.Tree.from_weights(O.weights_from_bytes(case_input(c)))
        assert O.bitvec_str(t.as_bin()) == c["bits"], c["source"]
    for c in pinned["tree_bin_first_bit"]:
        t = O.Tree.from_weights(O.weights_from_bytes(case_input(c)))
        assert int(t.as_bin()[c["index"]]) == c["bit"]


def test_to_bytes(O, golden):
    pinned, _ = golden
    for c in pinned["to_bytes"]:
        data = case_input(c)
        t = O.Tree.from_weights(O.weights_from_bytes(data))
        comp, pad = O.compress_with_tree(data, t)
        out = O.to_bytes(comp, pad, t)
        assert out.hex() == c["hex"], c["source"]
        assert pad == c["padding"]
        assert out[0] == int(c["header_byte"], 16)
        assert int.from_bytes(out[1:5], "big") == c["tree_len"]
        # try_from_bytes -> decompress gives the input back (comp.rs:105-116)
        comp2, pad2, t2 = O.try_from_bytes(out)
        assert O.decompress(comp2, pad2, t2) == data
        assert t2.codes() == t.codes()


def test_tree_init_known_answer(O, golden):
    pinned, _ = golden
    c = pinned["tree_init_known_answer"]
    t = O.Tree.from_leaves(list(range(6)), c["weights"])
    codes = t.codes(6)
    assert [codes[i] for i in range(6)] == c["codes"], c["source"]


def test_single_leaf_and_empty(O, golden):
    pinned, _ = golden
    t = O.Tree.from_leaves([0], [pinned["single_leaf"]["weight"]])
    assert t.codes(1) == {0: "0"}
    with pytest.raises(O.OracleError) as e:
        O.Tree.from_weights(O.weights_from_bytes(b""))
    assert "provided empty weights" in str(e.value)


def test_byte_weights(O, golden):
    pinned, _ = golden
    bw = pinned["byte_weights"]
    w = O.weights_from_bytes(asc(bw[0]["input_ascii"]))
    assert w.get(ord("f")) == 5 and w.len == 1
    w = O.weights_from_bytes(asc(bw[1]["input_ascii"]))
    assert w.get(ord("a")) == 5
    w = O.weights_from_bytes(bytes.fromhex(bw[2]["input_hex"]))
    pairs = w.iter()
    assert all(b == f - 1 for b, f in pairs)
    assert pairs[-1] == (0, 1)  # the wrap duplicate the doctest tolerates
    a = O.weights_from_bytes(asc(bw[3]["add"][0]))
    a += O.weights_from_bytes(asc(bw[3]["add"][1]))
    assert (a.get(ord("a")), a.get(ord("b")), a.get(ord("c"))) == (5, 5, 1)
    # threaded_from_bytes doctest (weights.rs:290-291)
    assert O.weights_threaded(b"aaaaa", 12).get(ord("a")) == 5


def test_roundtrips(O, golden):
    pinned, _ = golden
    for c in pinned["roundtrips"]:
        data = case_input(c)
        t = O.Tree.from_weights(O.weights_from_bytes(data))
        comp, pad = O.compress_with_tree(data, t)
        assert O.decompress(comp, pad, t) == data, c["source"]


def test_tree_from_bin_roundtrip(O, golden):
    pinned, _ = golden
    for c in pinned["tree_from_bin_roundtrip"]:
        t = O.Tree.from_weights(O.weights_from_bytes(case_input(c)))
        t2 = O.Tree.try_from_bin(t.as_bin())
        assert t2.codes() == t.codes(), c["source"]


def test_errors(O, golden):
    pinned, _ = golden
    errs = {e["case"]: e for e in pinned["errors"]}
    e = errs["missing letter"]
    t = O.Tree.from_weights(O.weights_from_bytes(asc(e["tree_from_ascii"])))
    with pytest.raises(O.OracleError) as ex:
        O.compress_with_tree(asc(e["compress_ascii"]), t)
    assert e["message"] in str(ex.value) and f"({ord(e['missing'])})" in str(ex.value)
    for k in ("u8 tree read as u128", "u8 tree read as u128 (doctest)"):
        e = errs[k]
        t = O.Tree.from_weights(O.weights_from_bytes(asc(e["tree_from_ascii"])))
        with pytest.raises(O.OracleError):
            O.Tree.try_from_bin(t.as_bin(), e["letter_bits"])
    for k in ("too small for u128", "empty bitvec"):
        e = errs[k]
        with pytest.raises(O.OracleError) as ex:
            O.Tree.try_from_bin(e["bits"], e["letter_bits"])
        assert e["message"] in str(ex.value)


def test_survey_crosscheck(O, golden):
    """five vectors an independent scratch restatement produced"""
    _, derived = golden
    for c in derived["survey_crosscheck"]:
        data = bytes.fromhex(c["input_hex"])
        t = O.Tree.from_weights(O.weights_from_bytes(data))
        comp, pad = O.compress_with_tree(data, t)
        assert O.to_bytes(comp, pad, t).hex() == c["to_bytes"]


def test_derived_fixtures_reproduce(O, golden):
    """the committed derived.json is what the oracle computes today"""
    _, derived = golden
    for c in derived["small"]:
        data = bytes.fromhex(c["input_hex"])
        t = O.Tree.from_weights(O.weights_from_bytes(data))
        comp, pad = O.compress_with_tree(data, t)
        assert O.to_bytes(comp, pad, t).hex() == c["to_bytes"]
        assert O.decompress(comp, pad, t) == data


def test_fast_checker_matches_faithful(O):
    """the table-driven checker used at full sizes == the bit-serial restatement"""
    rng = np.random.default_rng(3)
    for n, hi in ((1, 3), (17, 256), (1000, 5), (65537, 40), (300_000, 256)):
        data = rng.integers(0, hi, n, dtype=np.uint8)
        data[: min(n, 7)] = np.arange(min(n, 7))  # a few extra letters
        t = O.Tree.from_weights(O.weights_from_bytes(data))
        code, ln = t.code_table()
        comp, pad = O.compress_with_tree(data, t)
        for th in (1, 3, 8):
            fast, bits = O.fast_encode(data, code, ln, threads=th)
            assert fast.tobytes() == comp
        assert (O.fast_hist(data, 4) == O.weights_from_bytes(data).as_array()).all()


def test_fast_roundtrip_matches_faithful(O):
    """the cpu-fast leg of bench.py (table-driven encode + decode over the
    encoder's job split) == the bit-serial restatement, incl. codes > 12 bits
    and a single-letter input"""
    rng = np.random.default_rng(4)
    skew = np.minimum(rng.geometric(0.35, 200_000) - 1, 255).astype(np.uint8)  # long codes
    cases = [np.frombuffer(b"z" * 9000, np.uint8), rng.integers(0, 256, 100_000, dtype=np.uint8), skew,
             O.gen_text(5, 250_001)]
    for data in cases:
        t = O.Tree.from_weights(O.weights_from_bytes(data))
        comp, pad = O.compress_with_tree(data, t)
        for th in (1, 5):
            fast, back, _, _ = O.fast_roundtrip(data, th)
            assert fast.tobytes() == comp
            assert np.array_equal(back, data)
