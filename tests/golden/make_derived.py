"""Generate tests/golden/derived.json from the C oracle.

DERIVED vectors: computed by this repo's plain-C restatement of the reference
(oracle/huff_oracle.c), NOT executed by the Rust reference (no Rust toolchain
exists in this image). The restatement itself is pinned by
reference_pinned.json. Five of the small vectors were independently computed
by the survey's scratch model and are listed under
"survey_crosscheck" for an extra consistency check.

Run:  python tests/golden/make_derived.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402


def h(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def full(data: bytes):
    t = O.Tree.from_weights(O.weights_from_bytes(data))
    comp, pad = O.compress_with_tree(data, t)
    return {"to_bytes": O.to_bytes(comp, pad, t).hex(), "padding": pad,
            "codes": {str(k): v for k, v in t.codes().items()}, "tree_bits": t.as_bin()}


def main():
    out = {"_about": __doc__.strip().splitlines()[0] + " See make_derived.py for provenance.",
           "small": [], "quirks": {}, "cli": [], "synthetic": [], "survey_crosscheck": []}

    smalls = [b"a", b"aaaa", bytes([0]), bytes([0, 1, 1]), bytes([0] * 5 + [7] * 3), bytes([255]),
              bytes([0, 255]), bytes(range(256)), b"hello world", bytes([0, 0, 1, 2, 3]), b"abracadabra",
              bytes([1, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 4, 4, 4, 4])]
    for s in smalls:
        out["small"].append({"input_hex": s.hex(), **full(s)})

    # Fibonacci weights: long codes, many heap ties
    fib = [1, 1]
    while len(fib) < 30:
        fib.append(fib[-1] + fib[-2])
    letters = list(range(1, 31))
    w = np.zeros(256, np.uint64)
    for l, f in zip(letters, fib):
        w[l] = f
    t = O.Tree.from_weights(O.weights_from_array(w))
    out["quirks"]["fibonacci30"] = {"weights": [int(x) for x in w], "codes": {str(k): v for k, v in t.codes().items()},
                                    "tree_bits": t.as_bin()}
    # equal weights (pure heap tie order)
    w = np.zeros(256, np.uint64)
    w[10:20] = 7
    w[200:205] = 3
    t = O.Tree.from_weights(O.weights_from_array(w))
    out["quirks"]["ties"] = {"weights": [int(x) for x in w], "codes": {str(k): v for k, v in t.codes().items()},
                             "tree_bits": t.as_bin()}
    # §C.1 iterator wrap duplicate and §C.2 merge double count
    out["quirks"]["iter_dup"] = {"input_hex": bytes([0, 1, 1]).hex(),
                                 "iter": O.weights_from_bytes(bytes([0, 1, 1])).iter()}
    out["quirks"]["iter_no_dup"] = {"input_hex": bytes([0, 1, 255]).hex(),
                                    "iter": O.weights_from_bytes(bytes([0, 1, 255])).iter()}
    data = bytes([0, 1] * 12)
    out["quirks"]["threaded_double_count"] = {"input_hex": data.hex(), "thread_num": 12,
                                              "w0_plain": O.weights_from_bytes(data).w[0],
                                              "w0_threaded": O.weights_threaded(data, 12).w[0],
                                              "weights_threaded": list(O.weights_threaded(data, 12).w)}

    # CLI file path (huff/src/comp.rs), incl. multi-block stitching
    rng = np.random.default_rng(7)
    texts = [O.gen_text(11, 3000), O.gen_text(12, 777), bytes(rng.integers(0, 256, 5000, dtype=np.uint8)),
             bytes([0, 1] * 40 + [3] * 9)]
    for k, d in enumerate(texts):
        d = bytes(d)
        for bs in (len(d) + 10, len(d), 1000, 64, 37):
            hff = O.cli_compress(d, bs)
            case = {"input_sha256": h(d), "input_kind": k, "n": len(d), "block_size": bs,
                    "hff_sha256": h(hff), "hff_len": len(hff)}
            try:
                rt = O.cli_decompress(hff, bs)
                case.update({"roundtrip_ok": rt == d, "decoded_sha256": h(rt), "decoded_len": len(rt)})
            except O.OracleError as e:  # e.g. -b smaller than the tree: MissingHeaderInfo
                case.update({"decompress_error": e.code})
            out["cli"].append(case)

    # synthetic generators at 1 MiB (generator definition = oracle/huff_oracle.c)
    n = 1 << 20
    for kind, gen in (("uniform", lambda: O.gen_uniform(0x5EED0001, n)),
                      ("zipf", lambda: O.gen_zipf(0x5EED0002, n)),
                      ("text", lambda: O.gen_text(0x5EED0005, n))):
        d = gen()
        t = O.Tree.from_weights(O.weights_from_bytes(d))
        code, ln = t.code_table()
        comp, bits = O.fast_encode(d, code, ln, threads=4)
        comp2, pad = O.compress_with_tree(d, t)
        assert comp.tobytes() == comp2, kind
        out["synthetic"].append({"kind": kind, "n": n, "input_sha256": h(d), "comp_sha256": h(comp2),
                                 "bits": int(bits), "maxlen": int(ln.max()), "padding": pad,
                                 "tree_bits": t.as_bin()})

    out["survey_crosscheck"] = [
        {"input_hex": "61", "to_bytes": "7700000002308000"},
        {"input_hex": "61616161", "to_bytes": "7400000002308000"},
        {"input_hex": "00", "to_bytes": "570000000380000080"},
        {"input_hex": "000101", "to_bytes": "340000000480600000c0"},
        {"input_hex": "0000000000070707", "to_bytes": "300000000480207000ffea"},
    ]
    with open(os.path.join(HERE, "derived.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
