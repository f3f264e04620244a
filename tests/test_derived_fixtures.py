"""The frozen derived vectors (tests/golden/derived.json, made by
tests/golden/make_derived.py from the oracle) checked against the oracle and
the product host code on the CPU, and against the GPU path on the GPU:

* quirks — the ByteWeights iterator's byte-0 re-yield and the threaded merge
  double count (weights.rs:396-441, :374-387, :293-319), heap tie order and
  Fibonacci depths (branch_heap.rs, tree_inner.rs:281-320);
* cli — `.hff` bytes of huff/src/comp.rs:177-227 (+ huff/src/utils.rs:2-25
  multi-block stitching) at several block sizes;
* synthetic — the 1 MiB configs[0]-size inputs of the three generators and
  their compressed streams (sha256).

The derived vectors are the oracle's, not a Rust run (the
reference cannot be built here); the oracle itself is pinned by the
reference's own known answers (reference_pinned.json, test_oracle_golden.py).
"""
import hashlib
import os
import tempfile

import numpy as np
import pytest


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def cli_inputs(O):
    """the inputs make_derived.py used for the `cli` section (by input_kind)"""
    rng = np.random.default_rng(7)
    return [bytes(O.gen_text(11, 3000)), bytes(O.gen_text(12, 777)),
            bytes(rng.integers(0, 256, 5000, dtype=np.uint8)), bytes([0, 1] * 40 + [3] * 9)]


def synthetic_input(O, kind, n):
    return {"uniform": lambda: O.gen_uniform(0x5EED0001, n), "zipf": lambda: O.gen_zipf(0x5EED0002, n),
            "text": lambda: O.gen_text(0x5EED0005, n)}[kind]()


def codes_of(c):
    return {int(k): v for k, v in c["codes"].items()}


# ---- CPU: oracle and product host code ---------------------------------------

def test_quirks_oracle_and_host(H, O, golden):
    _, derived = golden
    q = derived["quirks"]
    for name in ("fibonacci30", "ties"):
        w = np.array(q[name]["weights"], np.uint64)
        ot = O.Tree.from_weights(O.weights_from_array(w))
        assert ot.codes() == codes_of(q[name]) and ot.as_bin() == q[name]["tree_bits"], name
        t = H.HuffTree.from_weights(H.ByteWeights.from_array(w))
        assert t.read_codes() == codes_of(q[name]) and t.as_bin() == q[name]["tree_bits"], name
    for name in ("iter_dup", "iter_no_dup"):
        data = bytes.fromhex(q[name]["input_hex"])
        want = [tuple(p) for p in q[name]["iter"]]
        assert [tuple(p) for p in O.weights_from_bytes(data).iter()] == want, name
        counts = np.bincount(np.frombuffer(data, np.uint8), minlength=256)
        assert list(H.ByteWeights.from_array(counts)) == want, name
    c = q["threaded_double_count"]
    data = bytes.fromhex(c["input_hex"])
    assert O.weights_from_bytes(data).w[0] == c["w0_plain"]
    assert list(O.weights_threaded(data, c["thread_num"]).w) == c["weights_threaded"]
    assert c["weights_threaded"][0] == c["w0_threaded"] != c["w0_plain"]
    # the product's merge (huff_weights_add) over the CLI's 12 rations
    # (utils.rs:6-28: n / T each, the last takes the remainder; merged into
    # the last ration's weights in order, weights.rs:300-316)
    T, n = c["thread_num"], len(data)
    per = n // T if n >= T else n
    rations = [data[k * per:(k + 1) * per] for k in range(T - 1)] + [data[(T - 1) * per:]] if n >= T else [data]
    ws = [H.ByteWeights.from_array(np.bincount(np.frombuffer(r, np.uint8), minlength=256)) for r in rations]
    acc = ws[-1]
    for w in ws[:-1]:
        acc += w
    assert [int(x) for x in acc.as_array()] == c["weights_threaded"]


def test_cli_oracle(O, golden):
    _, derived = golden
    inputs = cli_inputs(O)
    for c in derived["cli"]:
        d = inputs[c["input_kind"]]
        assert sha(d) == c["input_sha256"] and len(d) == c["n"]
        hff = O.cli_compress(d, c["block_size"])
        assert sha(hff) == c["hff_sha256"] and len(hff) == c["hff_len"], c
        if "decompress_error" in c:
            with pytest.raises(O.OracleError) as e:
                O.cli_decompress(hff, c["block_size"])
            assert e.value.code == c["decompress_error"]
        else:
            rt = O.cli_decompress(hff, c["block_size"])
            assert sha(rt) == c["decoded_sha256"] and len(rt) == c["decoded_len"]
            assert (rt == d) == c["roundtrip_ok"]


def test_synthetic_oracle(O, golden):
    _, derived = golden
    for c in derived["synthetic"]:
        d = synthetic_input(O, c["kind"], c["n"])
        assert sha(d) == c["input_sha256"], c["kind"]
        t = O.Tree.from_weights(O.weights_from_bytes(d))
        assert t.as_bin() == c["tree_bits"]
        code, ln = t.code_table()
        comp, bits = O.fast_encode(d, code, ln, threads=4)
        assert sha(comp) == c["comp_sha256"] and bits == c["bits"] and int(ln.max()) == c["maxlen"]
        assert (8 - bits % 8) % 8 == c["padding"]


# ---- GPU: the product path -----------------------------------------------------

@pytest.mark.gpu
def test_quirks_gpu(H, O, ctx, golden):
    """the quirk inputs through the GPU histogram (plain and threaded), the
    host tree and huff_compress_with_tree, equal to the oracle's bytes"""
    _, derived = golden
    q = derived["quirks"]
    for name in ("iter_dup", "iter_no_dup"):
        data = bytes.fromhex(q[name]["input_hex"])
        w = H.ByteWeights.from_bytes(data, ctx)
        assert [tuple(p) for p in w] == [tuple(p) for p in q[name]["iter"]]
        t = H.HuffTree.from_weights(w)
        cd = H.compress_with_tree(data, t, ctx)
        ot = O.Tree.from_weights(O.weights_from_bytes(data))
        comp, pad = O.compress_with_tree(data, ot)
        assert cd.to_bytes() == O.to_bytes(comp, pad, ot)
        assert H.decompress(H.CompressData.try_from_bytes(cd.to_bytes()), ctx) == data
    c = q["threaded_double_count"]
    data = bytes.fromhex(c["input_hex"])
    w = H.ByteWeights.threaded_from_bytes(data, c["thread_num"], ctx)
    assert [int(x) for x in w.as_array()] == c["weights_threaded"]
    for name in ("fibonacci30", "ties"):  # streams over those trees
        wts = np.array(q[name]["weights"], np.uint64)
        letters = np.repeat(np.arange(256, dtype=np.uint8), np.minimum(wts, 5000).astype(np.int64))
        data = np.random.default_rng(3).permutation(letters).tobytes()
        t = H.HuffTree.from_weights(H.ByteWeights.from_array(wts))
        cd = H.compress_with_tree(data, t, ctx)
        ot = O.Tree.from_weights(O.weights_from_array(wts))
        comp, pad = O.compress_with_tree(data, ot)
        assert cd.comp_bytes() == comp and cd.padding_bits() == pad, name
        assert H.decompress(H.CompressData.try_from_bytes(cd.to_bytes()), ctx) == data, name


@pytest.mark.gpu
def test_cli_gpu(H, O, ctx, golden):
    """huff_file_compress / huff_file_decompress produce the frozen .hff bytes"""
    _, derived = golden
    inputs = cli_inputs(O)
    with tempfile.TemporaryDirectory() as d:
        for c in derived["cli"]:
            p = os.path.join(d, f"in{c['input_kind']}")
            with open(p, "wb") as f:
                f.write(inputs[c["input_kind"]])
            H.read_compress_write(p, p + ".hff", c["block_size"], ctx)
            hff = open(p + ".hff", "rb").read()
            assert sha(hff) == c["hff_sha256"] and len(hff) == c["hff_len"], c
            if "decompress_error" in c:
                with pytest.raises(H.CliError) as e:
                    H.read_decompress_write(p + ".hff", p + ".out", c["block_size"], ctx)
                assert e.value.code == c["decompress_error"]
                continue
            H.read_decompress_write(p + ".hff", p + ".out", c["block_size"], ctx)
            rt = open(p + ".out", "rb").read()
            assert sha(rt) == c["decoded_sha256"] and len(rt) == c["decoded_len"], c


@pytest.mark.gpu
def test_synthetic_gpu(H, O, ctx, golden):
    """the three 1 MiB inputs generated ON THE DEVICE, compressed by the device
    job: input, tree and stream hashes equal the frozen ones; the stream
    decodes back through the restart index and index-free"""
    import torch
    from huff_coding import device as D

    _, derived = golden
    for c in derived["synthetic"]:
        n = c["n"]
        x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        seed = {"uniform": 0x5EED0001, "zipf": 0x5EED0002, "text": 0x5EED0005}[c["kind"]]
        D.generate(ctx, c["kind"], seed, x.data_ptr(), n, cdf=D.zipf_cdf(1.2) if c["kind"] == "zipf" else None)
        torch.cuda.synchronize()
        assert sha(x[:n].cpu().numpy()) == c["input_sha256"], c["kind"]
        job = H.EncodeJob(ctx, x.data_ptr(), n)
        out = torch.zeros(n + 128, dtype=torch.uint8, device="cuda")
        tree, bits = job.compress(out.data_ptr(), out.numel())
        assert tree.as_bin() == c["tree_bits"] and bits == c["bits"], c["kind"]
        nbytes = (bits + 7) // 8
        torch.cuda.synchronize()
        assert sha(out[:nbytes].cpu().numpy()) == c["comp_sha256"], c["kind"]
        dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        job.decode(tree, out.data_ptr(), dec.data_ptr())
        torch.cuda.synchronize()
        assert torch.equal(dec[:n], x[:n])
        dec.fill_(0)
        got = D.decompress_dev(ctx, tree, out.data_ptr(), nbytes, c["padding"], dec.data_ptr(), n + 64)
        torch.cuda.synchronize()
        assert got == n and torch.equal(dec[:n], x[:n])
