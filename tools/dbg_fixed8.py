"""Debug: fixed-8 byte-map path vs the general kernels at a given size."""
import os, sys, torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "huff-encoding_amd"))
import huff_coding as H
from huff_coding import device as D

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
ctx = H.default_context()
x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
D.generate(ctx, "uniform", 0x5EED0001, x.data_ptr(), n)
job = H.EncodeJob(ctx, x.data_ptr(), n)
w = job.hist()
tree = H.HuffTree.from_weights(H.ByteWeights.from_array(w))
bits = job.bits(tree)
outs, decs = {}, {}
for mode in ("0", "1"):
    os.environ["HUFF_DISABLE_FIXED8"] = mode
    o = torch.zeros(bits // 8 + 64, dtype=torch.uint8, device="cuda")
    job.pack(tree, o.data_ptr(), o.numel())
    d = torch.zeros(n + 64, dtype=torch.uint8, device="cuda")
    job.decode(tree, o.data_ptr(), d.data_ptr())
    torch.cuda.synchronize()
    outs[mode], decs[mode] = o, d
    bad = (d[:n] != x[:n]).nonzero().flatten()
    print("mode", mode, "decode mismatches", bad.numel(), bad[:8].tolist(), flush=True)
bad = (outs["0"] != outs["1"]).nonzero().flatten()
print("pack fast vs general mismatches", bad.numel(), bad[:8].tolist())
