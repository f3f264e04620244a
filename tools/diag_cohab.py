#!/usr/bin/env python3
"""Wrong-letter reproducer with foreign co-resident waves: decode with the
library selected by HUFF_LIB_AB (the HUFF_DEC_EARLY_LOADS build) padded to one
decoder workgroup per CU (HUFF_DEC_LDS_EXTRA), while another kernel keeps the
rest of every CU busy on a side stream. Reports wrong bytes per decode for
each kind of side load."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "huff-encoding_amd"))
import torch  # noqa: E402

import huff_coding as H  # noqa: E402
from huff_coding import device as D  # noqa: E402


def main():
    ctx = H.Context(0)
    n = 1 << 24
    os.environ["HUFF_DISABLE_FIXED8"] = "1"
    x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    D.generate(ctx, "zipf", 0x5EED0002, x.data_ptr(), n, cdf=D.zipf_cdf(1.2))
    job = H.EncodeJob(ctx, x.data_ptr(), n)
    tree = H.HuffTree.from_weights(H.ByteWeights.from_array(job.hist()))
    bits = job.bits(tree)
    out = torch.zeros((bits + 7) // 8 + 64, dtype=torch.uint8, device="cuda")
    job.pack(tree, out.data_ptr(), out.numel())
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    big = torch.rand(1 << 28, device="cuda")
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    loads = {
        "none": lambda: None,
        "elementwise": lambda: [big.mul_(1.0000001) for _ in range(40)],
        "matmul": lambda: [a @ a for _ in range(40)],
        "shift64": lambda: [big.view(torch.int64).bitwise_right_shift_(1) for _ in range(40)],
    }
    for name, fn in loads.items():
        wrong, tasks = [], []
        for rep in range(int(os.environ.get("DIAG_REPS", "4"))):
            dec = torch.zeros(n + 64, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            with torch.cuda.stream(side):
                fn()
            for _ in range(5):  # several decodes while the side load runs
                job.decode(tree, out.data_ptr(), dec.data_ptr())
            torch.cuda.synchronize()
            bad = (dec[:n] != x[:n]).nonzero().flatten()
            wrong.append(int(bad.numel()))
            tasks.append(int(torch.unique(bad // 4096).numel()) if bad.numel() else 0)
        print(json.dumps({"side_load": name, "lds_extra": os.environ.get("HUFF_DEC_LDS_EXTRA"),
                          "wrong_bytes_last_of_5": wrong, "wrong_tasks": tasks}), flush=True)


main()
