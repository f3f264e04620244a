#!/usr/bin/env python3
"""Run huff_dev_calibrate on 1 GiB (both read shapes and both copy shapes,
5 iterations each) so a kernel trace gives each shape's duration:
    rocprofv3 --kernel-trace --stats -- python3 tools/calib_shapes.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "huff-encoding_amd"))
import torch  # noqa: E402

import huff_coding as H  # noqa: E402
from huff_coding import device as D  # noqa: E402

torch.cuda.set_device(0)
ctx = H.Context(0)
n = 1 << 30
a = torch.empty(n, dtype=torch.uint8, device="cuda")
b = torch.empty(n, dtype=torch.uint8, device="cuda")
a.random_(0, 256)
torch.cuda.synchronize()
print(D.calibrate(ctx, a.data_ptr(), b.data_ptr(), n, 5), flush=True)
