"""Data-generation throughput (npd_mc_generate, N=64, 2^20 codewords): python tools/gen_bench.py"""
import sys

import torch

sys.path.insert(0, ".")
from neural_polar_decoder_amd import reference_polar_code  # noqa: E402

code = reference_polar_code(64, 32)
B = 1 << 20
y = torch.empty(B, 64, device="cuda")
for want_msg in (False, True):
    for _ in range(2):
        code.mc_generate(B, 2.0, 1, 0, 0, want_msg=want_msg, out=y)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        code.mc_generate(B, 2.0, 1, 0, 0, want_msg=want_msg, out=y)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    print(f"mc_generate want_msg={want_msg}: {ms * 1e3:.1f} us per 2^20 codewords ({B / ms / 1e6:.2f} Gcw/s)")
