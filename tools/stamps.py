"""Per-phase cycle stamps of the SC streaming kernel (diagnostic build with -DNPD_SCF_STAMPS, loaded via
NPD_LIB): python tools/stamps.py"""
import sys

import torch

sys.path.insert(0, ".")
from neural_polar_decoder_amd import reference_polar_code  # noqa: E402

code = reference_polar_code(64, 32)
B = 1 << 20
ys = [code.mc_generate(B, s, 1234, i, 0, want_msg=False)[2] for i, s in enumerate([0., 1., 2., 3., 4.])]
hat = torch.empty(B, 32, device="cuda")
for it in range(3):
    c = torch.zeros(8, dtype=torch.int64, device="cuda")
    for i, y in enumerate(ys):
        code.sc_decode_mc(y, float(i), 1234, 0, c, msg_hat=hat)
    torch.cuda.synchronize()
c = c.cpu().tolist()
tiles = 5 * B // 64
names = ["philox", "wait+transpose+prefetch", "stores+row reads", "decode", "count"]
print("waves", c[7], " per wave-tile cycles: " + "  ".join(f"{n} {v / tiles:.0f}" for n, v in zip(names, c[2:7])))
