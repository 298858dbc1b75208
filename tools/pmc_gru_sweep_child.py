"""Child program for PMC passes on the headline GRU kernel (rocprofv3 --pmc ... -- python3 tools/pmc_gru_sweep_child.py):
the trained Polar(64,32) net on fp16x3, npd_gru_decode_count_sweep over 5 SNR points x 2^18 words, 3 launches."""
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from neural_polar_decoder_amd import reference_polar_code  # noqa: E402

B = 1 << 18
code = reference_polar_code(64, 32)
y = torch.empty(5, B, 64, device="cuda")
msg = None
for si, s in enumerate((0.0, 1.0, 2.0, 3.0, 4.0)):
    m, _, _ = code.mc_generate(B, s, 1234, si, 0, want_msg=msg is None, out=y[si])
    msg = m if msg is None else msg
net, dec, _, _ = bench.crisp_model(code, torch.device("cuda", 0), precision="fp16x3")
c = torch.zeros(5, 2, dtype=torch.int64, device="cuda")
for _ in range(3):
    dec.decode_count_sweep(net, y, msg, c)
torch.cuda.synchronize()
